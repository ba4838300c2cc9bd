"""Phase timeline of k_small (the one-launch small path) on cfg3 -- a lab tool, not a test.

Build the probe library on the CPU side first:  python tools/probe_small.py --build
then on the GPU box:                           python tools/probe_small.py
It loads tools/mb/libwtprune_probe.so (k_small compiled with -DWTP_SM_PROBE: workgroup b writes
s_memrealtime at phase i to stamps[2 + 16 b + i]), checks the result against the oracle and
prints, per phase, the median over workgroups and runs of (stamp - launch start) in microseconds.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PROBE_LIB = os.path.join(ROOT, "tools", "mb", "libwtprune_probe.so")
PHASES = [(6, "entry"), (0, "windows"), (1, "L0 loaded"), (10, "arrived 0"), (11, "barrier 0"),
          (2, "bin located"), (3, "slot written"), (4, "arrived 1"), (5, "barrier 1"), (7, "windows in LDS"),
          (8, "slots in LDS"), (9, "slot headers"), (12, "pass A"), (13, "ranks"), (14, "I start"),
          (15, "stores drained"), (16, "F1 axis-2"), (17, "F1 axis-1"), (18, "F2 axis-2"), (19, "F2 axis-1"),
          (20, "F3 axis-2"), (21, "F3 axis-1"), (22, "I3 axis-1"), (24, "I2 axis-1"), (26, "I1 axis-1")]


def build():
    from wavelettransforms_amd import build as B
    csrc = os.path.join(ROOT, "wavelettransforms_amd", "csrc")
    extra = [a for a in sys.argv[2:] if a.startswith("-D")]
    out = os.environ.get("PROBE_OUT", PROBE_LIB)
    cmd = [B.HIPCC] + B.FLAGS + ["-DWTP_SM_PROBE=1"] + extra + ["-o", out] + [os.path.join(csrc, s) for s in B.SOURCES]
    subprocess.check_call(cmd)


def main():
    os.environ["WTP_LIB_PATH"] = os.environ.get("PROBE_OUT", PROBE_LIB)
    import numpy as np
    import torch
    from oracle import oracle as O
    from wavelettransforms_amd import _native as N
    from wavelettransforms_amd import engine as eng
    from wavelettransforms_amd import workloads as W
    cfg = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "cfg3"
    spec = W.CONFIGS[cfg]
    ts = spec["tensors"]()
    xs = [eng.synth(s, seed, tid, e) for _, s, seed, tid, e in ts]
    stamps = torch.zeros(2 + 32 * 256, dtype=torch.int64, device="cuda")
    L = N.lib()
    runs = []
    warm = os.environ.get("PROBE_WARM")  # stamp the second of two back-to-back launches
    wouts = [torch.empty_like(x) for x in xs]
    dummy = torch.zeros_like(stamps)
    for it in range(60):
        stamps.zero_()
        stamps[0] = (1 << 62)
        if warm:
            dummy.zero_()
            dummy[0] = (1 << 62)
            L.wtp_set_kernel_stamps(dummy.data_ptr())
            eng.launch(xs, spec["wavelet"], spec["level"], spec["pct"], outs=wouts, carry_level=False)
        L.wtp_set_kernel_stamps(stamps.data_ptr())
        outs, resd = eng.launch(xs, spec["wavelet"], spec["level"], spec["pct"], outs=wouts, carry_level=False)
        torch.cuda.synchronize()
        L.wtp_set_kernel_stamps(None)
        s = stamps.cpu().numpy()
        t0 = s[0]
        blk = s[2:].reshape(256, 32)
        used = blk[:, 0] > 0
        if it >= 10:
            runs.append(((blk[used, :32] - t0) * 0.01, (s[1] - t0) * 0.01))
    res = eng.decode(resd, len(xs))
    for (name, s, seed, tid, e), o, r in zip(ts, outs, res):
        ref, rr = O.prune_tensor(W.synth_numpy(s, seed, tid, e), spec["wavelet"], spec["level"], spec["pct"])
        if not os.environ.get("PROBE_NOCHECK"):
            assert np.array_equal(o.cpu().numpy(), ref), name
    allb = np.concatenate([r[0] for r in runs])
    print("workgroups per launch:", runs[0][0].shape[0], " span (us) median %.2f" % np.median([r[1] for r in runs]))
    # the slowest workgroups at the first barrier: which tiles are they
    last = runs[-1][0]
    order = np.argsort(-last[:, 10])[:6]
    print("slowest arrivals (workgroup: entry, windows, L0, arrived):",
          ", ".join("%d: %.1f %.1f %.1f %.1f" % (w, last[w, 6], last[w, 0], last[w, 1], last[w, 10]) for w in order))
    for i, ph in PHASES:
        col = allb[:, i]
        print("%-16s median %6.2f  p10 %6.2f  p90 %6.2f  max %6.2f" % (ph, np.median(col), np.percentile(col, 10),
                                                                     np.percentile(col, 90), col.max()))


if __name__ == "__main__":
    if "--build" in sys.argv:
        build()
    else:
        main()
