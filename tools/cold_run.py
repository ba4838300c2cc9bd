"""The cold-Infinity-Cache leg of bench.py on its own, as a rocprofv3 target (a lab tool).

Each of N steps first writes a 512 MiB buffer (evicting the 256 MiB MALL), then runs one prune of
the configuration (default cfg2: the ResNet-18 conv state_dict, bior3.3 L5, p50) -- so the kernel
trace and the PMC passes of the prune kernel see HBM, not cache hits.
Usage: python tools/cold_run.py [--config cfg2|cfg3] [--steps N]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2", choices=["cfg2", "cfg3"])
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--flush", default="write", choices=["write", "read", "clean"],
                    help="write: a 512 MiB write before each prune (the Infinity Cache then holds dirty "
                         "lines of another buffer); read: a 512 MiB read (clean lines of another buffer); "
                         "clean: the write, then the read of a third buffer")
    a = ap.parse_args()
    import torch
    from wavelettransforms_amd import engine
    from wavelettransforms_amd import workloads as W
    dev = torch.device("cuda", 0)
    if a.config == "cfg2":
        wavelet, level, pct, ts = "bior3.3", 5, 50.0, W.resnet18_tensors(0)
    else:
        wavelet, level, pct, ts = "rbio2.2", 3, 50.0, W.mlp_tensors(3)
    xs = [engine.synth(s, seed, tid, e, device=dev) for (_, s, seed, tid, e) in ts]
    outs = [torch.empty_like(x) for x in xs]
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    flush_r = torch.ones(128 << 20, dtype=torch.float32, device=dev)
    for _ in range(3):
        engine.launch(xs, wavelet, level, pct, outs=outs, carry_level=False)
    torch.cuda.synchronize()
    for _ in range(a.steps):
        if a.flush in ("write", "clean"):
            flush.fill_(1)
        if a.flush in ("read", "clean"):
            flush_r.sum()
        engine.launch(xs, wavelet, level, pct, outs=outs, carry_level=False)
    torch.cuda.synchronize()
    print("cold leg done: %d steps of %s, flush %s" % (a.steps, a.config, a.flush))


if __name__ == "__main__":
    main()
