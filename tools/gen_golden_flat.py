"""Golden fixtures for the 1-D flattened mode (WTP_FLATTEN, include/wtprune.h).

Run under the oracle interpreter (PyWavelets 1.1.1 + NumPy 1.26.4):
    /opt/conda/bin/python3.9 tools/gen_golden_flat.py

The reference transform is 2-D (ResNet/dwt_pruning.py:67-77); SURVEY.md 8(f) rank 3 asks for
the north star's "1-D wavedec/waverec over flattened conv weight tensors" as an extension.  Its
semantics are the reference's per-tensor sequence with the 2-D calls swapped for their 1-D
PyWavelets counterparts on w.ravel():
  level = min(level, pywt.dwt_max_level(numel, dec_len))   (the clamp of :64-65, carried)
  pywt.wavedec(flat, wavelet, mode='periodization', level)  (pywt/_multilevel.py wavedec)
  pywt.coeffs_to_array -> percentile_based_thresholding (:25-32) -> pywt.array_to_coeffs
  pywt.waverec(..., mode='periodization')[:numel].reshape(shape)
ndim < 2 tensors keep the plain-percentile branch (:58-62).  Inputs come from the shared
deterministic generator (wavelettransforms_amd/workloads.py), so only outputs are stored.
"""
import hashlib
import importlib.util
import json
import os
import warnings

import numpy as np

warnings.filterwarnings("ignore")
import pywt  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden")
_spec = importlib.util.spec_from_file_location(
    "workloads", os.path.join(ROOT, "wavelettransforms_amd", "workloads.py"))
W = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(W)

SMALL = 20000  # store full outputs up to this many elements


def canon_hash(a):
    a = np.array(a, dtype=np.float32, copy=True).reshape(-1)
    a[a == 0] = 0
    return hashlib.sha256(a.tobytes()).hexdigest()


def mask_hash(mask):
    return hashlib.sha256(np.packbits(np.asarray(mask, bool).reshape(-1)).tobytes()).hexdigest()


def flat_restated(x, wavelet, level, pct):
    """One tensor of the flattened mode; returns (out, record)."""
    rec = {}
    if x.ndim < 2:
        thr = np.percentile(np.abs(x), pct)
        out = np.where(np.abs(x) < thr, 0, x)
        rec.update(eff_level=level, coeff_numel=int(x.size), thr64=float(thr), mask_count=int((np.abs(x) < thr).sum()))
    else:
        w = pywt.Wavelet(wavelet)
        flat = x.reshape(-1)
        L = min(level, pywt.dwt_max_level(flat.size, w.dec_len))
        coeffs = pywt.wavedec(flat, w, mode="periodization", level=L)
        arr, sl = pywt.coeffs_to_array(coeffs)
        thr = np.percentile(np.abs(arr), pct)
        mask = np.abs(arr) < thr  # legacy value-based casting: float32 compare
        pruned = np.where(mask, 0, arr)
        c2 = pywt.array_to_coeffs(pruned, sl, output_format="wavedec")
        y = pywt.waverec(c2, w, mode="periodization")
        out = np.asarray(y[:flat.size], dtype=np.float32).reshape(x.shape)
        rec.update(eff_level=int(L), coeff_numel=int(arr.size), thr64=float(thr), coeff_hash=canon_hash(arr),
                   mask_count=int(mask.sum()), mask_hash=mask_hash(mask))
    out = np.asarray(out, dtype=np.float32)
    rec.update(thr32_bits=int(np.array(rec["thr64"], np.float32).view(np.uint32)),
               zero_count=int((out == 0).sum()), out_hash=canon_hash(out))
    return out, rec


def main():
    shapes = [(13, 1), (7, 11), (2, 3, 5), (10, 128), (64, 3, 7, 7), (64, 64, 3, 3), (128, 784), (1, 1, 1, 1),
              (3, 1, 2, 2), (1001,)]
    wavelets = ["haar", "db2", "db8", "bior3.3", "rbio2.2", "coif2", "sym4"]
    cases, arrays = {}, {}
    for si, shape in enumerate(shapes):
        n = int(np.prod(shape))
        sigma = (2.0 / (shape[0] * (shape[-1] if len(shape) > 1 else 1))) ** 0.5
        e = W.sigma_exponent(sigma)
        for wi, wavelet in enumerate(wavelets):
            for level in (1, 3, 5):
                for pct in (23.599999999999998, 50.0, 90.0):
                    if n > SMALL and (level != 5 or pct != 50.0):
                        continue  # the large shapes: one configuration per wavelet
                    name = "flat_%s_%s_L%d_p%s" % ("x".join(map(str, shape)), wavelet, level, pct)
                    x = W.synth_numpy(shape, 300 + si, wi, e)
                    out, rec = flat_restated(x, wavelet, level, pct)
                    rec.update(shape=list(shape), wavelet=wavelet, level_in=level, pct=pct, synth=[300 + si, wi, e])
                    cases[name] = rec
                    if n <= SMALL:
                        arrays[name + "/out"] = out
    # the list form (multi_resolution_analysis): the clamped level carries over the list
    multi = []
    seq = [(64, 3, 7, 7), (16,), (10, 128), (5, 5), (64, 64, 3, 3)]
    lvl = 9
    for j, shape in enumerate(seq):
        x = W.synth_numpy(shape, 400, j, 27)
        out, rec = flat_restated(x, "db2", lvl, 61.8)
        if len(shape) >= 2:
            lvl = rec["eff_level"]
        rec.update(shape=list(shape), synth=[400, j, 27])
        multi.append(rec)
        arrays["multi/out%d" % j] = out
    manifest = {"generator": "tools/gen_golden_flat.py", "pywt": pywt.__version__, "numpy": np.__version__,
                "cases": cases, "multi_db2_L9_p61.8": multi}
    with open(os.path.join(OUT, "flat_manifest.json"), "w") as fh:
        json.dump(manifest, fh, indent=0, sort_keys=True)
    np.savez_compressed(os.path.join(OUT, "flat_cases.npz"), **arrays)
    print("%d flat cases, %d arrays" % (len(cases), len(arrays)))


if __name__ == "__main__":
    main()
