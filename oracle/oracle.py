"""ctypes front-end of the C oracle (oracle/wtprune_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker / CPU baseline, never by the product package
(wavelettransforms_amd), which fails loudly when its HIP library is missing.

Every function restates a reference call site; see the C file header for the file:line map.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

ERRORS = {
    -1: (ValueError, "Unknown wavelet name"),
    -2: (ValueError, "Level value is too low . Minimum level is 0."),
    -3: (ValueError, "Percentiles must be in the range [0, 100]"),
    -4: (IndexError, "index -1 is out of bounds for axis 0 with size 0"),
    -5: (IndexError, "too many indices for array"),
    -6: (MemoryError, "oracle allocation failed"),
}


class OrResult(ctypes.Structure):
    _fields_ = [
        ("numel", ctypes.c_int64),
        ("zero_count", ctypes.c_int64),
        ("nonzero", ctypes.c_int64),
        ("coeff_numel", ctypes.c_int64),
        ("packed_rows", ctypes.c_int64),
        ("packed_cols", ctypes.c_int64),
        ("thr64", ctypes.c_double),
        ("thr32", ctypes.c_float),
        ("max_abs", ctypes.c_float),
        ("eff_level", ctypes.c_int32),
        ("status", ctypes.c_int32),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER
        f32p, i64p = P(ctypes.c_float), P(ctypes.c_int64)
        L.or_wavelet_id.argtypes = [ctypes.c_char_p]
        L.or_wavelet_name.restype = ctypes.c_char_p
        L.or_dwt_max_level.argtypes = [ctypes.c_int64, ctypes.c_int]
        L.or_dwt1.argtypes = [f32p, ctypes.c_int64, ctypes.c_int, f32p, f32p]
        L.or_idwt1.argtypes = [f32p, f32p, ctypes.c_int64, ctypes.c_int, f32p]
        L.or_filters.argtypes = [ctypes.c_int, f32p]
        L.or_packed_shape.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int, i64p, i64p]
        L.or_wavedec2_packed.argtypes = [f32p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.c_int, ctypes.c_int, f32p]
        L.or_waverec2_packed.argtypes = [f32p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, f32p]
        L.or_percentile_abs.argtypes = [f32p, ctypes.c_int64, ctypes.c_double,
                                        P(ctypes.c_double), f32p]
        L.or_percentile_threshold.argtypes = [f32p, ctypes.c_int64, ctypes.c_double, f32p,
                                              P(ctypes.c_double), f32p]
        L.or_prune_tensor.argtypes = [f32p, f32p, ctypes.c_int, i64p, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_double, P(OrResult), f32p]
        L.or_prune_tensor_flat.argtypes = L.or_prune_tensor.argtypes
        L.or_prune_batch.argtypes = [ctypes.c_int, P(f32p), P(f32p), P(ctypes.c_int), i64p,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_double, P(OrResult),
                                     ctypes.c_int]
        L.or_synth_fill.argtypes = [f32p, ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint32,
                                    ctypes.c_int]
        L.or_min_prune.argtypes = [f32p, f32p, ctypes.c_int64, ctypes.c_double, i64p, f32p]
        L.or_random_prune.argtypes = [f32p, f32p, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64,
                                      ctypes.c_uint32, i64p]
        _lib = L
    return _lib


def _f32p(a):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _check(rc, wavelet=None):
    if rc != 0:
        exc, msg = ERRORS.get(rc, (RuntimeError, "oracle error %d" % rc))
        if rc == -1 and wavelet is not None:
            msg = ("Unknown wavelet name '%s', check wavelist() for the list of available "
                   "builtin wavelets." % wavelet)
        raise exc(msg)


def wavelet_id(name):
    return lib().or_wavelet_id(name.encode())


def dec_len(name):
    return lib().or_dec_len(wavelet_id(name))


def filters(name):
    wid = wavelet_id(name)
    F = lib().or_dec_len(wid)
    out = np.empty(4 * F, np.float32)
    lib().or_filters(wid, _f32p(out))
    return out.reshape(4, F)


def dwt_max_level(n, F):
    return lib().or_dwt_max_level(int(n), int(F))


def dwt1(x, wavelet):
    x = np.ascontiguousarray(x, np.float32)
    N = x.size
    O = (N + 1) // 2
    a, d = np.empty(O, np.float32), np.empty(O, np.float32)
    lib().or_dwt1(_f32p(x), N, wavelet_id(wavelet), _f32p(a), _f32p(d))
    return a, d


def idwt1(a, d, wavelet):
    a = np.ascontiguousarray(a, np.float32)
    d = np.ascontiguousarray(d, np.float32)
    out = np.empty(2 * a.size, np.float32)
    lib().or_idwt1(_f32p(a), _f32p(d), a.size, wavelet_id(wavelet), _f32p(out))
    return out


def packed_shape(H, W, L):
    pr, pc = ctypes.c_int64(), ctypes.c_int64()
    lib().or_packed_shape(H, W, L, ctypes.byref(pr), ctypes.byref(pc))
    return pr.value, pc.value


def wavedec2_packed(x, wavelet, level):
    """pywt.coeffs_to_array(pywt.wavedec2(x, wavelet, level, 'periodization', (-2,-1)), axes=(-2,-1))[0]"""
    x = np.ascontiguousarray(x, np.float32)
    H, W = x.shape[-2:]
    B = int(np.prod(x.shape[:-2]))
    PR, PC = packed_shape(H, W, level)
    P = np.empty(x.shape[:-2] + (PR, PC), np.float32)
    _check(lib().or_wavedec2_packed(_f32p(x), B, H, W, wavelet_id(wavelet), level, _f32p(P)))
    return P


def waverec2_packed(P, shape, wavelet, level, thr32=None):
    P = np.ascontiguousarray(P, np.float32)
    H, W = shape[-2:]
    B = int(np.prod(shape[:-2]))
    out = np.empty(tuple(shape), np.float32)
    _check(lib().or_waverec2_packed(_f32p(P), B, H, W, wavelet_id(wavelet), level,
                                    0 if thr32 is None else 1,
                                    0.0 if thr32 is None else float(thr32), _f32p(out)))
    return out


def percentile_abs(arr, pct):
    arr = np.ascontiguousarray(arr, np.float32).ravel()
    thr, mx = ctypes.c_double(), ctypes.c_float()
    _check(lib().or_percentile_abs(_f32p(arr), arr.size, float(pct), ctypes.byref(thr), ctypes.byref(mx)))
    return thr.value, mx.value


def percentile_based_thresholding(arr, pct):
    arr = np.ascontiguousarray(arr, np.float32)
    out = np.empty_like(arr)
    thr, mx = ctypes.c_double(), ctypes.c_float()
    _check(lib().or_percentile_threshold(_f32p(arr.ravel()), arr.size, float(pct),
                                         _f32p(out.reshape(-1)), ctypes.byref(thr), ctypes.byref(mx)))
    return out, thr.value


def prune_tensor(x, wavelet, level, pct, want_coeffs=False):
    """One tensor through dwt_pruning.py:53-89; returns (out, result dict[, packed coeffs])."""
    x = np.require(np.asarray(x, np.float32), requirements="C")  # keeps 0-d arrays 0-d
    out = np.empty_like(x)
    shape = (ctypes.c_int64 * max(1, x.ndim))(*x.shape)
    res = OrResult()
    wid = wavelet_id(wavelet)
    coeffs = None
    cptr = None
    if want_coeffs:
        if x.ndim >= 2:
            H, W = x.shape[-2:]
            maxL = dwt_max_level(min(H, W), lib().or_dec_len(wid)) if wid >= 0 else 0
            PR, PC = packed_shape(H, W, max(0, min(level, maxL)))
            coeffs = np.empty(x.shape[:-2] + (PR, PC), np.float32)
        else:
            coeffs = np.empty(x.shape, np.float32)
        cptr = _f32p(coeffs.reshape(-1))
    rc = lib().or_prune_tensor(_f32p(x.reshape(-1)) if x.size else None, _f32p(out.reshape(-1)) if x.size else None,
                               x.ndim, shape, wid, int(level), float(pct), ctypes.byref(res), cptr)
    _check(rc, wavelet)
    d = res.as_dict()
    return (out, d, coeffs) if want_coeffs else (out, d)


def prune_tensor_flat(x, wavelet, level, pct, want_coeffs=False):
    """The 1-D flattened mode (WTP_FLATTEN, include/wtprune.h): ndim >= 2 tensors through
    pywt.wavedec / coeffs_to_array / percentile threshold / waverec of w.ravel(); ndim < 2 as
    prune_tensor.  Returns (out, result dict[, packed coeffs])."""
    x = np.require(np.asarray(x, np.float32), requirements="C")
    if x.ndim < 2:
        return prune_tensor(x, wavelet, level, pct, want_coeffs)
    out = np.empty_like(x)
    shape = (ctypes.c_int64 * x.ndim)(*x.shape)
    res = OrResult()
    wid = wavelet_id(wavelet)
    coeffs, cptr = None, None
    if want_coeffs:
        n = x.size
        L = max(0, min(level, dwt_max_level(n, lib().or_dec_len(wid)))) if wid >= 0 else 0
        lens = [n]
        for _ in range(L):
            lens.append((lens[-1] + 1) // 2)
        coeffs = np.empty(lens[-1] + sum(lens[1:]), np.float32)
        cptr = _f32p(coeffs)
    rc = lib().or_prune_tensor_flat(_f32p(x.reshape(-1)) if x.size else None,
                                    _f32p(out.reshape(-1)) if x.size else None, x.ndim, shape, wid, int(level),
                                    float(pct), ctypes.byref(res), cptr)
    _check(rc, wavelet)
    d = res.as_dict()
    return (out, d, coeffs) if want_coeffs else (out, d)


def prune_batch(tensors, wavelet, level, pct, nthreads=1):
    """All tensors as one CPU-baseline step (threaded over tensors when nthreads > 1)."""
    n = len(tensors)
    xs = [np.ascontiguousarray(t, np.float32) for t in tensors]
    outs = [np.empty_like(t) for t in xs]
    f32pp = ctypes.POINTER(ctypes.c_float) * n
    ins_p = f32pp(*[_f32p(t.reshape(-1)) for t in xs])
    outs_p = f32pp(*[_f32p(t.reshape(-1)) for t in outs])
    ndims = (ctypes.c_int * n)(*[t.ndim for t in xs])
    shapes = (ctypes.c_int64 * (8 * n))()
    for i, t in enumerate(xs):
        for j, s in enumerate(t.shape):
            shapes[8 * i + j] = s
    res = (OrResult * n)()
    rc = lib().or_prune_batch(n, ins_p, outs_p, ndims, shapes, wavelet_id(wavelet), int(level),
                              float(pct), res, int(nthreads))
    _check(rc, wavelet)
    return outs, [r.as_dict() for r in res]


def min_prune(x, fraction):
    """percentage_min_pruning (min_weight_pruning.py:66-74), ties lowest index first.
    Returns (out, zero_count, t) with t the k-th smallest |x| (0.0 when k = 0)."""
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty_like(x)
    z = ctypes.c_int64()
    t = ctypes.c_float()
    rc = lib().or_min_prune(_f32p(x.reshape(-1)) if x.size else None, _f32p(out.reshape(-1)) if x.size else None,
                            int(x.size), float(fraction), ctypes.byref(z), ctypes.byref(t))
    if rc == -7:
        raise RuntimeError("selected index k out of range")
    _check(rc)
    return out, z.value, t.value


def random_prune(x, k, seed, tensor_id):
    """random_pruning's per-layer step (random_pruning.py:53-56) with the keyed permutation of
    csrc/wt_perm.h in place of torch.randperm; returns (out, zero_count)."""
    x = np.require(np.asarray(x, np.float32), requirements="C")
    out = np.empty_like(x)
    z = ctypes.c_int64()
    rc = lib().or_random_prune(_f32p(x.reshape(-1)) if x.size else None, _f32p(out.reshape(-1)) if x.size else None,
                               x.size, int(k), int(seed), int(tensor_id), ctypes.byref(z))
    _check(rc)
    return out, z.value


def synth(shape, seed, tensor_id, e):
    n = int(np.prod(shape))
    out = np.empty(n, np.float32)
    lib().or_synth_fill(_f32p(out), n, seed, tensor_id, int(e))
    return out.reshape(shape)


def max_threads():
    return lib().or_omp_max_threads()
