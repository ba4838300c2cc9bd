"""ctypes binding of libwtprune.so (include/wtprune.h).

The library is the product: there is no CPU fallback.  If it is missing this module raises
at first use, and every public entry point of the package fails loudly.  torch is imported
first so that the library's libamdhip64.so.7 dependency binds to the HIP runtime torch has
already loaded (one HIP runtime per process).
"""
import ctypes
import os

import torch  # noqa: F401  (binds libamdhip64.so.7 before our library is loaded)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("WTP_LIB_PATH") or os.path.join(HERE, "_lib", "libwtprune.so")  # override: A/B lab builds
MAX_DIMS = 8

WTP_OK = 0
WTP_EBADWAVELET = -1
WTP_EBADLEVEL = -2
WTP_EBADPCT = -3
WTP_EEMPTY = -4
WTP_ECROP = -5
WTP_EARG = -6
WTP_EWORKSPACE = -7
WTP_EHIP = -8


class WtpTensor(ctypes.Structure):
    _fields_ = [("in_", ctypes.c_void_p), ("out", ctypes.c_void_p), ("ndim", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("shape", ctypes.c_int64 * MAX_DIMS)]


class WtpResult(ctypes.Structure):
    _fields_ = [("numel", ctypes.c_int64), ("zero_count", ctypes.c_int64), ("coeff_numel", ctypes.c_int64),
                ("thr64", ctypes.c_double), ("thr32_bits", ctypes.c_uint32), ("max_abs_bits", ctypes.c_uint32),
                ("eff_level", ctypes.c_int32), ("path", ctypes.c_int32)]


RESULT_BYTES = ctypes.sizeof(WtpResult)
_lib = None


class NativeLibraryMissing(RuntimeError):
    pass


def lib():
    """Load libwtprune.so; raise NativeLibraryMissing (never fall back) if it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryMissing(
                "wavelettransforms_amd: %s is missing; build it with `python -m wavelettransforms_amd.build` "
                "(the HIP path has no CPU fallback)" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        vp, i64, i32, f64, sz = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double, ctypes.c_size_t
        tp = ctypes.POINTER(WtpTensor)
        sigs = {
            "wtp_abi_version": ([], i32),
            "wtp_wavelet_count": ([], i32),
            "wtp_wavelet_name": ([i32], ctypes.c_char_p),
            "wtp_wavelet_id": ([ctypes.c_char_p], i32),
            "wtp_dec_len": ([i32], i32),
            "wtp_max_level": ([i64, i32], i32),
            "wtp_packed_shape": ([i64, i64, i32, ctypes.POINTER(i64), ctypes.POINTER(i64)], i32),
            "wtp_workspace_size": ([tp, i32, i32, i32], sz),
            "wtp_workspace_init": ([vp, sz, vp], i32),
            "wtp_prune_f32": ([tp, i32, i32, i32, f64, vp, sz, vp, vp], i32),
            "wtp_prune_layers_f32": ([tp, i32, i32, i32, f64, vp, sz, vp, vp], i32),
            "wtp_workspace_size_ex": ([tp, i32, i32, i32, i32], sz),
            "wtp_prune_ex_f32": ([tp, i32, i32, i32, f64, i32, vp, sz, vp, vp], i32),
            "wtp_threshold_f32": ([vp, vp, i64, f64, vp, sz, vp, vp], i32),
            "wtp_dwt_workspace_size": ([i64, i64, i64, i32], sz),
            "wtp_wavedec2_f32": ([vp, vp, i64, i64, i64, i32, i32, vp, sz, vp], i32),
            "wtp_waverec2_f32": ([vp, vp, i64, i64, i64, i32, i32, vp, vp, sz, vp], i32),
            "wtp_synth_f32": ([vp, i64, ctypes.c_uint64, ctypes.c_uint32, i32, vp], i32),
            "wtp_set_stage_events": ([ctypes.POINTER(ctypes.c_void_p), i32], i32),
            "wtp_min_prune_workspace_size": ([tp, i32, f64], sz),
            "wtp_min_prune_f32": ([tp, i32, f64, vp, sz, vp, vp], i32),
            "wtp_random_prune_f32": ([tp, i32, ctypes.POINTER(i64), ctypes.c_uint64, vp, vp], i32),
            "wtp_count_small_f32": ([vp, i64, ctypes.c_float, vp, vp], i32),
            "wtp_set_resident": ([i32], i32),
            "wtp_set_pipeline": ([i32], i32),
            "wtp_set_fused_select": ([i32], i32),
            "wtp_set_interior": ([i32], i32),
            "wtp_resident_capacity": ([], i32),
            "wtp_set_resident_timeout_us": ([ctypes.c_uint], ctypes.c_uint),
            "wtp_set_kernel_stamps": ([vp], i32),
            "wtp_last_error": ([], ctypes.c_char_p),
            "wtp_last_error_tensor": ([], i32),
        }
        missing = {}
        for name, (args, ret) in sigs.items():
            if os.environ.get("WTP_LIB_PATH") and not hasattr(L, name):
                # an A/B lab build of an older revision: entry points added since are absent; a
                # call to one raises an error that names it (not a bare AttributeError)
                missing[name] = _missing_entry(name)
                continue
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = ret
        if L.wtp_abi_version() != 1:
            raise NativeLibraryMissing("libwtprune.so ABI version mismatch")
        _lib = _LabLib(L, missing) if missing else L
    return _lib


def _missing_entry(name):
    def call(*_a, **_k):
        raise NativeLibraryMissing("%s (WTP_LIB_PATH) has no entry point %s: it was built from an older "
                                   "revision" % (LIB_PATH, name))
    return call


class _LabLib:
    """A lab library (WTP_LIB_PATH) with the entry points it lacks replaced by stubs that raise."""

    def __init__(self, L, missing):
        self._L, self._missing = L, missing

    def __getattr__(self, name):
        if name in self._missing:
            return self._missing[name]
        return getattr(self._L, name)


def exported_symbols():
    """Names declared in include/wtprune.h (checked against the .so by the CPU tests)."""
    import re
    hdr = os.path.join(os.path.dirname(HERE), "include", "wtprune.h")
    with open(hdr) as fh:
        src = fh.read()
    return sorted(set(re.findall(r"\b(wtp_[a-z0-9_]+)\s*\(", src)))


def last_error():
    return lib().wtp_last_error().decode(errors="replace")
