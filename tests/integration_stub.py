"""INTEGRATION.md section 2's ctypes binding, verbatim (tests/test_native_abi.py checks that the
document's code block equals this file's body; tests/test_gpu_integration_stub.py runs it on the GPU).
Test infrastructure: the binding a maintainer would paste next to main_pruning.py."""
# --- begin INTEGRATION.md block ---
import ctypes, torch

torch.zeros(1, device="cuda")             # load torch's HIP runtime first (one runtime per process)
lib = ctypes.CDLL("wavelettransforms_amd/_lib/libwtprune.so")

class WtpTensor(ctypes.Structure):        # wtp_tensor
    _fields_ = [("in_", ctypes.c_void_p), ("out", ctypes.c_void_p), ("ndim", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("shape", ctypes.c_int64 * 8)]

class WtpResult(ctypes.Structure):        # wtp_result
    _fields_ = [("numel", ctypes.c_int64), ("zero_count", ctypes.c_int64), ("coeff_numel", ctypes.c_int64),
                ("thr64", ctypes.c_double), ("thr32_bits", ctypes.c_uint32), ("max_abs_bits", ctypes.c_uint32),
                ("eff_level", ctypes.c_int32), ("path", ctypes.c_int32)]

lib.wtp_wavelet_id.argtypes = [ctypes.c_char_p]
lib.wtp_workspace_size.argtypes = [ctypes.POINTER(WtpTensor), ctypes.c_int, ctypes.c_int, ctypes.c_int]
lib.wtp_workspace_size.restype = ctypes.c_size_t
lib.wtp_workspace_init.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
lib.wtp_prune_layers_f32.argtypes = [ctypes.POINTER(WtpTensor), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_double, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                     ctypes.c_void_p]
lib.wtp_last_error.restype = ctypes.c_char_p

def prune_layers(weights, wavelet, level, percentile):
    """weights: contiguous float32 CUDA tensors (e.g. every Conv2d.weight). In place."""
    n = len(weights)
    descs = (WtpTensor * n)()
    for d, w in zip(descs, weights):
        d.in_ = d.out = w.data_ptr(); d.ndim = w.dim()
        for i, s in enumerate(w.shape): d.shape[i] = s
    wid = lib.wtp_wavelet_id(wavelet.encode())
    nbytes = lib.wtp_workspace_size(descs, n, wid, level)
    ws = torch.empty(max(nbytes, 256), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    lib.wtp_workspace_init(ws.data_ptr(), ws.numel(), stream)   # once per workspace
    res = torch.empty(n * ctypes.sizeof(WtpResult), dtype=torch.uint8, device="cuda")
    rc = lib.wtp_prune_layers_f32(descs, n, wid, level, percentile, ws.data_ptr(), ws.numel(),
                                  res.data_ptr(), stream)
    if rc != 0:
        raise ValueError(lib.wtp_last_error().decode())
    recs = (WtpResult * n).from_buffer_copy(res.cpu().numpy().tobytes())
    return [(r.numel, r.numel - r.zero_count, r.zero_count) for r in recs]  # prune_layer_weights' tuple

lib.wtp_prune_f32.argtypes = lib.wtp_prune_layers_f32.argtypes

def multi_resolution_analysis(weights, wavelet, level, percentile):
    """dwt_pruning.py:35-95 over a list: the clamped level carries from one tensor to the next. In place."""
    n = len(weights)
    descs = (WtpTensor * n)()
    for d, w in zip(descs, weights):
        d.in_ = d.out = w.data_ptr(); d.ndim = w.dim()
        for i, s in enumerate(w.shape): d.shape[i] = s
    wid = lib.wtp_wavelet_id(wavelet.encode())
    nbytes = lib.wtp_workspace_size(descs, n, wid, level)
    ws = torch.empty(max(nbytes, 256), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    lib.wtp_workspace_init(ws.data_ptr(), ws.numel(), stream)
    res = torch.empty(n * ctypes.sizeof(WtpResult), dtype=torch.uint8, device="cuda")
    rc = lib.wtp_prune_f32(descs, n, wid, level, percentile, ws.data_ptr(), ws.numel(), res.data_ptr(), stream)
    if rc != 0:
        raise ValueError(lib.wtp_last_error().decode())
    return list((WtpResult * n).from_buffer_copy(res.cpu().numpy().tobytes()))
# --- end INTEGRATION.md block ---
