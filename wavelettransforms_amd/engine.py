"""Device-resident execution of the DWT -> percentile-threshold -> IDWT path for torch tensors.

`launch()` issues one batched launch sequence (libwtprune.so) for a list of CUDA float32
tensors on the current stream and returns the outputs plus the device-side result records;
`prune()` additionally waits and decodes them.  Nothing here computes on the CPU: the
numbers come from the HIP kernels, the host only packs pointers and decodes results.
"""
import ctypes
import warnings

import numpy as np
import torch

from . import _native as N

RESULT_DTYPE = np.dtype([("numel", "<i8"), ("zero_count", "<i8"), ("coeff_numel", "<i8"), ("thr64", "<f8"),
                         ("thr32_bits", "<u4"), ("max_abs_bits", "<u4"), ("eff_level", "<i4"), ("path", "<i4")])
assert RESULT_DTYPE.itemsize == N.RESULT_BYTES

_workspaces = {}


def wavelet_id(name):
    return N.lib().wtp_wavelet_id(str(name).encode()) if isinstance(name, str) else -1


def workspace(device, nbytes, stream=None):
    """Grow-only, zero-initialised workspace per (device, stream): the selection, barrier and
    parity state of a call live in it, so calls on distinct streams need distinct workspaces
    (include/wtprune.h).  The library keeps it clean between calls on its stream.  Each stream
    ever used keeps its workspace (at the largest size it needed: a cfg5-sized call holds the
    packed coefficients of its images) until release_workspaces() drops it."""
    device = torch.device(device)
    if device.index is None:
        device = torch.device(device.type, torch.cuda.current_device())
    if stream is None:
        stream = torch.cuda.current_stream(device)
    key = (device.index, stream.cuda_stream)
    ws = _workspaces.get(key)
    if ws is None or ws.numel() < nbytes:
        if torch.cuda.is_current_stream_capturing():
            # the zero-fill below becomes a node of the graph and re-zeroes the workspace on every
            # replay (correct, but a memset of the whole workspace per replay): warm the call up on
            # the capturing stream first (torch.cuda.graph(g, stream=s) after a call on s)
            warnings.warn("wavelettransforms_amd: workspace allocated inside a graph capture; its "
                          "zero-fill is replayed with the graph", RuntimeWarning, stacklevel=3)
        # allocated (and zeroed) on the call's stream, so the caching allocator ties the block to it
        with torch.cuda.stream(stream):
            ws = torch.zeros(max(int(nbytes), 256), dtype=torch.uint8, device=device)
        _workspaces[key] = ws
    return ws


def release_workspaces(device=None, stream=None):
    """Drop the cached workspaces (all, one device's, or one (device, stream)'s): their memory goes
    back to torch's caching allocator.  Call it after the stream's work has been waited for or
    when retiring a stream whose handle may be recycled; the next call allocates a zeroed one."""
    for key in list(_workspaces):
        if device is not None and key[0] != torch.device(device).index:
            continue
        if stream is not None and key[1] != stream.cuda_stream:
            continue
        del _workspaces[key]


def _results(n, device, stream):
    with torch.cuda.stream(stream):
        return torch.empty(n * N.RESULT_BYTES, dtype=torch.uint8, device=device)


def check_outs(tensors, outs):
    """Caller-supplied outputs must be dense float32 CUDA tensors shaped like their inputs: the
    library writes numel contiguous floats from out.data_ptr()."""
    if len(outs) != len(tensors):
        raise ValueError("wavelettransforms_amd: %d outputs for %d tensors" % (len(outs), len(tensors)))
    for i, (x, y) in enumerate(zip(tensors, outs)):
        if not isinstance(y, torch.Tensor) or not y.is_cuda or y.dtype != torch.float32:
            raise TypeError("wavelettransforms_amd: outs[%d] must be a float32 CUDA tensor" % i)
        if y.device != x.device or y.numel() != x.numel():
            raise ValueError("wavelettransforms_amd: outs[%d] has %d elements on %s, input %d on %s"
                             % (i, y.numel(), y.device, x.numel(), x.device))
        if not y.is_contiguous():
            raise ValueError("wavelettransforms_amd: outs[%d] is not contiguous" % i)


def _as_desc(tensors, outs):
    arr = (N.WtpTensor * max(1, len(tensors)))()
    for i, (x, y) in enumerate(zip(tensors, outs)):
        d = arr[i]
        d.in_ = x.data_ptr() if x.numel() else None
        d.out = y.data_ptr() if y.numel() else None
        d.ndim = x.dim()
        for j, s in enumerate(x.shape):
            d.shape[j] = s
    return arr


def raise_for(code, tensors, wavelet):
    """Map a library status to the exception the reference path raises at that point."""
    L = N.lib()
    msg = N.last_error()
    t = L.wtp_last_error_tensor()
    if code == N.WTP_EBADWAVELET:
        raise ValueError("Unknown wavelet name '%s', check wavelist() for the list of available builtin "
                         "wavelets." % wavelet)
    if code in (N.WTP_EBADLEVEL, N.WTP_EBADPCT):
        raise ValueError(msg)
    if code == N.WTP_EEMPTY:
        raise IndexError(msg)
    if code == N.WTP_ECROP:
        x = tensors[t] if 0 <= t < len(tensors) else None
        if x is not None and x.dim() > 4:
            raise RuntimeError("shape '%s' is invalid for input of size %d" % (list(x.shape), _recon_numel(x)))
        raise IndexError(msg)
    raise RuntimeError("libwtprune: %s (status %d)" % (msg, code))


def _recon_numel(x):
    # size of the waverec2 output after the reference's 4-index crop (for the error message)
    shape = list(x.shape)
    h, w = shape[-2], shape[-1]
    shape[-1] = 2 * ((w + 1) // 2)
    if x.dim() >= 6:
        shape[-2] = 2 * ((h + 1) // 2)
    n = 1
    for s in shape:
        n *= s
    return n


def check_tensors(tensors):
    for x in tensors:
        if not isinstance(x, torch.Tensor):
            raise TypeError("expected torch.Tensor, got %r" % type(x))
        if not x.is_cuda:
            raise ValueError("wavelettransforms_amd runs on the GPU: tensor on %s (move it to cuda)" % x.device)
        if x.dtype != torch.float32:
            raise TypeError("wavelettransforms_amd: float32 weights only (got %s)" % x.dtype)


WTP_CARRY_LEVEL, WTP_FLATTEN, WTP_NO_RESIDENT = 1, 2, 4  # include/wtprune.h


def launch(tensors, wavelet, level, pct, outs=None, carry_level=True, stream=None, flatten=False,
           no_resident=False, results=None):
    """Enqueue the path for `tensors` (CUDA float32) on `stream` (default: current stream).
    Returns (outs, results_dev) without synchronising; results_dev is a uint8 CUDA tensor of
    len(tensors) wtp_result records.  carry_level=True is multi_resolution_analysis over a
    list (the clamped level carries over, dwt_pruning.py:64-65); False is one call per layer
    (prune_layer_weights / wavelet_pruning).  flatten=True: the 1-D flattened mode (WTP_FLATTEN).
    A record whose path reads MODE_FAULT was not computed (the resident launch's grid was not
    co-resident; nothing was stored for that tensor): prune() re-runs such tensors itself.
    results: optional uint8 CUDA tensor of len(tensors) records (8-byte aligned) to write into."""
    check_tensors(tensors)
    tensors = [x.contiguous() for x in tensors]
    if outs is None:
        outs = [torch.empty_like(x) for x in tensors]
    else:
        check_outs(tensors, outs)
    n = len(tensors)
    if n == 0:
        return outs, None
    device = tensors[0].device
    L = N.lib()
    wid = wavelet_id(wavelet)
    desc = _as_desc(tensors, outs)
    flags = ((WTP_CARRY_LEVEL if carry_level else 0) | (WTP_FLATTEN if flatten else 0)
             | (WTP_NO_RESIDENT if no_resident else 0))
    nbytes = L.wtp_workspace_size_ex(desc, n, wid, int(level), flags)
    if stream is None:
        stream = torch.cuda.current_stream(device)
    ws = workspace(device, nbytes if nbytes else 256, stream)
    if results is None:
        res = _results(n, device, stream)
    else:
        if (results.dtype != torch.uint8 or not results.is_cuda or results.numel() < n * N.RESULT_BYTES
                or results.data_ptr() % 8):
            raise ValueError("wavelettransforms_amd: results must be %d 8-byte aligned CUDA bytes" % (n * N.RESULT_BYTES))
        res = results
    rc = L.wtp_prune_ex_f32(desc, n, wid, int(level), float(pct), flags, ws.data_ptr(), ws.numel(), res.data_ptr(),
                            ctypes.c_void_p(stream.cuda_stream))
    if rc != N.WTP_OK:
        raise_for(rc, tensors, wavelet)
    return outs, res


MODE_FAULT = 99  # WTP_PATH_FAULT: the resident launch timed out for this tensor and stored nothing
MODE_SMALL = 4   # WTP_PATH_SMALL: the whole call ran as one launch (csrc/small.hip)


def carried_level(tensors, wavelet, level, flatten=False):
    """The level multi_resolution_analysis passes on after `tensors` (dwt_pruning.py:64-65: every
    tensor with ndim >= 2 clamps it to pywt.dwt_max_level of min(kh, kw) -- of numel in the
    flattened mode)."""
    L = N.lib()
    F = L.wtp_dec_len(wavelet_id(wavelet))
    lvl = int(level)
    for x in tensors:
        if x.dim() >= 2:
            n = x.numel() if flatten else min(x.shape[-2], x.shape[-1])
            lvl = min(lvl, int(L.wtp_max_level(int(n), int(F))))
    return lvl


def fault_mask(results_dev, n):
    """Per-tensor flags: True where the record reads MODE_FAULT (host copy of the records)."""
    host = results_dev.cpu().numpy().view(RESULT_DTYPE)[:n]
    return host["path"] == MODE_FAULT


def decode(results_dev, n):
    host = results_dev.cpu().numpy().view(RESULT_DTYPE)[:n]
    out = []
    if (host["path"] == MODE_FAULT).any():
        raise RuntimeError("wavelettransforms_amd: records of a resident launch that timed out (MODE_FAULT); "
                           "re-run those tensors with no_resident=True (prune() does this itself)")
    for r in host:
        d = {k: r[k].item() for k in RESULT_DTYPE.names}
        d["thr32"] = float(np.array(d["thr32_bits"], np.uint32).view(np.float32))
        d["max_abs"] = np.array(d["max_abs_bits"], np.uint32).view(np.float32)[()]
        d["nonzero"] = d["numel"] - d["zero_count"]
        out.append(d)
    return out


def set_resident(enabled):
    """Allow (default) or forbid the one-launch resident form of level-0 groups; returns the previous setting."""
    return bool(N.lib().wtp_set_resident(1 if enabled else 0))


def set_pipeline(enabled):
    """Overlap each launch group's selection with the next group's forward transform on a side
    stream (True / 1, the default); False / 0 one stream (include/wtprune.h wtp_set_pipeline).
    Returns the previous mode."""
    mode = (1 if enabled else 0) if isinstance(enabled, bool) else int(enabled)
    return int(N.lib().wtp_set_pipeline(mode))


def set_fused_select(enabled):
    """Fused selection for launch groups of large wavelet-transformed tensors (True / 1, the
    default): the window from a transform of input patches before the forward, the forward
    classifying the coefficients it writes, no re-read of the packed array; False / 0 the
    window / collect / select passes over the packed array (include/wtprune.h
    wtp_set_fused_select).  Identical results either way.  Returns the previous mode."""
    return int(N.lib().wtp_set_fused_select(1 if enabled else 0))


def set_interior(enabled):
    """Filter-bank kernel choice (include/wtprune.h wtp_set_interior): 2 the interior tiles in the
    edge-free kernels and the frame around them in their edge form, True / 3 the same but a small
    level in one launch of the edge form (default), 1 the frame in the general kernel, False / 0
    every tile in the general kernel; returns the previous mode."""
    mode = (3 if enabled else 0) if isinstance(enabled, bool) else int(enabled)
    return int(N.lib().wtp_set_interior(mode))


def resident_capacity():
    """Workgroups (of 49152 weights) the resident launch can hold on the current device; 0: never used."""
    return int(N.lib().wtp_resident_capacity())


def prune(tensors, wavelet, level, pct, outs=None, carry_level=True, flatten=False):
    """launch() + wait + decoded per-tensor records (numel, zero_count, nonzero, thr64, ...).
    Tensors whose resident launch faulted (their inputs and outputs untouched) are re-run once in
    the three-launch form -- only those: a tensor pruned in place must not be pruned twice.  Under
    carry_level each one re-runs at the level the list carried into it (computed from the shapes
    of the tensors before it), as an independent call, grouped by that level."""
    outs, res = launch(tensors, wavelet, level, pct, outs=outs, carry_level=carry_level, flatten=flatten)
    if res is None:
        return outs, []
    n = len(tensors)
    bad = fault_mask(res, n)
    if bad.any():
        idx = [i for i in range(n) if bad[i]]
        groups = {}
        for i in idx:
            lvl = carried_level(tensors[:i], wavelet, level, flatten) if carry_level else int(level)
            groups.setdefault(lvl, []).append(i)
        merged = res.clone().view(n, N.RESULT_BYTES)
        for lvl, g in groups.items():
            _, res2 = launch([tensors[i] for i in g], wavelet, lvl, pct, outs=[outs[i] for i in g],
                             carry_level=False, flatten=flatten, no_resident=True)
            merged[g] = res2.view(len(g), N.RESULT_BYTES)
        res = merged.view(-1)
    return outs, decode(res, n)


def min_prune(tensors, fraction, outs=None):
    """percentage_min_pruning (min_weight_pruning.py:66-74) of every tensor (CUDA float32) in one
    launch sequence: zero the int(numel * fraction) smallest |w|; ties at the boundary lowest
    flat index first.  Returns (outs, records); outs may be the inputs (in place)."""
    check_tensors(tensors)
    tensors = [x.contiguous() for x in tensors]
    if outs is None:
        outs = [torch.empty_like(x) for x in tensors]
    else:
        check_outs(tensors, outs)
    n = len(tensors)
    if n == 0:
        return outs, []
    device = tensors[0].device
    L = N.lib()
    desc = _as_desc(tensors, outs)
    nbytes = L.wtp_min_prune_workspace_size(desc, n, float(fraction))
    ws = workspace(device, nbytes if nbytes else 256)
    res = torch.empty(n * N.RESULT_BYTES, dtype=torch.uint8, device=device)
    rc = L.wtp_min_prune_f32(desc, n, float(fraction), ws.data_ptr(), ws.numel(), res.data_ptr(),
                             ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream))
    if rc != N.WTP_OK:
        msg = N.last_error()
        if rc == N.WTP_EARG and "NaN" in msg:
            raise ValueError(msg)
        if rc == N.WTP_EARG:
            raise RuntimeError(msg)  # torch.topk: "selected index k out of range"
        raise_for(rc, tensors, None)
    return outs, decode(res, n)


def random_prune(tensors, prune_counts, seed, outs=None):
    """random_pruning's per-layer step (random_pruning.py:53-56) for every tensor (CUDA float32)
    in one launch sequence: zero randperm(numel)[:k] -- k distinct flat positions of a keyed
    permutation (csrc/wt_perm.h; tensor index t keys tensor t).  Returns (outs, records)."""
    check_tensors(tensors)
    tensors = [x.contiguous() for x in tensors]
    if outs is None:
        outs = [torch.empty_like(x) for x in tensors]
    else:
        check_outs(tensors, outs)
    n = len(tensors)
    if n == 0:
        return outs, []
    if len(prune_counts) != n:
        raise ValueError("random_prune: %d prune counts for %d tensors" % (len(prune_counts), n))
    device = tensors[0].device
    desc = _as_desc(tensors, outs)
    ks = (ctypes.c_int64 * n)(*[int(k) for k in prune_counts])
    res = torch.empty(n * N.RESULT_BYTES, dtype=torch.uint8, device=device)
    rc = N.lib().wtp_random_prune_f32(desc, n, ks, ctypes.c_uint64(int(seed) & (2**64 - 1)), res.data_ptr(),
                                      ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream))
    if rc != N.WTP_OK:
        raise_for(rc, tensors, None)
    return outs, decode(res, n)


def count_small(x, thr):
    """#(|x| < thr) of a CUDA float32 tensor, thr rounded to float32 as torch's float compare does
    (calculate_sparsity, testing_suite/eval_model.py:14).  Returns a 0-d int64 CUDA tensor."""
    check_tensors([x])
    x = x.contiguous()
    cnt = torch.empty((), dtype=torch.int64, device=x.device)
    rc = N.lib().wtp_count_small_f32(x.data_ptr() if x.numel() else None, x.numel(), float(thr), cnt.data_ptr(),
                                     ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
    if rc != N.WTP_OK:
        raise RuntimeError(N.last_error())
    return cnt


def threshold(x, pct, out=None):
    """percentile_based_thresholding (dwt_pruning.py:25-32) of a CUDA float32 tensor."""
    check_tensors([x])
    x = x.contiguous()
    if out is None:
        out = torch.empty_like(x)
    else:
        check_outs([x], [out])
    L = N.lib()
    desc = _as_desc([x.reshape(-1)], [out.reshape(-1)])
    ws = workspace(x.device, L.wtp_workspace_size(desc, 1, -1, 0) or 256)
    res = torch.empty(N.RESULT_BYTES, dtype=torch.uint8, device=x.device)
    rc = L.wtp_threshold_f32(x.data_ptr() if x.numel() else None, out.data_ptr() if x.numel() else None,
                             x.numel(), float(pct), ws.data_ptr(), ws.numel(), res.data_ptr(),
                             ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
    if rc != N.WTP_OK:
        raise_for(rc, [x], None)
    return out, decode(res, 1)[0]


def wavedec2_packed(x, wavelet, level):
    """pywt.coeffs_to_array(pywt.wavedec2(x, wavelet, level, 'periodization', axes=(-2,-1)))[0] on the GPU."""
    check_tensors([x])
    x = x.contiguous()
    L = N.lib()
    H, W = x.shape[-2], x.shape[-1]
    B = x.numel() // max(1, H * W)
    pr, pc = ctypes.c_int64(), ctypes.c_int64()
    if L.wtp_packed_shape(H, W, int(level), ctypes.byref(pr), ctypes.byref(pc)) != 0:
        raise ValueError(N.last_error())
    P = torch.empty(tuple(x.shape[:-2]) + (pr.value, pc.value), dtype=torch.float32, device=x.device)
    nb = L.wtp_dwt_workspace_size(B, H, W, int(level))
    ws = torch.empty(max(nb, 256), dtype=torch.uint8, device=x.device)
    rc = L.wtp_wavedec2_f32(x.data_ptr(), P.data_ptr(), B, H, W, wavelet_id(wavelet), int(level), ws.data_ptr(),
                            ws.numel(), ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
    if rc != 0:
        raise_for(rc, [x], wavelet)
    return P


def waverec2_packed(P, shape, wavelet, level, thr32=None):
    """array_to_coeffs + waverec2 + crop to `shape` (optionally thresholding on load)."""
    L = N.lib()
    H, W = shape[-2], shape[-1]
    B = 1
    for s in shape[:-2]:
        B *= s
    out = torch.empty(tuple(shape), dtype=torch.float32, device=P.device)
    nb = L.wtp_dwt_workspace_size(B, H, W, int(level))
    ws = torch.empty(max(nb, 256), dtype=torch.uint8, device=P.device)
    thr = None
    if thr32 is not None:
        thr = torch.tensor([thr32], dtype=torch.float32, device=P.device)
    rc = L.wtp_waverec2_f32(P.contiguous().data_ptr(), out.data_ptr(), B, H, W, wavelet_id(wavelet), int(level),
                            thr.data_ptr() if thr is not None else None, ws.data_ptr(), ws.numel(),
                            ctypes.c_void_p(torch.cuda.current_stream(P.device).cuda_stream))
    if rc != 0:
        raise_for(rc, [P], wavelet)
    return out


def synth(shape, seed, tensor_id, e, device="cuda"):
    """Synthetic weights on the device (csrc/wt_synth.h), identical to workloads.synth_numpy."""
    n = 1
    for s in shape:
        n *= s
    out = torch.empty(tuple(shape), dtype=torch.float32, device=device)
    rc = N.lib().wtp_synth_f32(out.data_ptr() if n else None, n, seed, tensor_id, int(e),
                               ctypes.c_void_p(torch.cuda.current_stream(out.device).cuda_stream))
    if rc != 0:
        raise RuntimeError(N.last_error())
    return out
