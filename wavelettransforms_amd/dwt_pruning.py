"""Drop-in counterpart of ResNet/dwt_pruning.py (iAmGiG/WaveletTransforms) on MI355X.

Same public names, arguments, return values, printed lines and exceptions as the reference
module; the arithmetic runs in libwtprune.so (HIP, gfx950) on device-resident tensors:

  calculate_max_level          dwt_pruning.py:12-13
  analyze_pruning              dwt_pruning.py:16-22
  percentile_based_thresholding dwt_pruning.py:25-32
  multi_resolution_analysis    dwt_pruning.py:35-95
  prune_layer_weights          dwt_pruning.py:98-127   (alias prune_conv_layer)
  wavelet_pruning              dwt_pruning.py:130-174  (alias apply_dwt_pruning)

Differences by design (documented in DESIGN.md): `wavelet_pruning` prunes every Conv2d of
the model in ONE batched launch sequence instead of a per-layer loop (results and logs are
identical); weights that live on the CPU are moved to the current CUDA device for the
computation and the results are returned on the weight's own device; only
mode='periodization' exists (the only mode the reference uses).
"""
import os
from typing import List, Tuple

import numpy as np
import torch
import torch.nn as nn

from . import engine
from . import _native as N
from .utils import (append_to_experiment_log, check_and_set_pruned_instance_path, log_pruning_details,
                    save_model, setup_csv_writer)

__all__ = ["calculate_max_level", "analyze_pruning", "percentile_based_thresholding",
           "multi_resolution_analysis", "prune_layer_weights", "wavelet_pruning",
           "prune_conv_layer", "apply_dwt_pruning"]


def _dec_len(wavelet):
    wid = engine.wavelet_id(wavelet)
    if wid < 0:
        raise ValueError("Unknown wavelet name '%s', check wavelist() for the list of available builtin "
                         "wavelets." % wavelet)
    return N.lib().wtp_dec_len(wid)


def calculate_max_level(shape, wavelet):
    """pywt.dwt_max_level(min(shape[-2:]), Wavelet(wavelet).dec_len)  (dwt_pruning.py:12-13)."""
    return N.lib().wtp_max_level(int(min(shape[-2:])), _dec_len(wavelet))


def analyze_pruning(model: nn.Module):
    """Print the sparsity of every Conv2d weight (dwt_pruning.py:16-22)."""
    for name, module in model.named_modules():
        if isinstance(module, nn.Conv2d):
            w = module.weight.data
            zeros = torch.count_nonzero(w == 0).item()
            print(f"Layer {name}: Sparsity = {zeros / w.numel():.2%}")


def _cuda(x):
    if x.is_cuda:
        return x
    return x.to(torch.device("cuda", torch.cuda.current_device()))


def _print_threshold_line(percentile, rec):
    # reference :29-30 prints np.float64 threshold and np.float32 max (shortest repr each)
    print(f"Percentile: {percentile}, Threshold: {np.float64(rec['thr64'])}, Max Coeff: {rec['max_abs']}")


def percentile_based_thresholding(coeff_arr, percentile=90):
    """np.where(|a| < np.percentile(|a|, percentile), 0, a) with NumPy 1.x semantics
    (dwt_pruning.py:25-32).  Accepts a NumPy array (returns NumPy, like the reference) or a
    torch tensor (returns a tensor on the same device)."""
    as_numpy = isinstance(coeff_arr, np.ndarray)
    t = torch.from_numpy(np.ascontiguousarray(coeff_arr, dtype=np.float32)) if as_numpy else coeff_arr
    dev = t.device
    out, rec = engine.threshold(_cuda(t.detach()), percentile)
    _print_threshold_line(percentile, rec)
    if as_numpy:
        return out.cpu().numpy().reshape(np.shape(coeff_arr))
    return out.to(dev)


def _run(weights, wavelet, level, percentile, carry_level, verbose, flatten=False):
    devs = [w.device for w in weights]
    dev_w = [_cuda(w.detach()) for w in weights]
    outs, recs = engine.prune(dev_w, wavelet, level, percentile, carry_level=carry_level, flatten=flatten)
    outs = [o.to(d) for o, d in zip(outs, devs)]
    if verbose:
        for r in recs:
            _print_threshold_line(percentile, r)
    return outs, recs


def _mismatches(weights, recs, flatten=False):
    n = 0
    for w, r in zip(weights, recs):
        if flatten:  # one line of numel samples: odd lengths are cut back silently
            continue
        if w.dim() >= 2 and r["eff_level"] > 0:
            h, wd = w.shape[-2], w.shape[-1]
            if h % 2 or wd % 2:
                n += 1
    return n


def multi_resolution_analysis(weights: List[torch.Tensor], wavelet: str, level: int, percentile: float,
                              mode: str = "periodization", verbose: bool = True,
                              flatten: bool = False) -> Tuple[List[torch.Tensor], int]:
    """Wavelet-domain percentile pruning of each tensor (dwt_pruning.py:35-95).
    Returns (pruned tensors on their original devices, total count of exact zeros).
    flatten=True (an extension, not in the reference): the 1-D pywt.wavedec / waverec of every
    ndim >= 2 tensor's flattened weights instead of the 2-D transform over its last two axes
    (WTP_FLATTEN, include/wtprune.h)."""
    if mode != "periodization":
        raise NotImplementedError("only mode='periodization' is implemented (the reference's only mode)")
    if len(weights) == 0:
        return [], 0
    with torch.no_grad():
        outs, recs = _run(list(weights), wavelet, level, percentile, True, verbose, flatten)
    mism = _mismatches(weights, recs, flatten)
    if mism > 0:
        print(f"Warning: Shape mismatch occurred in {mism} weights")
    outs = [o.to(dtype=w.dtype).view(w.shape) for o, w in zip(outs, weights)]
    return outs, int(sum(r["zero_count"] for r in recs))


def prune_layer_weights(layer: nn.Module, wavelet: str, level: int, percentile: float,
                        verbose: bool = True, flatten: bool = False) -> Tuple[int, int, int]:
    """Prune layer.weight in place (the bias is untouched); returns (numel, non-zero after,
    zero count) -- dwt_pruning.py:98-127."""
    with torch.no_grad():
        w = layer.weight
        pruned, zero_count = multi_resolution_analysis([w], wavelet, level, percentile, verbose=verbose,
                                                       flatten=flatten)
        original = w.numel()
        nonzero = int(torch.count_nonzero(pruned[0]).item())
        if verbose:
            print(f"Original Param Count: {original}, Non-zero Params: {nonzero}, Total Pruned Count: {zero_count}")
        layer.weight.data = pruned[0]
        return original, nonzero, zero_count


def wavelet_pruning(model, wavelet: str, level: int, percentile: float, csv_path: str, guid: str,
                    verbose: bool = True, flatten: bool = False) -> str:
    """Prune every Conv2d weight of `model`, log per layer, save the model and append the run
    to the experiment log; returns the per-layer log path (dwt_pruning.py:130-174).
    All layers go through ONE batched device launch sequence (each layer keeps its own
    requested level, exactly as the reference's per-layer calls do)."""
    threshold_value = percentile / 100
    out_dir = check_and_set_pruned_instance_path(
        f"{wavelet}_threshold-{threshold_value}_level-{level}_guid-{guid[:4]}/selective_pruned")
    log_path = os.path.join(out_dir, "log.csv")
    writer, fh = setup_csv_writer(os.path.normpath(log_path), mode="w")
    convs = [(name, m) for name, m in model.named_modules() if isinstance(m, nn.Conv2d)]
    total_pruned = 0
    total_nonzero = 0
    with torch.no_grad():
        weights = [m.weight for _, m in convs]
        outs, recs = _run(weights, wavelet, level, percentile, False, False, flatten) if convs else ([], [])
        for (name, m), out, rec in zip(convs, outs, recs):
            m.weight.data = out.to(dtype=m.weight.dtype).view(m.weight.shape)
            numel, zeros = rec["numel"], rec["zero_count"]
            nonzero = numel - zeros
            if verbose:  # the reference's per-layer output order (:29-30, :91-93, :121-122)
                _print_threshold_line(percentile, rec)
                if _mismatches([out], [rec], flatten):
                    print("Warning: Shape mismatch occurred in 1 weights")
                print(f"Original Param Count: {numel}, Non-zero Params: {nonzero}, Total Pruned Count: {zeros}")
            total_pruned += zeros
            total_nonzero += nonzero
            log_pruning_details(writer, guid, wavelet, level, threshold_value, "selective", numel, nonzero, zeros,
                                name)
    fh.close()
    save_model(model, out_dir)
    append_to_experiment_log(os.path.normpath(csv_path), guid, wavelet, level, threshold_value, "selective",
                             total_pruned, total_nonzero, out_dir)
    print(f"Selectively pruned model saved at {out_dir}")
    return log_path


# names used by the north-star description of the same functions
prune_conv_layer = prune_layer_weights
apply_dwt_pruning = wavelet_pruning
