"""Drop-in counterpart of ResNet/min_weight_pruning.py (iAmGiG/WaveletTransforms) on MI355X.

The minimum-weight baseline that main_pruning.py runs beside the DWT pruning: every layer named
in the selective (DWT) log loses the same fraction of its smallest-magnitude weights, the
fraction being the DWT run's overall pruned fraction.  Same names, arguments, printed lines,
CSV rows and directory layout as the reference:

  read_selective_pruning_log      min_weight_pruning.py:42-51
  calculate_dwt_pruning_percentage min_weight_pruning.py:54-63
  percentage_min_pruning          min_weight_pruning.py:66-74   (GPU: libwtprune k-th select)
  min_weight_pruning              min_weight_pruning.py:77-139  (all layers in one launch sequence)

torch.topk(largest=False) leaves the order among equal magnitudes unspecified; here the lowest
flat indices go first among weights equal to the k-th smallest |w|.  The pruned counts (what
the reference logs) are exact either way.
"""
import csv
import os
from queue import Queue
from typing import Dict, Optional

import torch

from . import engine
from .utils import (append_to_experiment_log, check_and_set_pruned_instance_path, log_pruning_details, save_model,
                    setup_csv_writer)

__all__ = ["read_selective_pruning_log", "calculate_dwt_pruning_percentage", "percentage_min_pruning",
           "min_weight_pruning"]


def read_selective_pruning_log(selective_log_path: str) -> Dict[str, int]:
    pruned_layers = {}
    with open(selective_log_path, "r") as log_file:
        for row in csv.DictReader(log_file):
            pruned_layers[row["Layer Name"]] = int(row["Original Parameter Count"])
    return pruned_layers


def calculate_dwt_pruning_percentage(selective_log_path: str) -> float:
    total_params = 0
    total_pruned = 0
    with open(selective_log_path, "r") as log_file:
        for row in csv.DictReader(log_file):
            total_params += int(row["Original Parameter Count"])
            total_pruned += int(row["Total Pruned Count"])
    return total_pruned / total_params if total_params > 0 else 0.0


def _on_gpu(t):
    return t if t.is_cuda else t.to(torch.device("cuda", torch.cuda.current_device()))


def _min_prune_inplace(tensors, fraction):
    """Prune every tensor in place (any device); returns the per-tensor records."""
    work = [_on_gpu(w.detach()).reshape(-1) for w in tensors]
    work = [w if w.is_contiguous() else w.contiguous() for w in work]
    _, recs = engine.min_prune(work, fraction, outs=work)
    for w, src in zip(work, tensors):
        flat = src.data.view(-1) if src.is_contiguous() else None
        if flat is not None and flat.data_ptr() == w.data_ptr():
            continue
        with torch.no_grad():
            src.data.copy_(w.view_as(src))
    return recs


def percentage_min_pruning(weights: torch.Tensor, prune_percentage: float) -> torch.Tensor:
    """Prune a percentage of weights with the smallest absolute values (in place, like the
    reference's view assignment); returns the weights viewed in their own shape."""
    flatten_weights = weights.view(-1)
    _min_prune_inplace([flatten_weights], prune_percentage)
    return flatten_weights.view_as(weights)


def min_weight_pruning(model, selective_log_path: str, guid: str, wavelet: str, level: int, threshold: float,
                       csv_path: str, log_queue: Optional[Queue] = None) -> None:
    """Apply minimum weight pruning based on the overall pruning percentage from DWT-based pruning."""
    print(f"Starting min_weight_pruning with GUID: {guid}")
    min_pruned_dir = check_and_set_pruned_instance_path(
        f"{wavelet}_threshold-{threshold}_level-{level}_guid-{guid[:4]}/min_pruned")
    min_log_path = os.path.join(min_pruned_dir, "log.csv")
    min_csv_writer, min_log_file = setup_csv_writer(min_log_path, mode="w")
    try:
        overall_prune_percentage = calculate_dwt_pruning_percentage(selective_log_path)
        print(f"Overall pruning percentage from DWT: {overall_prune_percentage:.2%}")
        pruned_layers = read_selective_pruning_log(selective_log_path)
        print(f"Layers to be pruned: {list(pruned_layers.keys())}")

        modules = list(model.named_modules())
        targets = [(name, m) for name, m in modules
                   if name in pruned_layers and hasattr(m, "weight") and isinstance(m.weight, torch.Tensor)]
        recs = {}
        if targets:
            with torch.no_grad():
                out = _min_prune_inplace([m.weight for _, m in targets], overall_prune_percentage)
            recs = {name: r for (name, _), r in zip(targets, out)}

        total_params = 0
        total_pruned = 0
        for name, module in modules:
            if name in pruned_layers:
                if name in recs:
                    original_param_count = pruned_layers[name]
                    non_zero_params_after_pruning = recs[name]["nonzero"]
                    actual_pruned_count = original_param_count - non_zero_params_after_pruning
                    log_pruning_details(min_csv_writer, guid, wavelet, level, threshold, "min",
                                        original_param_count, non_zero_params_after_pruning, actual_pruned_count,
                                        name)
                    total_params += original_param_count
                    total_pruned += actual_pruned_count
                    print(f"Pruned layer: {name}, Original params: {original_param_count}, "
                          f"Pruned: {actual_pruned_count}")
                else:
                    print(f"Warning: Layer {name} does not have weights or is not a tensor.")
            else:
                print(f"Skipping layer: {name} (not in selective pruning log)")

        save_model(model, min_pruned_dir)
        if log_queue is not None:
            log_queue.put((guid, wavelet, level, threshold, "min",
                           total_pruned, total_params - total_pruned, min_pruned_dir))
        else:
            append_to_experiment_log(csv_path, guid, wavelet, level, threshold,
                                     "min", total_pruned, total_params - total_pruned, min_pruned_dir)
        min_log_file.close()
        print(f"Minimum weight pruning completed. Pruned {total_pruned} out of {total_params} parameters.")
        print(f"Actual pruning percentage: {total_pruned/total_params:.2%}")
    except Exception as e:
        print(f"Error in min_weight_pruning: {str(e)}")
        raise
