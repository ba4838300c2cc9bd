"""Drop-in counterpart of ResNet/random_pruning.py (iAmGiG/WaveletTransforms) on MI355X.

The random baseline main_pruning.py runs beside the DWT pruning (main_pruning.py:191-199): every
Conv2d layer named in the selective (DWT) log loses as many weights as the DWT pruning removed
from it ("Total Pruned Count"), at random positions.  Same name, arguments, printed lines, CSV
rows and directory layout as the reference (random_pruning.py:11-82).

The positions: the reference zeroes torch.randperm(numel)[:prune_count] (random_pruning.py:53-55).
Here every layer's positions are the first prune_count values of a keyed pseudo-random
permutation of [0, numel) (csrc/wt_perm.h), computed on the GPU one position per thread, all
layers in one launch sequence.  The key is drawn from torch's default CPU generator, so
torch.manual_seed makes a run reproducible, but torch's Philox stream is not reproduced: the
positions differ from the reference's, the counts (the only thing its logs record) follow the
same rule -- k distinct positions, Python's slice rule for k, count_nonzero afterwards.
"""
import csv
import os
from queue import Queue
from typing import Optional

import torch
import torch.nn as nn

from . import engine
from .utils import (append_to_experiment_log, check_and_set_pruned_instance_path, get_layer, log_pruning_details,
                    save_model, setup_csv_writer)

__all__ = ["random_pruning", "random_prune_tensors"]


def _draw_seed():
    return int(torch.randint(0, 2**62, (1,), dtype=torch.int64).item())


def random_prune_tensors(tensors, prune_counts, seed=None):
    """Zero randperm(numel)[:k] of every tensor in place (any device; CUDA float32 is pruned where
    it lies).  Returns the per-tensor records (numel, zero_count, nonzero)."""
    seed = _draw_seed() if seed is None else int(seed)
    recs = [None] * len(tensors)
    # a tensor named twice is pruned twice, in order (the reference's sequential loop): one launch
    # sequence per run of distinct tensors, so no launch prunes the same storage twice at once
    batches, cur, seen = [], [], set()
    for i, w in enumerate(tensors):
        key = (str(w.device), w.data_ptr())
        if key in seen:
            batches.append(cur)
            cur, seen = [], set()
        cur.append(i)
        seen.add(key)
    if cur:
        batches.append(cur)
    dev = torch.device("cuda", torch.cuda.current_device())
    for bno, idx in enumerate(batches):
        srcs = [tensors[i] for i in idx]
        work = [(s.detach() if s.is_cuda else s.detach().to(dev)).reshape(-1) for s in srcs]
        work = [w if w.is_contiguous() else w.contiguous() for w in work]
        _, out = engine.random_prune(work, [prune_counts[i] for i in idx], seed + bno, outs=work)
        for i, w, src, r in zip(idx, work, srcs, out):
            recs[i] = r
            flat = src.data.view(-1) if src.is_contiguous() else None
            if flat is None or flat.data_ptr() != w.data_ptr():
                with torch.no_grad():
                    src.data.copy_(w.view_as(src))
    return recs


def random_pruning(model, selective_log_path: str, guid: str, wavelet: str, level: int, threshold: float,
                   csv_path: str, log_queue: Optional[Queue] = None) -> None:
    """Apply random pruning to the model based on the selective pruning log."""
    total_pruned_count = 0
    total_non_zero_params = 0
    random_pruned_dir = check_and_set_pruned_instance_path(
        f"{wavelet}_threshold-{threshold}_level-{level}_guid-{guid[:4]}/random_pruned")
    random_log_path = os.path.join(random_pruned_dir, "log.csv")
    random_csv_writer, random_log_file = setup_csv_writer(os.path.normpath(random_log_path), mode="w")

    # pass 1 (host): the rows, their layers and the reference's prints, in file order
    rows = []
    with open(selective_log_path, "r") as log_file:
        for row in csv.DictReader(log_file):
            layer_name = row["Layer Name"]
            original_param_count = int(row["Original Parameter Count"])
            prune_count = int(row["Total Pruned Count"])
            print(f"Processing layer: {layer_name} with prune count: {prune_count}")
            layer = get_layer(model, layer_name)
            if layer and isinstance(layer, nn.Conv2d):
                rows.append((layer_name, original_param_count, prune_count, layer))
            else:
                print(f"Layer not found or not a Conv2D layer: {layer_name}")

    # pass 2 (GPU): every layer's randperm(numel)[:prune_count] = 0 in one launch sequence
    if rows:
        with torch.no_grad():
            recs = random_prune_tensors([r[3].weight.data for r in rows], [r[2] for r in rows])
        for (layer_name, original_param_count, _, _), rec in zip(rows, recs):
            non_zero_params_after_pruning = rec["nonzero"]
            actual_pruned_count = original_param_count - non_zero_params_after_pruning
            log_pruning_details(random_csv_writer, guid, wavelet, level, threshold, "random",
                                original_param_count, non_zero_params_after_pruning, actual_pruned_count, layer_name)
            total_pruned_count += actual_pruned_count
            total_non_zero_params += non_zero_params_after_pruning

    save_model(model, random_pruned_dir)
    if log_queue is not None:
        log_queue.put((guid, wavelet, level, threshold, "random",
                       total_pruned_count, total_non_zero_params, random_pruned_dir))
    else:
        append_to_experiment_log(csv_path, guid, wavelet, level, threshold,
                                 "random", total_pruned_count, total_non_zero_params, random_pruned_dir)
    random_log_file.close()
    print("Random pruning completed.")
