"""calculate_sparsity of ResNet/testing_suite/eval_model.py:7-20 on MI355X.

The sparsity the evaluation harness reports for a pruned model: the fraction of weights (params
with dim > 1; biases and norms skipped) whose magnitude is below `threshold`.  Every count runs on
the GPU (libwtprune k_count_small, one launch per parameter, all on one stream) and the host reads
the summed count once.  CPU parameters are copied to the current device first.
"""
import torch

from . import engine

__all__ = ["calculate_sparsity"]


def calculate_sparsity(model, threshold=1e-6):
    """Calculate the sparsity of the model."""
    total_params = 0
    near_zero = None
    dev = torch.device("cuda", torch.cuda.current_device())
    for param in model.parameters():
        if param.dim() > 1:  # only weights, not biases
            total_params += param.numel()
            p = param.detach()
            p = p if p.is_cuda else p.to(dev)
            if p.dtype != torch.float32:
                p = p.float()
            c = engine.count_small(p, threshold)
            near_zero = c if near_zero is None else near_zero.add_(c.to(near_zero.device))
    if total_params == 0:
        return 0.0  # avoid division by zero
    return int(near_zero.item()) / total_params
