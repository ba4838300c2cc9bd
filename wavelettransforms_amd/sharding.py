"""cfg4: the layers of ONE model sharded over the ranks of one node, reassembled with a single
all-gather (torch.distributed; backend "nccl" = RCCL over xGMI on MI355X, "gloo" in CPU tests).

Every tensor is an independent selection population (its percentile is per tensor), so the
path itself needs no exchange: each rank prunes the layers the LPT table assigns to it, then
ONE all_gather_into_tensor of the flat pruned shards (padded to the largest shard) plus ONE
all-gather of the per-layer result records reassemble the pruned state_dict on every rank.
The table is computed identically on every rank from the shapes alone.
"""
import numpy as np
import torch
import torch.distributed as dist

from .workloads import lpt_shard

REC_FIELDS = ("numel", "zero_count", "coeff_numel", "thr64", "thr32_bits", "max_abs_bits", "eff_level", "path")


class ShardPlan:
    def __init__(self, shapes, world):
        self.shapes = [tuple(s) for s in shapes]
        self.numels = [int(np.prod(s)) if len(s) else 1 for s in self.shapes]
        self.world = world
        self.owner, self.loads = lpt_shard(self.numels, world)
        self.mine = [[i for i in range(len(self.shapes)) if self.owner[i] == r] for r in range(world)]
        self.offset = [0] * len(self.shapes)  # element offset inside the owner's flat shard
        for r in range(world):
            o = 0
            for i in self.mine[r]:
                self.offset[i] = o
                o += self.numels[i]
        self.max_shard = max(self.loads) if self.loads else 0


def _pack_records(recs):
    a = np.zeros((len(recs), len(REC_FIELDS)), np.float64)
    for i, r in enumerate(recs):
        for j, k in enumerate(REC_FIELDS):
            a[i, j] = float(r[k])
    return a


def prune_sharded(weights, wavelet, level, pct, prune_fn, group=None, device=None):
    """weights: list of tensors (the same list on every rank).  prune_fn(list_of_tensors) ->
    (outs, records) runs this rank's share (engine.prune with carry_level=False on the GPU).
    Returns (all pruned tensors on every rank, per-layer records, timing dict)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    plan = ShardPlan([w.shape for w in weights], world)
    device = device or weights[0].device
    mine = plan.mine[rank]
    outs, recs = prune_fn([weights[i] for i in mine]) if mine else ([], [])
    flat = torch.zeros(plan.max_shard, dtype=torch.float32, device=device)
    for i, o in zip(mine, outs):
        flat[plan.offset[i]:plan.offset[i] + plan.numels[i]] = o.reshape(-1)
    rec_local = np.zeros((max(1, max(len(m) for m in plan.mine)), len(REC_FIELDS)), np.float64)
    if recs:
        rec_local[:len(recs)] = _pack_records(recs)
    rec_t = torch.from_numpy(rec_local).to(device)
    if world > 1:
        gathered = torch.empty(world * plan.max_shard, dtype=torch.float32, device=device)
        dist.all_gather_into_tensor(gathered, flat, group=group)
        rec_all = torch.empty((world * rec_t.shape[0], rec_t.shape[1]), dtype=rec_t.dtype, device=device)
        dist.all_gather_into_tensor(rec_all, rec_t, group=group)  # concatenated along dim 0
        rec_all = rec_all.view(world, rec_t.shape[0], rec_t.shape[1])
    else:
        gathered, rec_all = flat, rec_t.unsqueeze(0)
    rec_np = rec_all.cpu().numpy()
    full, records = [], []
    for i, s in enumerate(plan.shapes):
        r = plan.owner[i]
        base = r * plan.max_shard + plan.offset[i]
        full.append(gathered[base:base + plan.numels[i]].view(s))
        row = rec_np[r, plan.mine[r].index(i)]
        rec = {k: row[j] for j, k in enumerate(REC_FIELDS)}
        for k in REC_FIELDS:
            if k != "thr64":
                rec[k] = int(rec[k])
        rec["nonzero"] = rec["numel"] - rec["zero_count"]
        records.append(rec)
    return full, records, plan
