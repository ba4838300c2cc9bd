"""cfg4: the layers of ONE model sharded over the ranks of one node, reassembled with a single
all-gather (torch.distributed; backend "nccl" = RCCL over xGMI on MI355X, "gloo" in CPU tests).

Every tensor is an independent selection population (its percentile is per tensor, as each
Conv2d is its own multi_resolution_analysis call in the reference loop, dwt_pruning.py:158-164),
so the path itself needs no exchange: each rank prunes the layers the LPT table assigns to it
straight into its flat shard (the outputs are views of the shard), then ONE
all_gather_into_tensor of the shards -- the per-layer result records ride in the same buffer,
as raw bytes behind the weights -- reassembles the pruned state_dict on every rank.  Compute
and collective are stream-ordered: nothing waits on the host before the all-gather.

The table is computed identically on every rank from the shapes alone.  After the collective
every rank holds every record, so a resident launch that timed out on one rank (its tensors'
records read MODE_FAULT; nothing was stored for them) is seen by all ranks alike: the owners
re-run exactly those tensors in the three-launch form and all ranks join one more all-gather.
"""
import numpy as np
import torch
import torch.distributed as dist

from .workloads import lpt_shard

REC_FIELDS = ("numel", "zero_count", "coeff_numel", "thr64", "thr32_bits", "max_abs_bits", "eff_level", "path")
MODE_FAULT = 99


def _record_dtype():
    """struct wtp_result (include/wtprune.h)."""
    return np.dtype([("numel", "<i8"), ("zero_count", "<i8"), ("coeff_numel", "<i8"), ("thr64", "<f8"),
                     ("thr32_bits", "<u4"), ("max_abs_bits", "<u4"), ("eff_level", "<i4"), ("path", "<i4")])


REC_BYTES = _record_dtype().itemsize  # 48
REC_WORDS = REC_BYTES // 4


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
        self.max_layers = max(1, max(len(m) for m in self.mine))
        # one rank's slice of the gathered buffer: its weights, then its records (float32 words,
        # 16-byte aligned: the kernels update the records' 8-byte counters in place)
        self.rec_off = (self.max_shard + 3) // 4 * 4
        self.slice = self.rec_off + self.max_layers * REC_WORDS


def _host_records_bytes(recs):
    """Host record dicts (the CPU test double's output) as wtp_result bytes."""
    a = np.zeros(len(recs), _record_dtype())
    for i, r in enumerate(recs):
        for k in REC_FIELDS:
            a[i][k] = r[k]
    return a.view(np.uint8)


class _Shard:
    """One rank's flat slice of the gathered buffer: its weights (the outputs are views of it), then
    its wtp_result records."""

    def __init__(self, weights, plan, rank, device):
        self.weights, self.plan, self.rank = weights, plan, rank
        self.mine = plan.mine[rank]
        self.buf = torch.zeros(plan.slice, dtype=torch.float32, device=device)
        self.views = [self.buf[plan.offset[i]:plan.offset[i] + plan.numels[i]].view(plan.shapes[i]) for i in self.mine]
        self.recs_u8 = self.buf[plan.rec_off:].view(torch.uint8)

    def run(self, idx, wavelet, level, pct, prune_fn=None, no_resident=False):
        mine, recs_u8 = self.mine, self.recs_u8
        ins = [self.weights[i] for i in idx]
        outs = [self.views[mine.index(i)] for i in idx]
        if prune_fn is None:
            from . import engine
            if idx == mine:  # the records land in place, behind the weights
                engine.launch(ins, wavelet, level, pct, outs=outs, carry_level=False, no_resident=no_resident,
                              results=recs_u8[:len(idx) * REC_BYTES])
            else:
                _, res = engine.launch(ins, wavelet, level, pct, outs=outs, carry_level=False,
                                       no_resident=no_resident)
                for j, i in enumerate(idx):
                    k = mine.index(i)
                    recs_u8[k * REC_BYTES:(k + 1) * REC_BYTES].copy_(res[j * REC_BYTES:(j + 1) * REC_BYTES])
        else:
            host = _host_records_bytes(prune_fn(ins, outs))
            for j, i in enumerate(idx):
                k = mine.index(i)
                recs_u8[k * REC_BYTES:(k + 1) * REC_BYTES].copy_(
                    torch.from_numpy(host[j * REC_BYTES:(j + 1) * REC_BYTES].copy()))


def shard_local(weights, wavelet, level, pct, plan, rank, device=None, prune_fn=None):
    """Rank `rank`'s share of `plan`, pruned into its flat slice (no communication): the slice
    prune_sharded contributes to the all-gather.  Returns the slice (float32 tensor)."""
    sh = _Shard(weights, plan, rank, device or weights[0].device)
    if sh.mine:
        sh.run(sh.mine, wavelet, level, pct, prune_fn)
    return sh.buf


def assemble(gathered, plan):
    """(world, slice) gathered buffer -> (every pruned tensor as a view, per-layer records)."""
    recs = _decode_all(gathered, plan)
    full = []
    for i, s in enumerate(plan.shapes):
        r = plan.owner[i]
        full.append(gathered[r, plan.offset[i]:plan.offset[i] + plan.numels[i]].view(s))
    return full, recs


def prune_sharded(weights, wavelet, level, pct, prune_fn=None, group=None, device=None):
    """weights: list of tensors (the same list on every rank).  prune_fn=None runs this rank's share
    on the GPU (engine.launch, one batched launch sequence, carry_level=False as wavelet_pruning
    does); a test double prune_fn(inputs, out_views) -> list of record dicts may replace it.
    Returns (all pruned tensors on every rank, per-layer records, plan)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    plan = ShardPlan([w.shape for w in weights], world)
    sh = _Shard(weights, plan, rank, device or weights[0].device)
    if sh.mine:
        sh.run(sh.mine, wavelet, level, pct, prune_fn)

    def gather():
        if world == 1:
            return sh.buf.view(1, -1)
        out = torch.empty(world * plan.slice, dtype=torch.float32, device=sh.buf.device)
        dist.all_gather_into_tensor(out, sh.buf, group=group)
        return out.view(world, -1)

    gathered = gather()
    full, recs = assemble(gathered, plan)
    faulted = [i for i in range(len(weights)) if recs[i]["path"] == MODE_FAULT]
    if faulted:  # every rank sees the same set: the owners re-run, everyone gathers again
        redo = [i for i in faulted if plan.owner[i] == rank]
        if redo:
            sh.run(redo, wavelet, level, pct, prune_fn, no_resident=True)
        full, recs = assemble(gather(), plan)
    return full, recs, plan


def _decode_all(gathered, plan):
    host = gathered[:, plan.rec_off:].contiguous().cpu().numpy().view(np.uint8)
    dt = _record_dtype()
    records = []
    for i in range(len(plan.shapes)):
        r = plan.owner[i]
        k = plan.mine[r].index(i)
        row = host[r, k * REC_BYTES:(k + 1) * REC_BYTES].copy().view(dt)[0]
        rec = {f: row[f].item() for f in REC_FIELDS}
        rec["nonzero"] = rec["numel"] - rec["zero_count"]
        records.append(rec)
    return records
