"""cfg4: the layers of ONE model sharded over the ranks of one node, reassembled with a single
grouped exchange (torch.distributed; backend "nccl" = RCCL over xGMI on MI355X, "gloo" in CPU tests).

Every tensor is an independent selection population (its percentile is per tensor, as each
Conv2d is its own multi_resolution_analysis call in the reference loop, dwt_pruning.py:158-164),
so the path itself needs no exchange: each rank prunes the layers the LPT table assigns to it
straight into ITS region of the flat state_dict buffer (the outputs are views of it), and the
per-layer result records ride in the same region, as raw bytes behind the weights.  Then ONE
grouped exchange reassembles the pruned state_dict on every rank.

The exchange moves each rank's real bytes, unpadded: rank r's region is exactly its weights (16-byte
aligned) plus its records, and the regions lie back to back in rank order.  It is a full-mesh
all-gather -- every rank sends its region straight to each peer and receives each peer's region
in place (batch_isend_irecv: one NCCL group call of 2 (N - 1) point-to-point operations).  On
MI355X each GPU has a direct xGMI link to each of its 7 peers, so the 7 copies of a region run on
7 links at once and the exchange takes about (largest region) / (one link's bandwidth), where a
ring all-gather pushes every other rank's bytes through one link in turn.  Compute
and exchange are stream-ordered: nothing waits on the host before it.

A second exchange form is selectable (`exchange="allgather"`, SURVEY.md 8e's north_star wording):
every region padded to the largest one (rounded to 16 bytes) so that the regions sit at
r * stride, and ONE all_gather_into_tensor in place (rank r contributes full[r * stride : (r + 1) *
stride]).  RCCL runs it as a ring over xGMI: each link carries (N - 1) x stride bytes one after
another, so at N = 8 it moves 7 x 9.4 MB per link where the full mesh moves one region per link
 -- kept as the fallback and the comparison for the first multi-GPU runs.

The table is computed identically on every rank from the shapes alone.  After the exchange every
rank holds every record, so a resident launch that timed out on one rank (its tensors' records
read MODE_FAULT; nothing was stored for them) is seen by all ranks alike: the owners re-run exactly
those tensors in the three-launch form and all ranks join one more exchange.
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


def _align4(n):
    return (n + 3) // 4 * 4


class ShardPlan:
    """LPT owner of every tensor, and the layout of the flat state_dict buffer (float32 words):
    rank r's region [base[r], base[r] + size[r]) holds its tensors back to back (offset[i] into the
    region), then from rec_off[r] its records (16-byte aligned: the kernels update the records'
    8-byte counters in place, and every region starts 16-byte aligned for the float4 paths)."""

    EXCHANGES = ("p2p", "allgather")

    def __init__(self, shapes, world, exchange="p2p"):
        if exchange not in self.EXCHANGES:
            raise ValueError("exchange must be one of %s, got %r" % (self.EXCHANGES, exchange))
        self.exchange = exchange
        self.shapes = [tuple(s) for s in shapes]
        self.numels = [int(np.prod(s)) if len(s) else 1 for s in self.shapes]
        self.world = world
        self.owner, self.loads = lpt_shard(self.numels, world)
        self.mine = [[i for i in range(len(self.shapes)) if self.owner[i] == r] for r in range(world)]
        self.offset = [0] * len(self.shapes)  # element offset inside the owner's region
        for r in range(world):
            o = 0
            for i in self.mine[r]:
                self.offset[i] = o
                o += self.numels[i]
        self.max_shard = max(self.loads) if self.loads else 0
        self.rec_off = [_align4(self.loads[r]) for r in range(world)]
        self.size = [self.rec_off[r] + len(self.mine[r]) * REC_WORDS for r in range(world)]
        if exchange == "allgather":
            # padded regions at r * stride: the in-place all_gather_into_tensor layout
            self.stride = _align4(max(self.size)) if world else 0
            self.base = [r * self.stride for r in range(world)]
            self.total = self.stride * world
        else:
            self.stride = None
            self.base = [int(b) for b in np.concatenate([[0], np.cumsum(self.size)[:-1]])] if world else []
            self.total = int(sum(self.size))

    def region(self, r):
        return self.base[r], self.base[r] + self.size[r]

    def bytes_sent(self, r):
        """Bytes rank r puts on the wire in one exchange: its region to each peer (p2p), or in a
        ring all-gather (N - 1) padded regions -- its own and the ones it forwards."""
        if self.exchange == "allgather":
            return 4 * self.stride * (self.world - 1)
        return 4 * self.size[r] * (self.world - 1)

    def bytes_received(self, r):
        """Bytes rank r receives in one exchange (every other region once; padded for allgather)."""
        if self.exchange == "allgather":
            return 4 * self.stride * (self.world - 1)
        return 4 * (self.total - self.size[r])


def _host_records_bytes(recs):
    """Host record dicts (the CPU test double's output) as wtp_result bytes."""
    a = np.zeros(len(recs), _record_dtype())
    for i, r in enumerate(recs):
        for k in REC_FIELDS:
            a[i][k] = r[k]
    return a.view(np.uint8)


class _Shard:
    """One rank's region of the flat state_dict buffer `full` (allocated here when not given): its
    weights (the outputs are views of it), then its wtp_result records."""

    def __init__(self, weights, plan, rank, device, full=None):
        self.weights, self.plan, self.rank = weights, plan, rank
        self.mine = plan.mine[rank]
        if full is None:
            full = torch.empty(plan.total, dtype=torch.float32, device=device)
        self.full = full
        b0, b1 = plan.region(rank)
        self.buf = full[b0:b1]
        self.views = [self.buf[plan.offset[i]:plan.offset[i] + plan.numels[i]].view(plan.shapes[i]) for i in self.mine]
        self.recs_u8 = self.buf[plan.rec_off[rank]:].view(torch.uint8)

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


def exchange(full, plan, rank, group=None):
    """The all-gather of the regions (stream-ordered behind the compute that wrote the region; waits
    for completion).  plan.exchange "p2p": this rank's region of `full` goes to every peer and every
    peer's region lands in place, as ONE group of point-to-point operations; "allgather": ONE
    in-place all_gather_into_tensor of the padded regions."""
    if plan.world == 1:
        return
    if plan.exchange == "allgather":
        b0 = plan.base[rank]
        dist.all_gather_into_tensor(full[:plan.total], full[b0:b0 + plan.stride], group=group)
        return
    b0, b1 = plan.region(rank)
    mine = full[b0:b1]
    ops = []
    for p in range(plan.world):
        if p == rank:
            continue
        peer = dist.get_global_rank(group, p) if group is not None else p
        c0, c1 = plan.region(p)
        # a rank that owns no tensor (world > number of layers) has an empty region: both sides
        # read that from the shared plan and post no operation for it
        if b1 > b0:
            ops.append(dist.P2POp(dist.isend, mine, peer, group))
        if c1 > c0:
            ops.append(dist.P2POp(dist.irecv, full[c0:c1], peer, group))
    if not ops:
        return
    for req in dist.batch_isend_irecv(ops):
        req.wait()


def shard_local(weights, wavelet, level, pct, plan, rank, device=None, prune_fn=None, full=None):
    """Rank `rank`'s share of `plan`, pruned into its region (no communication): the bytes
    prune_sharded contributes to the exchange.  Returns the region (float32 tensor); with `full`
    given it is written in place there."""
    sh = _Shard(weights, plan, rank, device or weights[0].device, full)
    if sh.mine:
        sh.run(sh.mine, wavelet, level, pct, prune_fn)
    return sh.buf


def assemble(full, plan):
    """Flat state_dict buffer (plan.total words, every region in place) -> (every pruned tensor as a
    view, per-layer records)."""
    full = full.reshape(-1)
    recs = _decode_all(full, plan)
    out = []
    for i, s in enumerate(plan.shapes):
        b = plan.base[plan.owner[i]] + plan.offset[i]
        out.append(full[b:b + plan.numels[i]].view(s))
    return out, recs


def prune_sharded(weights, wavelet, level, pct, prune_fn=None, group=None, device=None, exchange_kind="p2p"):
    """weights: list of tensors (the same list on every rank).  prune_fn=None runs this rank's share
    on the GPU (engine.launch, one batched launch sequence, carry_level=False as wavelet_pruning
    does); a test double prune_fn(inputs, out_views) -> list of record dicts may replace it.
    exchange_kind: "p2p" (full mesh, unpadded) or "allgather" (padded, one all_gather_into_tensor).
    Returns (all pruned tensors on every rank, per-layer records, plan)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    plan = ShardPlan([w.shape for w in weights], world, exchange_kind)
    sh = _Shard(weights, plan, rank, device or weights[0].device)
    if sh.mine:
        sh.run(sh.mine, wavelet, level, pct, prune_fn)
    exchange(sh.full, plan, rank, group)
    full, recs = assemble(sh.full, plan)
    faulted = [i for i in range(len(weights)) if recs[i]["path"] == MODE_FAULT]
    if faulted:  # every rank sees the same set: the owners re-run, everyone exchanges again
        redo = [i for i in faulted if plan.owner[i] == rank]
        if redo:
            sh.run(redo, wavelet, level, pct, prune_fn, no_resident=True)
        exchange(sh.full, plan, rank, group)
        full, recs = assemble(sh.full, plan)
    return full, recs, plan


def _decode_all(full, plan):
    # only the record words travel to the host: every region's tail, concatenated in rank order
    tails = [full[plan.base[r] + plan.rec_off[r]:plan.base[r] + plan.size[r]] for r in range(plan.world)]
    host = torch.cat(tails).cpu().numpy().view(np.uint8)
    first = np.concatenate([[0], np.cumsum([len(m) for m in plan.mine])[:-1]]).astype(int)
    dt = _record_dtype()
    records = []
    for i in range(len(plan.shapes)):
        r = plan.owner[i]
        k = plan.mine[r].index(i)
        o = (int(first[r]) + k) * REC_BYTES
        row = host[o:o + REC_BYTES].copy().view(dt)[0]
        rec = {f: row[f].item() for f in REC_FIELDS}
        rec["nonzero"] = rec["numel"] - rec["zero_count"]
        records.append(rec)
    return records
