"""cfg4 sharding: LPT plan and the all-gather reassembly, world_size 2 over gloo on
the CPU.  The per-rank prune function is a test double (the C oracle, layer by layer, writing into
the flat-shard views); on the GPU the same code path runs engine.launch over RCCL
(tests/test_gpu_sharding.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from wavelettransforms_amd import workloads as W
from wavelettransforms_amd.sharding import REC_BYTES, REC_WORDS, ShardPlan, prune_sharded


def test_lpt_plan_resnet18():
    shapes = [s for _, s, *_ in W.resnet18_tensors(0)]
    for world, cap in [(1, 11_166_912), (2, None), (4, 2_949_120), (8, 2_359_296)]:
        plan = ShardPlan(shapes, world)
        assert sorted(i for m in plan.mine for i in m) == list(range(len(shapes)))
        assert sum(plan.loads) == 11_166_912
        if cap:
            assert plan.max_shard == cap
        for r in range(world):  # offsets tile each rank's flat shard exactly
            o = 0
            for i in plan.mine[r]:
                assert plan.offset[i] == o
                o += plan.numels[i]
            assert o == plan.loads[r]
        # the regions lie back to back, 16-byte aligned, unpadded: weights + <= 3 pad words + records
        assert plan.base[0] == 0 and plan.total == sum(plan.size)
        for r in range(world):
            assert plan.base[r] % 4 == 0 and plan.rec_off[r] % 4 == 0
            assert plan.size[r] - plan.loads[r] - len(plan.mine[r]) * REC_WORDS in range(4)
            if r + 1 < world:
                assert plan.base[r + 1] == plan.base[r] + plan.size[r]
            assert plan.bytes_received(r) == 4 * (plan.total - plan.size[r])
        if world == 8:  # every rank receives at most the whole model's weights (+ records)
            assert max(plan.bytes_received(r) for r in range(world)) <= 4 * 11_166_912 + 20 * REC_BYTES + 8 * 12


def test_lpt_plan_allgather_layout():
    """exchange="allgather": the same LPT table, every region padded to one 16-byte-aligned stride
    and placed at r * stride (the in-place all_gather_into_tensor layout)"""
    shapes = [s for _, s, *_ in W.resnet18_tensors(0)]
    for world in (1, 2, 3, 4, 8):
        p2p, ag = ShardPlan(shapes, world), ShardPlan(shapes, world, "allgather")
        assert ag.mine == p2p.mine and ag.offset == p2p.offset and ag.size == p2p.size
        assert ag.stride % 4 == 0 and ag.stride >= max(ag.size)
        assert ag.base == [r * ag.stride for r in range(world)] and ag.total == world * ag.stride
        for r in range(world):
            assert ag.bytes_received(r) == 4 * ag.stride * (world - 1) >= p2p.bytes_received(r)
    with pytest.raises(ValueError):
        ShardPlan(shapes, 2, "ring")


def _oracle_prune(wavelet, level, pct):
    from oracle import oracle as O

    def fn(sub, outs):
        recs = []
        for x, y in zip(sub, outs):
            o, r = O.prune_tensor(x.numpy(), wavelet, level, pct)
            y.copy_(torch.from_numpy(np.ascontiguousarray(o)))
            recs.append({"numel": r["numel"], "zero_count": r["zero_count"], "coeff_numel": r["coeff_numel"],
                         "thr64": r["thr64"], "eff_level": r["eff_level"], "path": 0,
                         "thr32_bits": int(np.float32(r["thr32"]).view(np.uint32)),
                         "max_abs_bits": int(np.float32(r["max_abs"]).view(np.uint32))})
        return recs
    return fn


def _tensors(ntens):
    ts = W.resnet18_tensors(0)[:7] + [("mlp", (10, 128), 101, 1, 14)]
    return ts if ntens is None else ts[:ntens]


def _worker(rank, world, port, q, ntens=None, kind="p2p"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ts = _tensors(ntens)
        xs = [torch.from_numpy(W.synth_numpy(s, seed, tid, e)) for _, s, seed, tid, e in ts]
        full, recs, plan = prune_sharded(xs, "haar", 2, 61.8, _oracle_prune("haar", 2, 61.8),
                                         device=torch.device("cpu"), exchange_kind=kind)
        q.put((rank, [f.numpy().copy() for f in full], recs, plan.mine))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_world(world, ntens=None, kind="p2p"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, ntens, kind)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    got = []
    while len(got) < world:
        try:
            got.append(q.get(timeout=5))
        except queue.Empty:
            assert all(p.exitcode in (None, 0) for p in procs), [p.exitcode for p in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


@pytest.mark.timeout(300)
@pytest.mark.parametrize("kind", ["p2p", "allgather"])
def test_prune_sharded_gloo_world2(kind):
    from oracle import oracle as O
    world = 2
    got = _run_world(world, kind=kind)
    ts = _tensors(None)
    refs = [O.prune_tensor(W.synth_numpy(s, seed, tid, e), "haar", 2, 61.8) for _, s, seed, tid, e in ts]
    mines = [g[3] for g in got]
    assert all(m == mines[0] for m in mines) and all(mines[0])  # both ranks own layers
    for rank, full, recs, _ in got:  # every rank holds the whole pruned state_dict
        for (ref, rr), f, r in zip(refs, full, recs):
            assert np.array_equal(f, ref)
            assert r["zero_count"] == rr["zero_count"] and r["eff_level"] == rr["eff_level"]
            assert np.float64(r["thr64"]).tobytes() == np.float64(rr["thr64"]).tobytes()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("kind", ["p2p", "allgather"])
def test_prune_sharded_gloo_more_ranks_than_tensors(kind):
    """world 3 over 2 tensors: one rank owns nothing, its region is empty and no zero-element
    point-to-point operation is posted for it (p2p; the padded all-gather carries its stride of
    padding); every rank still ends with the whole result"""
    from oracle import oracle as O
    got = _run_world(3, ntens=2, kind=kind)
    ts = _tensors(2)
    refs = [O.prune_tensor(W.synth_numpy(s, seed, tid, e), "haar", 2, 61.8) for _, s, seed, tid, e in ts]
    mines = got[0][3]
    assert sum(1 for m in mines if not m) == 1
    for rank, full, recs, _ in got:
        for (ref, rr), f, r in zip(refs, full, recs):
            assert np.array_equal(f, ref)
            assert r["zero_count"] == rr["zero_count"]
