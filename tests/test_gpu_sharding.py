"""cfg4 on the GPU (the reference's per-layer loop dwt_pruning.py:158-164 spread
over ranks): prune_sharded with the HIP path, in one process over a world-1 "nccl" (RCCL) group,
and the per-rank compute of the world-2/4/8 LPT plans run one after another and assembled exactly
as the exchange lays them out -- every pruned tensor and record against the C oracle, bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from oracle import oracle as O
from wavelettransforms_amd import workloads as W
from wavelettransforms_amd.sharding import REC_BYTES, ShardPlan, _Shard, assemble, prune_sharded, shard_local

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def model():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    ts = W.resnet18_tensors(0)
    host = [W.synth_numpy(s, seed, tid, e) for _, s, seed, tid, e in ts]
    dev = [torch.from_numpy(x).cuda() for x in host]
    return host, dev


def _refs(host, wavelet, level, pct):
    return [O.prune_tensor(x, wavelet, level, pct) for x in host]


def _check(full, recs, refs):
    for f, r, (ro, rr) in zip(full, recs, refs):
        assert np.array_equal(f.cpu().numpy(), ro)
        assert r["zero_count"] == rr["zero_count"] and r["eff_level"] == rr["eff_level"]
        assert np.float64(r["thr64"]).tobytes() == np.float64(rr["thr64"]).tobytes()
        assert r["numel"] == rr["numel"] and r["path"] != 99


@pytest.mark.parametrize("wavelet,level,pct", [("bior3.3", 5, 50.0), ("haar", 5, 61.8)])
def test_prune_sharded_world1_rccl(model, wavelet, level, pct):
    host, dev = model
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        full, recs, plan = prune_sharded(dev, wavelet, level, pct)
        torch.cuda.synchronize()
        assert plan.world == 1
        _check(full, recs, _refs(host, wavelet, level, pct))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_lpt_plans_assembled(model, world):
    """Every rank's region of the world-N plan computed on this GPU into the flat buffer, where the
    exchange leaves them, then unpacked by the same code prune_sharded uses."""
    host, dev = model
    plan = ShardPlan([x.shape for x in host], world)
    # each rank's region written in place, as the exchange leaves them side by side
    full_buf = torch.full((plan.total,), float("nan"), dtype=torch.float32, device="cuda")
    for r in range(world):
        shard_local(dev, "bior3.3", 5, 50.0, plan, r, full=full_buf)
    full, recs = assemble(full_buf, plan)
    _check(full, recs, _refs(host, "bior3.3", 5, 50.0))
    # unpadded: every rank receives exactly the other ranks' weights + records
    n_w = sum(plan.numels)
    for r in range(world):
        assert plan.bytes_received(r) <= 4 * (n_w - plan.loads[r]) + 4 * 3 * world + REC_BYTES * len(host)
    if world == 8:
        assert plan.max_shard == 2_359_296
        assert max(plan.bytes_received(r) for r in range(world)) <= 44_667_648 + REC_BYTES * len(host) + 4 * 3 * 8


def test_sharded_fault_recovery_world1(model):
    """a resident launch forced to time out (bound 0 us) inside prune_sharded -- every
    record faults, the owner re-runs those tensors in the three-launch form, and the result is the
    oracle's bit for bit (records included, no path 99 left)."""
    from wavelettransforms_amd import _native as N
    host, dev = model
    L = N.lib()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    prev = L.wtp_set_resident_timeout_us(0)
    try:
        full, recs, plan = prune_sharded(dev, "bior3.3", 5, 50.0)
        torch.cuda.synchronize()
    finally:
        L.wtp_set_resident_timeout_us(prev)
        dist.destroy_process_group()
    _check(full, recs, _refs(host, "bior3.3", 5, 50.0))
    # the shard_local + assemble flow under the same forced timeout, out of place and in place (the
    # inputs are the buffer's own views): a faulted record is visible (path 99, nothing stored: the
    # input bytes are intact), and re-running the faulted tensors restores exact results
    plan = ShardPlan([x.shape for x in host], 2)
    for in_place in (False, True):
        full_buf = torch.zeros(plan.total, dtype=torch.float32, device="cuda")
        if in_place:
            ins = []
            for i, x in enumerate(dev):
                b = plan.base[plan.owner[i]] + plan.offset[i]
                v = full_buf[b:b + plan.numels[i]].view(x.shape)
                v.copy_(x)
                ins.append(v)
        else:
            ins = dev
        prev = L.wtp_set_resident_timeout_us(0)
        try:
            for r in range(2):
                shard_local(ins, "bior3.3", 5, 50.0, plan, r, full=full_buf)
            torch.cuda.synchronize()
        finally:
            L.wtp_set_resident_timeout_us(prev)
        _, recs0 = assemble(full_buf, plan)
        bad = [i for i, r in enumerate(recs0) if r["path"] == 99]
        for i in bad:
            b = plan.base[plan.owner[i]] + plan.offset[i]
            got = full_buf[b:b + plan.numels[i]].cpu().numpy()
            want = host[i].reshape(-1) if in_place else np.zeros_like(got)
            assert np.array_equal(got, want)  # nothing stored for a faulted tensor
        for r in range(2):
            sh = _Shard(ins, plan, r, torch.device("cuda"), full_buf)
            redo = [i for i in bad if plan.owner[i] == r]
            if redo:
                sh.run(redo, "bior3.3", 5, 50.0, no_resident=True)
        full, recs = assemble(full_buf, plan)
        _check(full, recs, _refs(host, "bior3.3", 5, 50.0))
