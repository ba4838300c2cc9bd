"""cfg4 on the GPU (the reference's per-layer loop dwt_pruning.py:158-164 spread
over ranks): prune_sharded with the HIP path, in one process over a world-1 "nccl" (RCCL) group,
and the per-rank compute of the world-2/4/8 LPT plans run one after another and assembled exactly
as the all-gather lays them out -- every pruned tensor and record against the C oracle, bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from oracle import oracle as O
from wavelettransforms_amd import workloads as W
from wavelettransforms_amd.sharding import ShardPlan, assemble, prune_sharded, shard_local

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
    """Every rank's slice of the world-N plan computed on this GPU, stacked as
    all_gather_into_tensor stacks them, then unpacked by the same code prune_sharded uses."""
    host, dev = model
    plan = ShardPlan([x.shape for x in host], world)
    gathered = torch.stack([shard_local(dev, "bior3.3", 5, 50.0, plan, r) for r in range(world)])
    full, recs = assemble(gathered, plan)
    _check(full, recs, _refs(host, "bior3.3", 5, 50.0))
    if world == 8:
        assert plan.max_shard == 2_359_296
