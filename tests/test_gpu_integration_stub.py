"""The C-ABI entries exactly as INTEGRATION.md section 2 documents them, with real work on the GPU
(include/wtprune.h:91-101; the reference call sites main_pruning.py:54 and dwt_pruning.py:35-95):
`prune_layers` (wtp_workspace_init + wtp_prune_layers_f32, in place) over cfg2, and
`multi_resolution_analysis` (wtp_prune_f32, the level carried over the list) over DWT tensors --
both against the C oracle bit for bit."""
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests import golden_io as G

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def stub():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    cwd = os.getcwd()
    os.chdir(ROOT)  # the documented binding loads the library by its in-tree relative path
    try:
        from tests import integration_stub
    finally:
        os.chdir(cwd)
    return integration_stub


def test_prune_layers_cfg2_in_place(stub):
    ts = G.W.resnet18_tensors(0)
    xs = [torch.from_numpy(G.W.synth_numpy(s, seed, tid, e)).cuda() for _, s, seed, tid, e in ts]
    ptrs = [x.data_ptr() for x in xs]
    refs = [O.prune_tensor(x.cpu().numpy(), "bior3.3", 5, 50.0) for x in xs]
    for _ in range(2):  # the second call re-initialises a fresh workspace, as the stub does per call
        ys = [x.clone() for x in xs]
        tup = stub.prune_layers(ys, "bior3.3", 5, 50.0)
        torch.cuda.synchronize()
        for y, (ref, rr), (numel, nonzero, zeros) in zip(ys, refs, tup):
            assert np.array_equal(y.cpu().numpy(), ref)
            assert zeros == rr["zero_count"] and numel == y.numel() and nonzero == numel - zeros
    assert [x.data_ptr() for x in xs] == ptrs


def test_multi_resolution_analysis_carries_level(stub):
    """wtp_prune_f32: a 64x64 image first (db4 level 4 allowed), then a 3x3 conv (clamps to 0), then
    a 32x32 image that inherits level 0 from the clamp, exactly as dwt_pruning.py:64-65 carries it."""
    rng = np.random.default_rng(5)
    shapes = [(2, 64, 64), (16, 8, 3, 3), (32, 32), (4, 3, 40, 24)]
    xs_np = [(rng.standard_normal(s) * 0.05).astype(np.float32) for s in shapes]
    xs = [torch.from_numpy(x).cuda() for x in xs_np]
    recs = stub.multi_resolution_analysis(xs, "db4", 4, 61.8)
    lvl, F = 4, O.dec_len("db4")
    for x, y, r in zip(xs_np, xs, recs):
        lvl = min(lvl, O.dwt_max_level(min(x.shape[-2], x.shape[-1]), F))
        ref, rr = O.prune_tensor(x.copy(), "db4", lvl, 61.8)
        assert np.array_equal(y.cpu().numpy(), ref)
        assert r.eff_level == rr["eff_level"] == lvl
        assert r.zero_count == rr["zero_count"]
        assert G.f64_bits_equal(r.thr64, rr["thr64"])
