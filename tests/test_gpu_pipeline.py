"""GPU parity of the pipelined form of a multi-group call (include/wtprune.h wtp_set_pipeline):
with more than one launch group (24 tensors) of wavelet-transformed tensors, each group's
selection runs on the library's side stream while the caller's stream runs the next group's
forward levels (mode 1; round 5's lane-stream mode 2 was removed in round 6).  The results must equal
the single-stream form and the C oracle bit for bit (values, float64 threshold bits, zero counts),
eagerly and inside a captured HIP graph, on the caller's default and non-default streams; a
level-0 tensor mixed into a group is covered too."""
import warnings

import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests import golden_io as G

pytestmark = pytest.mark.gpu

# 3 launch groups of 24 / 24 / 3 tensors; mixed geometries, one level-0 tensor (1x1 kernel)
SHAPES = [(2, 3, 64, 64), (1, 1, 130, 97), (3, 2, 33, 40), (1, 4, 128, 128)] * 12 + [(16, 8, 1, 1), (2, 2, 96, 80),
                                                                                     (1, 1, 200, 64)]


@pytest.fixture(scope="module")
def eng():
    from wavelettransforms_amd import engine
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    prev = engine.set_pipeline(True)
    yield engine
    engine.set_pipeline(prev)


def _inputs(eng):
    return [eng.synth(s, 7, i, 6 + (i % 5)) for i, s in enumerate(SHAPES)]


def _run(eng, xs, pipeline, wavelet="db8", level=3, pct=60.0, stream=None):
    prev = eng.set_pipeline(pipeline)
    try:
        outs, resd = eng.launch(xs, wavelet, level, pct, carry_level=False, stream=stream)
        torch.cuda.synchronize()
        return [o.cpu().numpy() for o in outs], eng.decode(resd, len(xs))
    finally:
        eng.set_pipeline(prev)


def _equal(a, b):
    (oa, ra), (ob, rb) = a, b
    for x, y, p, q in zip(oa, ob, ra, rb):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32))
        # path is a diagnostic: the window form a group takes (inline sample or k_window) depends on
        # the group's size, so it may differ with the grouping; the results may not
        assert p["zero_count"] == q["zero_count"] and p["eff_level"] == q["eff_level"]
        assert G.f64_bits_equal(p["thr64"], q["thr64"])


@pytest.mark.parametrize("mode", [1])
@pytest.mark.parametrize("wavelet,level,pct", [("db8", 3, 60.0), ("bior3.3", 5, 50.0), ("haar", 2, 0.0)])
def test_pipelined_equals_single_stream_and_oracle(eng, wavelet, level, pct, mode):
    xs = _inputs(eng)
    a = _run(eng, xs, mode, wavelet, level, pct)
    b = _run(eng, xs, 0, wavelet, level, pct)
    _equal(a, b)
    for i in (0, 1, 25, 48, 50):  # every group, the level-0 tensor, the odd shapes
        ref, rr = O.prune_tensor(G.W.synth_numpy(SHAPES[i], 7, i, 6 + (i % 5)), wavelet, level, pct)
        assert np.array_equal(a[0][i], ref)
        assert a[1][i]["zero_count"] == rr["zero_count"]
        assert G.f64_bits_equal(a[1][i]["thr64"], rr["thr64"])


@pytest.mark.parametrize("mode", [1])
def test_pipelined_on_a_side_stream_of_the_caller(eng, mode):
    xs = _inputs(eng)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        a = _run(eng, xs, mode, stream=s)
    _equal(a, _run(eng, xs, 0))


@pytest.mark.parametrize("mode", [1])
def test_pipelined_graph_capture_and_replay(eng, mode):
    """The side stream forks from and joins the captured stream: the graph replays
    the call; several calls in one capture, as bench.py captures its steps."""
    xs = _inputs(eng)
    ref = _run(eng, xs, 0)
    prev = eng.set_pipeline(mode)
    try:
        outs = [torch.empty_like(x) for x in xs]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):  # warm-up: workspace and side stream created outside the capture
            eng.launch(xs, "db8", 3, 60.0, outs=outs, carry_level=False, stream=s)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        # captured on the warmed stream (its workspace exists: no zero-fill is captured)
        with warnings.catch_warnings():
            warnings.simplefilter("error")
            with torch.cuda.graph(g, stream=s):
                for _ in range(3):
                    _, resd = eng.launch(xs, "db8", 3, 60.0, outs=outs, carry_level=False)
        for o in outs:
            o.zero_()
        g.replay()
        g.replay()
        torch.cuda.synchronize()
        _equal(([o.cpu().numpy() for o in outs], eng.decode(resd, len(xs))), ref)
    finally:
        eng.set_pipeline(prev)
