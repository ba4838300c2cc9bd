"""The one-launch small path (csrc/small.hip, k_small) on the GPU: calls whose tensors are all 2-D
transforms with a small population run pywt.wavedec2 -> np.percentile -> np.where -> pywt.waverec2
(ResNet/dwt_pruning.py:67-88) as ONE launch.  Every case is checked bit for bit against the C
oracle and against the multi-launch form of the same call (WTP_NO_RESIDENT), across filter lengths
(the specialised ones and the generic kernel), levels, odd extents (non-tight packing, the
odd-length repeat of periodization), batch dimensions, percentiles and degenerate data, plus the
timeout path (nothing stored, the call re-run in the multi-launch form)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests import golden_io as G
from wavelettransforms_amd import _native as N
from wavelettransforms_amd import engine as eng

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"


def _dev(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).cuda()


def _same(out, ref, r, rr):
    assert np.array_equal(out, ref, equal_nan=True)
    assert r["zero_count"] == rr["zero_count"] and r["eff_level"] == rr["eff_level"]
    assert G.f64_bits_equal(r["thr64"], rr["thr64"]) or (np.isnan(r["thr64"]) and np.isnan(rr["thr64"]))
    assert r["coeff_numel"] == rr["coeff_numel"]


def _both(xs, wavelet, level, pct, carry=False):
    """the call as k_small, and again in the multi-launch form: outputs and records identical"""
    outs, res = eng.prune(xs, wavelet, level, pct, carry_level=carry)
    o2, r2 = eng.launch(xs, wavelet, level, pct, carry_level=carry, no_resident=True)
    r2 = eng.decode(r2, len(xs))
    for a, b, ra, rb in zip(outs, o2, res, r2):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32)) or np.array_equal(
            a.cpu().numpy(), b.cpu().numpy(), equal_nan=True)
        assert ra["zero_count"] == rb["zero_count"] and ra["thr32_bits"] == rb["thr32_bits"]
    return outs, res


# F = 2, 4, 6, 8, 10, 12, 16, 18 take specialised kernels; db7 (14) and db10 (20) the generic one
WAVELETS = ["haar", "db2", "rbio2.2", "bior3.3", "db5", "coif2", "db8", "db9", "db7", "db10"]
SHAPES = [(128, 784), (10, 128), (64, 64), (2, 200), (1, 1, 97, 130), (2, 3, 31, 64), (1, 2, 77, 512), (300, 300),
          (4, 1, 33, 33), (96, 40)]


@pytest.mark.parametrize("wavelet", WAVELETS)
def test_small_path_equals_oracle(wavelet):
    """Every case equals the oracle in either form; a deep level whose tile windows outgrow the
    LDS arena keeps the multi-launch form, the rest take the one-launch path."""
    paths = []
    for j, shp in enumerate(SHAPES):
        e = G.W.sigma_exponent((2.0 / (shp[-1] * shp[-2])) ** 0.5)
        host = G.W.synth_numpy(shp, 21, j, e)
        for level, pct in [(5, 37.5), (1, 50.0), (2, 90.0)]:
            ref, rr = O.prune_tensor(host, wavelet, level, pct)
            if rr["eff_level"] < 1:
                continue
            outs, (r,) = _both([_dev(host)], wavelet, level, pct)
            paths.append(r["path"])
            _same(outs[0].cpu().numpy(), ref, r, rr)
    assert paths.count(eng.MODE_SMALL) >= len(paths) // 2, paths


@pytest.mark.parametrize("pct", [0.0, 0.5, 50.0, 99.99, 100.0])
def test_cfg3_percentiles(pct):
    ts = G.W.mlp_tensors(3)
    host = [G.W.synth_numpy(s, seed, tid, e) for _, s, seed, tid, e in ts]
    outs, res = _both([_dev(h) for h in host], "rbio2.2", 3, pct)
    for h, o, r in zip(host, outs, res):
        ref, rr = O.prune_tensor(h, "rbio2.2", 3, pct)
        assert r["path"] == eng.MODE_SMALL
        _same(o.cpu().numpy(), ref, r, rr)


def test_multi_tensor_carry_and_mixed_levels():
    shapes = [(64, 96), (10, 128), (34, 50), (3, 8, 8)]  # SM_MAX_SEG tensors
    host = [G.W.synth_numpy(s, 5, j, 24) for j, s in enumerate(shapes)]
    outs, res = _both([_dev(h) for h in host], "db2", 4, 61.8, carry=True)
    lvl = 4
    for h, o, r in zip(host, outs, res):
        ref, rr = O.prune_tensor(h, "db2", lvl, 61.8)
        lvl = min(lvl, rr["eff_level"])
        assert r["path"] == eng.MODE_SMALL
        _same(o.cpu().numpy(), ref, r, rr)


@pytest.mark.parametrize("kind", ["constant", "zeros", "ties", "nan", "tiny", "huge"])
def test_degenerate_data(kind):
    rng = np.random.default_rng(7)
    x = rng.standard_normal((64, 96)).astype(np.float32)
    if kind == "constant":
        x[:] = 0.75
    elif kind == "zeros":
        x[:] = 0.0
    elif kind == "ties":
        x = np.round(x * 2.0).astype(np.float32) / 2.0
    elif kind == "nan":
        x[5, 7] = np.nan
    elif kind == "tiny":
        x *= np.float32(1e-39)  # subnormal coefficients
    elif kind == "huge":
        x *= np.float32(1e37)
    for wavelet, pct in [("haar", 50.0), ("bior3.3", 37.5), ("db8", 12.5)]:
        ref, rr = O.prune_tensor(x, wavelet, 3, pct)
        outs, (r,) = _both([_dev(x)], wavelet, 3, pct)
        assert r["path"] == eng.MODE_SMALL
        _same(outs[0].cpu().numpy(), ref, r, rr)


@pytest.mark.parametrize("split", ["columns", "rows", "one_tile"])
def test_tile_local_distributions_differ(split):
    """Tiles whose local |c| distributions sit far from the segment's: most workgroups hold no
    key of the ranks' bin (empty slots after barrier 0) and a few hold nearly all of it, up to
    the slot capacity (more: the digit-pass fallback over P behind two more barriers) -- results
    still equal the oracle and the multi-launch form."""
    host = G.W.synth_numpy((128, 784), 11, 0, 26)
    if split == "columns":
        host[:, : host.shape[1] // 2] *= np.float32(1e3)
    elif split == "rows":
        host[host.shape[0] // 3:] *= np.float32(1e-3)
    else:
        host[:16, :64] *= np.float32(1e4)
    for pct in (50.0, 10.0, 90.0):
        ref, rr = O.prune_tensor(host, "rbio2.2", 3, pct)
        outs, (r,) = _both([_dev(host)], "rbio2.2", 3, pct)
        assert r["path"] == eng.MODE_SMALL
        _same(outs[0].cpu().numpy(), ref, r, rr)


def test_in_place():
    host = G.W.synth_numpy((128, 784), 3, 0, 26)
    xt = _dev(host)
    outs, (r,) = eng.prune([xt], "rbio2.2", 3, 50.0, outs=[xt])
    ref, rr = O.prune_tensor(host, "rbio2.2", 3, 50.0)
    assert r["path"] == eng.MODE_SMALL
    _same(xt.cpu().numpy(), ref, r, rr)


def test_timeout_stores_nothing_then_retried():
    """A zero wait bound: every multi-workgroup segment poisons its first barrier -- nothing is
    stored (the in-place input is intact), the records read WTP_PATH_FAULT, and prune() re-runs
    those tensors in the multi-launch form."""
    L = N.lib()
    ts = G.W.mlp_tensors(3)
    host = [G.W.synth_numpy(s, seed, tid, e) for _, s, seed, tid, e in ts]
    prev = L.wtp_set_resident_timeout_us(0)
    try:
        seen = 0
        for _ in range(50):  # a fault needs an early workgroup to find its barrier incomplete
            xs = [_dev(h) for h in host]
            _, resd = eng.launch(xs, "rbio2.2", 3, 50.0, outs=xs, carry_level=False)
            torch.cuda.synchronize()
            faulted = eng.fault_mask(resd, len(xs))
            for i in range(len(xs)):
                if faulted[i]:  # all or nothing: a faulted tensor's in-place input is intact
                    assert np.array_equal(xs[i].cpu().numpy(), host[i])
                    seen += 1
            if faulted[0]:
                break
        assert seen, "no launch faulted at a zero wait bound"
        xs = [_dev(h) for h in host]
        outs, res = eng.prune(xs, "rbio2.2", 3, 50.0, outs=xs, carry_level=False)
    finally:
        L.wtp_set_resident_timeout_us(prev)
    for h, o, r in zip(host, outs, res):
        ref, rr = O.prune_tensor(h, "rbio2.2", 3, 50.0)
        assert r["path"] != eng.MODE_FAULT
        _same(o.cpu().numpy(), ref, r, rr)


def test_ineligible_calls_keep_the_multi_launch_form():
    """a level-0 tensor in the call (here a 3x3 kernel at bior3.3), a 1-D tensor, or a population
    over the bound: the whole call takes the multi-launch form"""
    for shapes, wavelet in [([(64, 96), (8, 8, 3, 3)], "bior3.3"), ([(64, 96), (100,)], "haar"),
                            ([(1024, 1100)], "haar")]:
        host = [G.W.synth_numpy(s, 9, j, 24) for j, s in enumerate(shapes)]
        outs, res = eng.prune([_dev(h) for h in host], wavelet, 3, 50.0, carry_level=False)
        for h, o, r in zip(host, outs, res):
            ref, rr = O.prune_tensor(h, wavelet, 3, 50.0)
            assert r["path"] != eng.MODE_SMALL
            _same(o.cpu().numpy(), ref, r, rr)
