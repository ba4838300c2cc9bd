"""GPU parity: the HIP path (libwtprune.so through the C ABI) against the golden fixtures
(PyWavelets 1.1.1 + NumPy 1.26.4 running the reference's call sequence) and against the C
oracle on the same inputs.  Bar: bit-exact values (signed zeros compared by value), identical
thresholds (float64 bits), identical zero counts and coefficient-domain masks."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests import golden_io as G

pytestmark = pytest.mark.gpu

CASES = sorted(G.manifest()["cases"])


@pytest.fixture(scope="module")
def eng():
    from wavelettransforms_amd import engine
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return engine


def _dev(x):
    return torch.from_numpy(np.array(x, dtype=np.float32)).cuda()


def _f32_same(a_bits, b_bits):
    # NaN payload/sign differs between x86 (inf - inf = -nan) and the GPU (+nan); any NaN
    # threshold prunes nothing, so NaN == NaN here; everything else must match bit for bit
    a = np.array(a_bits, np.uint32).view(np.float32)
    b = np.array(b_bits, np.uint32).view(np.float32)
    return (np.isnan(a) and np.isnan(b)) or int(a_bits) == int(b_bits)


def _check(rec, out_np, r):
    assert r["eff_level"] == rec["eff_level"]
    assert G.f64_bits_equal(r["thr64"], rec["thr64"]), (r["thr64"], rec["thr64"])
    assert _f32_same(r["thr32_bits"], rec["thr32_bits"])
    assert _f32_same(r["max_abs_bits"], rec["max_abs_bits"])
    assert r["zero_count"] == rec["zero_count"]
    assert r["coeff_numel"] == rec["coeff_numel"]
    assert G.canon_hash(out_np) == rec["out_hash"]


def test_device_synth_matches_numpy(eng):
    for shape, seed, tid, e in [((64, 3, 7, 7), 0, 0, 30), ((4096, 4096), 5, 3, 29), ((1001,), 9, 2, 24)]:
        a = eng.synth(shape, seed, tid, e).cpu().numpy()
        b = G.W.synth_numpy(shape, seed, tid, e)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("name", CASES)
def test_golden_case(eng, name):
    rec = G.manifest()["cases"][name]
    x = G.case_input(name)
    xt = _dev(x)
    if "error" in rec:
        with pytest.raises((ValueError, IndexError, RuntimeError)) as ei:
            eng.prune([xt], rec["wavelet"], rec["level_in"], rec["pct"])
        assert ei.type.__name__ == rec["error"]
        return
    outs, (r,) = eng.prune([xt], rec["wavelet"], rec["level_in"], rec["pct"])
    out = outs[0].cpu().numpy()
    _check(rec, out, r)
    arrs = G.arrays()
    if name + "/out" in arrs:
        assert np.array_equal(out, arrs[name + "/out"], equal_nan=True)
    # coefficient-domain: the device forward transform + packing equals pywt's coeff_arr
    if x.ndim >= 2 and rec["eff_level"] > 0:
        P = eng.wavedec2_packed(xt, rec["wavelet"], rec["eff_level"]).cpu().numpy()
        assert G.canon_hash(P) == rec["coeff_hash"]
        mask = np.abs(P) < np.float32(r["thr32"])
        assert int(mask.sum()) == rec["mask_count"]
        assert G.mask_hash(mask) == rec["mask_hash"]


def test_multi_tensor_level_carry(eng):
    recs = G.manifest()["multi"]["haar_L5_p50"]
    arrs = G.arrays()
    xs = [_dev(arrs["multi/in%d" % j]) for j in range(len(recs))]
    outs, res = eng.prune(xs, "haar", 5, 50.0, carry_level=True)
    for j, (rec, r) in enumerate(zip(recs, res)):
        assert r["eff_level"] == rec["eff_level"]
        assert np.array_equal(outs[j].cpu().numpy(), arrs["multi/out%d" % j])


@pytest.mark.parametrize("cfg", ["cfg2_bior33_L5", "cfg2_haar_L5", "cfg3_rbio22_L3", "b1024_db8_L5",
                                 "cfg5_db8_L5_block0"])
def test_large_configs(eng, cfg):
    recs = G.manifest()["large"][cfg]
    # group records by percentile: one batched call per percentile over all tensors
    by_pct = {}
    for rec in recs:
        by_pct.setdefault(rec["pct"], []).append(rec)
    for pct, group in by_pct.items():
        xs = [eng.synth(tuple(r["shape"]), *r["synth"]) for r in group]
        outs, res = eng.prune(xs, group[0]["wavelet"], group[0]["level_in"], pct, carry_level=False)
        for rec, o, r in zip(group, outs, res):
            _check(rec, o.cpu().numpy(), r)


def test_batched_resnet18_equals_oracle_per_layer(eng):
    """cfg2 in one launch sequence == the oracle layer by layer, values bit for bit."""
    ts = G.W.resnet18_tensors(0)
    xs = [eng.synth(s, seed, tid, e) for _, s, seed, tid, e in ts]
    outs, res = eng.prune(xs, "bior3.3", 5, 50.0, carry_level=False)
    for (name, s, seed, tid, e), o, r in zip(ts, outs, res):
        ref, rr = O.prune_tensor(G.W.synth_numpy(s, seed, tid, e), "bior3.3", 5, 50.0)
        assert np.array_equal(o.cpu().numpy(), ref), name
        assert r["zero_count"] == rr["zero_count"] and G.f64_bits_equal(r["thr64"], rr["thr64"])


# odd 2-D shapes raise IndexError in the reference (the crop of dwt_pruning.py:79-82 is 4-D),
# so odd extents come with batch dims here
MIXED_SHAPES = [(64, 64), (3, 2, 40, 70), (1, 1, 97, 130), (2, 1, 33, 33), (2, 200), (128, 784), (10, 128),
                (5, 3, 7, 7), (64, 64, 3, 3), (256, 256), (1, 2, 77, 512), (2, 3, 31, 64), (1, 1, 513, 65),
                (64, 32), (300, 300)]


# every specialised filter length of the tiled filter bank (F = 2, 4, 6, 8, 10, 12, 16, 18, with
# H = F/2 odd and even: the packed synthesis-column blocks pair rows by the parity of H), the
# generic tiled kernels (db7: F = 14, coif4: F = 24) and the per-point kernels (dmey: F = 62)
@pytest.mark.parametrize("wavelet", ["haar", "db2", "rbio2.2", "bior3.3", "db5", "coif2", "db8", "db9", "db7",
                                     "coif4", "dmey"])
def test_grouped_levels_mixed_batch(eng, wavelet):
    """One call over 15 tensors of mixed sizes, batch dims and clamped levels: the same level of
    every tensor runs as one grouped filter-bank launch (more than FB_GROUP images, so the group
    splits), small levels on the per-point kernels; each tensor == the oracle bit for bit."""
    xs, refs = [], []
    for j, shp in enumerate(MIXED_SHAPES):
        e = G.W.sigma_exponent((2.0 / (shp[-1] * shp[-2])) ** 0.5)
        xs.append(eng.synth(shp, 11, j, e))
        refs.append(O.prune_tensor(G.W.synth_numpy(shp, 11, j, e), wavelet, 5, 37.5))
    outs, res = eng.prune(xs, wavelet, 5, 37.5, carry_level=False)
    for shp, o, r, (ref, rr) in zip(MIXED_SHAPES, outs, res, refs):
        assert np.array_equal(o.cpu().numpy(), ref), shp
        assert r["zero_count"] == rr["zero_count"] and r["eff_level"] == rr["eff_level"], shp
        assert G.f64_bits_equal(r["thr64"], rr["thr64"]), shp


def test_window_miss_falls_back_to_full_scan(eng):
    """Data whose sampled positions are unrepresentative: the sample window misses the true
    order statistics and k_select must fall back to the exact full radix select (path 3)."""
    n, ng, grp = 300_000, 32768 // 16, 16
    x = np.full(n, 2.0, np.float32)
    rng = np.random.default_rng(3)
    x += rng.integers(0, 1 << 12, n).astype(np.float32) * np.float32(2.0 ** -20)
    for g in range(ng):
        s = g * (n - grp) // (ng - 1)
        x[s:s + grp] = 1.0
    x[::7] *= -1
    outs, (r,) = eng.prune([_dev(x).reshape(300, 1000)], "bior3.3", 0, 37.5)   # level 0: raw values
    ref, rr = O.prune_tensor(x.reshape(300, 1000), "bior3.3", 0, 37.5)
    assert r["path"] == 3
    assert np.array_equal(outs[0].cpu().numpy(), ref)
    assert G.f64_bits_equal(r["thr64"], rr["thr64"]) and r["zero_count"] == rr["zero_count"]


def test_window_paths_and_extremes(eng):
    """Large level-0 populations at the percentile extremes (open windows) and mid-range."""
    x = eng.synth((512, 512, 3, 3), 4, 4, 27)
    xn = x.cpu().numpy()
    for pct in (0.0, 0.001, 12.5, 50.0, 99.999, 100.0):
        outs, (r,) = eng.prune([x], "db8", 5, pct)
        ref, rr = O.prune_tensor(xn, "db8", 5, pct)
        assert np.array_equal(outs[0].cpu().numpy(), ref), pct
        assert G.f64_bits_equal(r["thr64"], rr["thr64"]), pct


@pytest.mark.parametrize("n", [1, 2, 3, 5, 7, 4097, 16383, 16385, 2 * 16384 + 4099, 100_003])
def test_ragged_and_unaligned_level0(eng, n):
    """Level-0 populations of every length class (n % 4, partial last chunk), from 16-byte
    aligned and unaligned (offset by one float) device pointers, in one batched call."""
    rng = np.random.default_rng(n)
    x = (rng.standard_normal(n + 1) * 0.05).astype(np.float32)
    x[rng.integers(0, n, max(1, n // 50))] = 0.0
    base = _dev(x)
    aligned, unaligned = base[:n].clone(), base[1:n + 1]
    assert unaligned.data_ptr() % 16 != 0
    out_u = torch.empty(n + 1, dtype=torch.float32, device=base.device)[1:]
    outs, res = eng.prune([aligned, unaligned], "db8", 5, 38.2, outs=[torch.empty_like(aligned), out_u],
                          carry_level=False)
    for xin, o, r in zip((x[:n], x[1:n + 1]), outs, res):
        ref, rr = O.prune_tensor(xin.copy(), "db8", 5, 38.2)
        assert np.array_equal(o.cpu().numpy(), ref)
        assert r["zero_count"] == rr["zero_count"] and G.f64_bits_equal(r["thr64"], rr["thr64"])


def test_in_place_and_workspace_reuse(eng):
    ts = G.W.resnet18_tensors(0)[:6]
    xs = [eng.synth(s, seed, tid, e) for _, s, seed, tid, e in ts]
    first, r1 = eng.prune([x.clone() for x in xs], "haar", 2, 61.8, carry_level=False)
    # a different call in between must not leave state behind in the shared workspace
    eng.prune([eng.synth((1, 2, 130, 97), 1, 1, 25)], "db8", 3, 10.0)
    same = [x.clone() for x in xs]
    outs, r2 = eng.prune(same, "haar", 2, 61.8, outs=same, carry_level=False)  # in place
    for a, b, ra, rb in zip(first, outs, r1, r2):
        assert torch.equal(a, b) and ra["zero_count"] == rb["zero_count"]


def test_perfect_reconstruction_full_size(eng):
    """At the cfg5 block size: waverec2(wavedec2(x)) equals the oracle's round trip bit for bit
    (the oracle at percentile 0 prunes nothing, so its output IS waverec2(wavedec2(x))), the packed
    coefficients equal the oracle's, and the round trip is within PyWavelets' float32
    perfect-reconstruction tolerance of x (RMS < 6e-7 * max|x|, pywt/tests/test_perfect_reconstruction.py)."""
    e = G.W.sigma_exponent((2.0 / 4096) ** 0.5)
    x = eng.synth((4096, 4096), 5, 7, e)
    P = eng.wavedec2_packed(x, "db8", 5)
    y = eng.waverec2_packed(P, (4096, 4096), "db8", 5)
    host = G.W.synth_numpy((4096, 4096), 5, 7, e)
    ref, rr, coeffs = O.prune_tensor(host, "db8", 5, 0.0, want_coeffs=True)
    assert rr["zero_count"] == int((ref == 0).sum())
    assert np.array_equal(P.cpu().numpy().view(np.uint32), coeffs.view(np.uint32))
    assert np.array_equal(y.cpu().numpy(), ref)
    err = (y - x).float()
    rms = float(torch.sqrt(torch.mean(err * err)))
    assert rms < 6e-7 * float(x.abs().max())


def test_reference_api_mirror(eng):
    from wavelettransforms_amd import dwt_pruning as D
    x = G.case_input("stem_haar_L5_p50")
    rec = G.manifest()["cases"]["stem_haar_L5_p50"]
    outs, zc = D.multi_resolution_analysis([_dev(x)], "haar", 5, 50.0, verbose=False)
    assert zc == rec["zero_count"]
    assert G.canon_hash(outs[0].cpu().numpy()) == rec["out_hash"]
    # CPU tensors are accepted and returned on the CPU, like the reference
    outs_cpu, zc2 = D.multi_resolution_analysis([torch.from_numpy(x)], "haar", 5, 50.0, verbose=False)
    assert outs_cpu[0].device.type == "cpu" and zc2 == zc
    v = G.case_input("vec1000_p23.6")
    out_np = D.percentile_based_thresholding(v, 23.599999999999998)
    assert G.canon_hash(out_np) == G.manifest()["cases"]["vec1000_p23.6"]["out_hash"]
