"""GPU parity of the two forms of the level-0 selection: the one-launch resident kernel
(k_resident: weights held in registers across a grid barrier) and the three-launch form
(k_window / k_collect / k_mask_select).  Both must equal the C oracle bit for bit (values,
float64 threshold bits, zero counts) on the same inputs, including the fallbacks (window miss,
in place) and groups too large for the resident grid."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests import golden_io as G

pytestmark = pytest.mark.gpu

RES_CHUNK = 49152  # weights per resident workgroup (csrc/wtp_internal.h)


@pytest.fixture(scope="module")
def eng():
    from wavelettransforms_amd import engine
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    prev = engine.set_resident(True)
    yield engine
    engine.set_resident(prev)


@pytest.fixture(params=[True, False], ids=["resident", "three_launch"])
def mode(request, eng):
    prev = eng.set_resident(request.param)
    yield request.param
    eng.set_resident(prev)


def _dev(x):
    return torch.from_numpy(np.array(x, dtype=np.float32)).cuda()


def _same(o, ref, r, rr):
    assert np.array_equal(o, ref)
    assert r["zero_count"] == rr["zero_count"]
    assert G.f64_bits_equal(r["thr64"], rr["thr64"])
    assert r["eff_level"] == rr["eff_level"]


def test_capacity_covers_cfg2(eng):
    cap = eng.resident_capacity()
    assert cap >= 232, cap  # 256 CUs on MI355X; cfg2 needs 231 workgroups
    need = sum(-(-int(np.prod(s)) // RES_CHUNK) for _, s, *_ in G.W.resnet18_tensors(0))
    assert need <= cap


@pytest.mark.parametrize("pct", [0.0, 10.0, 50.0, 78.60000000000001, 100.0])
def test_cfg2_both_forms_equal_oracle(eng, mode, pct):
    ts = G.W.resnet18_tensors(0)
    xs = [eng.synth(s, seed, tid, e) for _, s, seed, tid, e in ts]
    outs, res = eng.prune(xs, "bior3.3", 5, pct, carry_level=False)
    for (name, s, seed, tid, e), o, r in zip(ts, outs, res):
        ref, rr = O.prune_tensor(G.W.synth_numpy(s, seed, tid, e), "bior3.3", 5, pct)
        _same(o.cpu().numpy(), ref, r, rr)
        if pct < 100.0:  # pct 100: the window is open above and its buckets overflow -> full scan (path 3)
            assert r["path"] in (1, 2), (name, r["path"])


def test_cfg2_in_place(eng, mode):
    ts = G.W.resnet18_tensors(0)
    xs = [eng.synth(s, seed, tid, e) for _, s, seed, tid, e in ts]
    refs = [O.prune_tensor(x.cpu().numpy(), "bior3.3", 5, 50.0) for x in xs]
    outs, res = eng.prune(xs, "bior3.3", 5, 50.0, outs=xs, carry_level=False)
    for x, o, r, (ref, rr) in zip(xs, outs, res, refs):
        assert o.data_ptr() == x.data_ptr()
        _same(o.cpu().numpy(), ref, r, rr)


def test_cfg2_in_place_full_scan_with_selectors(eng):
    """in place, pct 100 sends every shared segment down the full-scan path while its
    selector workgroup is in the grid.  The selector publishes the threshold before it counts the
    zeros over the segment's input, which the data workgroups are then overwriting; the count holds
    because where(|x| < thr, 0, x) maps every key below bits(thr) to +0 (still below) and leaves the
    rest -- this test pins that invariant against the oracle."""
    ts = G.W.resnet18_tensors(0)
    for pct in (100.0, 99.99999):
        xs = [eng.synth(s, seed, tid, e) for _, s, seed, tid, e in ts]
        refs = [O.prune_tensor(x.cpu().numpy(), "bior3.3", 5, pct) for x in xs]
        outs, res = eng.prune(xs, "bior3.3", 5, pct, outs=xs, carry_level=False)
        full = 0
        for (_, s, *_), x, o, r, (ref, rr) in zip(ts, xs, outs, res, refs):
            assert o.data_ptr() == x.data_ptr()
            _same(o.cpu().numpy(), ref, r, rr)
            full += r["path"] == 3 and int(np.prod(s)) > RES_CHUNK
        if pct == 100.0:
            assert full > 0


def _miss_input(n, seed):
    """Values whose sampled positions (SAMPLE_GROUP-float groups spread evenly) hold 1.0 while
    the rest are ~2.0: the sample window misses the true order statistics."""
    ng, grp = 4096 // 16, 16
    x = np.full(n, 2.0, np.float32)
    rng = np.random.default_rng(seed)
    x += rng.integers(0, 1 << 12, n).astype(np.float32) * np.float32(2.0 ** -20)
    for g in range(ng):
        s = int(g * ((n - grp) / (ng - 1)))
        x[s:s + grp] = 1.0
    x[::7] *= -1
    return x


@pytest.mark.parametrize("in_place", [False, True], ids=["out_of_place", "in_place"])
def test_window_miss_full_scan(eng, mode, in_place):
    n = 300_000
    x = _miss_input(n, 3)
    ref, rr = O.prune_tensor(x.reshape(300, 1000), "bior3.3", 0, 37.5)
    xt = _dev(x).reshape(300, 1000)
    outs, (r,) = eng.prune([xt], "bior3.3", 0, 37.5, outs=[xt] if in_place else None)
    assert r["path"] == 3
    _same(outs[0].cpu().numpy(), ref, r, rr)


@pytest.mark.parametrize("n", [1, 3, 4097, RES_CHUNK - 1, RES_CHUNK, RES_CHUNK + 5, 3 * RES_CHUNK + 4099])
def test_ragged_and_unaligned(eng, mode, n):
    rng = np.random.default_rng(n)
    x = (rng.standard_normal(n + 1) * 0.05).astype(np.float32)
    x[rng.integers(0, n, max(1, n // 50))] = 0.0
    base = _dev(x)
    aligned, unaligned = base[:n].clone(), base[1:n + 1]
    out_u = torch.empty(n + 1, dtype=torch.float32, device=base.device)[1:]
    outs, res = eng.prune([aligned, unaligned], "db8", 5, 38.2, outs=[torch.empty_like(aligned), out_u],
                          carry_level=False)
    for xin, o, r in zip((x[:n], x[1:n + 1]), outs, res):
        ref, rr = O.prune_tensor(xin.copy(), "db8", 5, 38.2)
        _same(o.cpu().numpy(), ref, r, rr)


def test_nan_and_inf(eng, mode):
    rng = np.random.default_rng(7)
    a = (rng.standard_normal(100_000) * 0.05).astype(np.float32)
    b = a.copy()
    a[123] = np.nan
    b[77] = np.inf
    b[99_000] = -np.inf
    outs, res = eng.prune([_dev(a), _dev(b)], "db8", 5, 50.0, carry_level=False)
    for xin, o, r in zip((a, b), outs, res):
        ref, rr = O.prune_tensor(xin.copy(), "db8", 5, 50.0)
        assert np.array_equal(o.cpu().numpy(), ref, equal_nan=True)
        assert r["zero_count"] == rr["zero_count"]


def test_ties_and_zeros(eng, mode):
    """Heavily tied keys (few distinct magnitudes, many exact zeros): counts and masks exact."""
    rng = np.random.default_rng(11)
    x = rng.integers(-3, 4, 600_000).astype(np.float32) * np.float32(0.25)
    for pct in (0.0, 23.599999999999998, 50.0, 61.8, 99.0):
        outs, (r,) = eng.prune([_dev(x)], "haar", 0, pct)
        ref, rr = O.prune_tensor(x.copy(), "haar", 0, pct)
        _same(outs[0].cpu().numpy(), ref, r, rr)


def test_more_segments_than_one_group(eng, mode):
    """30 level-0 tensors: two launch groups back to back (the parity regions alternate)."""
    shapes = [(64, 64, 3, 3), (128, 64, 1, 1), (256, 32, 3, 3)] * 10
    xs, refs = [], []
    for j, s in enumerate(shapes):
        e = G.W.sigma_exponent(G.W.conv_sigma(s))
        xs.append(eng.synth(s, 21, j, e))
        refs.append(O.prune_tensor(G.W.synth_numpy(s, 21, j, e), "bior3.3", 5, 61.8))
    outs, res = eng.prune(xs, "bior3.3", 5, 61.8, carry_level=False)
    for o, r, (ref, rr) in zip(outs, res, refs):
        _same(o.cpu().numpy(), ref, r, rr)


@pytest.mark.parametrize("in_place", [False, True], ids=["out_of_place", "in_place"])
def test_shared_segments_without_room_for_selectors(eng, in_place):
    """24 shared segments of 10 workgroups each: 240 chunks leave no room for the 24 selector
    workgroups beside them (one per CU), so every segment selects for itself (the local chain);
    beside the selector form on cfg2, the same results."""
    cap = eng.resident_capacity()
    n = 10 * RES_CHUNK - 3
    xs = [eng.synth((n,), 41, j, 27 + (j % 3)) for j in range(24)]
    if not (24 * 10 <= cap < 24 * 10 + 24):  # the case needs a 240..263-CU part (MI355X: 256)
        pytest.skip("resident capacity %d: no 240-chunk grid without room for 24 selectors" % cap)
    hosts = [x.cpu().numpy() for x in xs]
    outs, res = eng.prune(xs, "bior3.3", 5, 61.8, outs=xs if in_place else None, carry_level=False)
    for h, o, r in zip(hosts, outs, res):
        ref, rr = O.prune_tensor(h, "bior3.3", 5, 61.8)
        _same(o.cpu().numpy(), ref, r, rr)
        assert r["path"] in (1, 2)


def test_group_larger_than_resident_grid_falls_back(eng):
    """A level-0 group needing more workgroups than resident_capacity() runs the three-launch
    form (same results)."""
    cap = eng.resident_capacity()
    n = (cap + 8) * RES_CHUNK
    x = eng.synth((n,), 31, 0, 27)
    outs, (r,) = eng.prune([x], "haar", 0, 50.0)
    ref, rr = O.prune_tensor(x.cpu().numpy(), "haar", 0, 50.0)
    _same(outs[0].cpu().numpy(), ref, r, rr)


def test_alternating_forms_share_the_workspace(eng):
    """Resident and three-launch calls interleaved on one workspace: each leaves the parity
    regions clean for the other."""
    ts = G.W.resnet18_tensors(0)[:8]
    xs = [eng.synth(s, seed, tid, e) for _, s, seed, tid, e in ts]
    first, r0 = eng.prune(xs, "bior3.3", 5, 50.0, carry_level=False)
    for k in range(6):
        eng.set_resident(k % 2 == 0)
        outs, res = eng.prune(xs, "bior3.3", 5, 50.0, carry_level=False)
        for a, b, ra, rb in zip(first, outs, r0, res):
            assert torch.equal(a, b) and ra["zero_count"] == rb["zero_count"]
    eng.set_resident(True)


@pytest.fixture
def short_waits(eng):
    """Every wait of the resident launch bounded by 0 us: workgroups that find their segment's
    barrier incomplete on the first poll time out (wtp_set_resident_timeout_us)."""
    from wavelettransforms_amd import _native as N
    prev = N.lib().wtp_set_resident_timeout_us(0)
    yield
    N.lib().wtp_set_resident_timeout_us(prev)


def test_timeout_stores_nothing_in_place(eng, short_waits):
    """A resident launch whose waits time out must leave the caller's tensors untouched (in place:
    the input IS the output) and flag the tensors MODE_FAULT; the others are exact."""
    ts = G.W.resnet18_tensors(0)
    host = [G.W.synth_numpy(s, seed, tid, e) for _, s, seed, tid, e in ts]
    xs = [_dev(x) for x in host]
    _, res = eng.launch(xs, "bior3.3", 5, 50.0, outs=xs, carry_level=False)
    torch.cuda.synchronize()
    bad = eng.fault_mask(res, len(xs))
    assert bad.any(), "a 0 us bound should fault the multi-workgroup segments"
    for i, (x, h) in enumerate(zip(xs, host)):
        if bad[i]:
            assert np.array_equal(x.cpu().numpy().view(np.uint32), h.view(np.uint32)), "faulted tensor %d modified" % i
        else:
            ref, _ = O.prune_tensor(h, "bior3.3", 5, 50.0)
            assert np.array_equal(x.cpu().numpy(), ref)


def test_timeout_retried_by_prune(eng, short_waits):
    """engine.prune re-runs the faulted tensors in the three-launch form: the results equal the
    oracle, in place and out of place, per layer and with the level carried over the list."""
    ts = G.W.resnet18_tensors(0)
    host = [G.W.synth_numpy(s, seed, tid, e) for _, s, seed, tid, e in ts]
    for inplace in (True, False):
        for carry in (False, True):
            xs = [_dev(x) for x in host]
            outs, recs = eng.prune(xs, "bior3.3", 5, 50.0, outs=xs if inplace else None, carry_level=carry)
            for h, o, r in zip(host, outs, recs):
                ref, rr = O.prune_tensor(h, "bior3.3", 5, 50.0)
                _same(o.cpu().numpy(), ref, r, rr)
                assert r["path"] != eng.MODE_FAULT


def test_workspace_per_stream(eng):
    """Calls on two streams at once use distinct workspaces (the selection state lives there)."""
    ts = G.W.resnet18_tensors(0)[:8]
    host = [G.W.synth_numpy(s, seed, tid, e) for _, s, seed, tid, e in ts]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    xa = [_dev(x) for x in host]
    xb = [_dev(-x) for x in host]
    torch.cuda.synchronize()
    got = {}
    for name, s, xs in (("a", s1, xa), ("b", s2, xb)):
        with torch.cuda.stream(s):
            got[name] = eng.launch(xs, "bior3.3", 5, 37.5, carry_level=False, stream=s)
    torch.cuda.synchronize()
    assert eng.workspace(xa[0].device, 256, s1).data_ptr() != eng.workspace(xa[0].device, 256, s2).data_ptr()
    for name, sign in (("a", 1.0), ("b", -1.0)):
        outs, res = got[name]
        for h, o, r in zip(host, outs, eng.decode(res, len(outs))):
            ref, rr = O.prune_tensor(sign * h, "bior3.3", 5, 37.5)
            _same(o.cpu().numpy(), ref, r, rr)


def _finish_with_retry(eng, xs, outs, res, wavelet, level, pct):
    """engine.prune's fault handling for a launch made elsewhere: the tensors whose resident launch
    timed out (nothing stored) are re-run once in the three-launch form; returns (records, faults)."""
    n = len(xs)
    bad = eng.fault_mask(res, n)
    recs = None
    if bad.any():
        idx = [i for i in range(n) if bad[i]]
        merged = res.clone().view(n, -1)
        _, r2 = eng.launch([xs[i] for i in idx], wavelet, level, pct, outs=[outs[i] for i in idx],
                           carry_level=False, no_resident=True)
        merged[idx] = r2.view(len(idx), -1)
        res = merged.view(-1)
    recs = eng.decode(res, n)
    return recs, int(bad.sum())


def test_two_full_calls_on_two_streams(eng):
    """two full cfg2 calls at once on two streams -- each a 240-workgroup
    k_resident launch of one workgroup per CU, together more than the chip's 256 CUs hold.  Whatever
    the hardware interleaves, both calls end bit-exact against the oracle, a tensor whose launch was
    not co-resident faults within the wait bound (2 ms) and is re-run, and the pair completes in
    well under the round-5 bound of 200 ms."""
    import time
    ts = G.W.resnet18_tensors(0)
    host = [G.W.synth_numpy(s, seed, tid, e) for _, s, seed, tid, e in ts]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    xa = [_dev(x) for x in host]
    xb = [_dev(-x) for x in host]
    for s, xs in ((s1, xa), (s2, xb)):  # workspaces exist before the timed pair
        with torch.cuda.stream(s):
            eng.launch(xs, "bior3.3", 5, 50.0, carry_level=False, stream=s)
    torch.cuda.synchronize()
    worst, faults = 0.0, 0
    for rep in range(5):
        t0 = time.perf_counter()
        got = {}
        for name, s, xs in (("a", s1, xa), ("b", s2, xb)):
            with torch.cuda.stream(s):
                got[name] = eng.launch(xs, "bior3.3", 5, 50.0, carry_level=False, stream=s)
        torch.cuda.synchronize()
        recs = {}
        for name, xs in (("a", xa), ("b", xb)):
            outs, res = got[name]
            recs[name], f = _finish_with_retry(eng, xs, outs, res, "bior3.3", 5, 50.0)
            faults += f
        torch.cuda.synchronize()
        worst = max(worst, time.perf_counter() - t0)
        if rep == 0 or rep == 4:
            for name, sign in (("a", 1.0), ("b", -1.0)):
                outs = got[name][0]
                for h, o, r in zip(host, outs, recs[name]):
                    ref, rr = O.prune_tensor(sign * h, "bior3.3", 5, 50.0)
                    _same(o.cpu().numpy(), ref, r, rr)
    print("two concurrent cfg2 calls: worst pair %.2f ms, %d faulted tensors over 5 pairs" % (worst * 1e3, faults))
    assert worst < 0.05, worst


def test_resident_beside_long_kernels(eng):
    """a cfg2 call on one stream while another stream runs ~5 ms of grid-filling
    elementwise kernels (2 GiB in place, 8 passes): bit-exact against the oracle, and the call ends
    within the wait bound plus a re-run of the call (events on its own stream)."""
    ts = G.W.resnet18_tensors(0)
    host = [G.W.synth_numpy(s, seed, tid, e) for _, s, seed, tid, e in ts]
    xs = [_dev(x) for x in host]
    big = torch.ones(512 << 20, dtype=torch.float32, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(s2):
        eng.launch(xs, "bior3.3", 5, 50.0, carry_level=False, stream=s2)
    torch.cuda.synchronize()
    worst, faults = 0.0, 0
    for rep in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s1):
            for _ in range(8):
                big.mul_(1.0)
        with torch.cuda.stream(s2):
            torch.cuda._sleep(200_000)  # let the other stream's kernels take the CUs first
            a.record(s2)
            outs, res = eng.launch(xs, "bior3.3", 5, 50.0, carry_level=False, stream=s2)
            b.record(s2)
        torch.cuda.synchronize()
        recs, f = _finish_with_retry(eng, xs, outs, res, "bior3.3", 5, 50.0)
        faults += f
        worst = max(worst, a.elapsed_time(b))
        for h, o, r in zip(host, outs, recs):
            ref, rr = O.prune_tensor(h, "bior3.3", 5, 50.0)
            _same(o.cpu().numpy(), ref, r, rr)
    print("cfg2 beside 8 x 2 GiB elementwise passes: worst call %.3f ms, %d faulted tensors" % (worst, faults))
    assert worst < 50.0, worst


def test_outs_validated(eng):
    x = eng.synth((64, 64, 3, 3), 1, 1, 26)
    with pytest.raises(ValueError):
        eng.launch([x], "bior3.3", 5, 50.0, outs=[torch.empty(64, 64, 3, 6, device="cuda")[..., ::2]])
    with pytest.raises(ValueError):
        eng.launch([x], "bior3.3", 5, 50.0, outs=[torch.empty(10, device="cuda")])
    with pytest.raises(TypeError):
        eng.launch([x], "bior3.3", 5, 50.0, outs=[torch.empty(64, 64, 3, 3, device="cuda", dtype=torch.float64)])


def _halves_input(n, seed, scale_b):
    """The second half of every 2048-element run (the float4 slots of waves 4-7 of a resident
    workgroup) drawn from a distribution scaled by scale_b: the chunk's waves see different local
    distributions."""
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(n) * 0.05).astype(np.float32)
    x[(np.arange(n) % 2048) >= 1024] *= np.float32(scale_b)
    return x


@pytest.mark.parametrize("pct", [10.0, 50.0, 90.0])
@pytest.mark.parametrize("in_place", [False, True], ids=["out_of_place", "in_place"])
def test_structured_halves(eng, mode, pct, in_place):
    n = 600_000
    x = _halves_input(n, 5, 1.06)
    ref, rr = O.prune_tensor(x.reshape(600, 1000), "bior3.3", 0, pct)
    xt = _dev(x).reshape(600, 1000)
    outs, (r,) = eng.prune([xt], "bior3.3", 0, pct, outs=[xt] if in_place else None)
    assert r["path"] in (1, 2), r["path"]
    _same(outs[0].cpu().numpy(), ref, r, rr)


def test_nan_and_inf_in_either_half(eng, mode):
    """NaN / inf in the first or the second half of a 2048-element run (loaded by different waves
    of a resident workgroup), and past the first chunk."""
    rng = np.random.default_rng(9)
    base = (rng.standard_normal(200_000) * 0.05).astype(np.float32)
    cases = []
    for pos in (1500, 50_000 + 2047, 700):  # B, B, A half
        a = base.copy()
        a[pos] = np.nan
        b = base.copy()
        b[pos] = -np.inf
        cases += [a, b]
    outs, res = eng.prune([_dev(c) for c in cases], "db8", 5, 61.8, carry_level=False)
    for xin, o, r in zip(cases, outs, res):
        ref, rr = O.prune_tensor(xin.copy(), "db8", 5, 61.8)
        assert np.array_equal(o.cpu().numpy(), ref, equal_nan=True)
        assert r["zero_count"] == rr["zero_count"]
        assert G.f64_bits_equal(r["thr64"], rr["thr64"]) or (np.isnan(r["thr64"]) and np.isnan(rr["thr64"]))


@pytest.mark.parametrize("n", [4000, 40_000, RES_CHUNK])
def test_solo_overflow_then_reuse(eng, n):
    """A one-workgroup segment whose staging columns overflow (a zero-heavy / constant tensor:
    every key inside the window) takes the full scan; the parity flip of that launch must leave
    the workspace clean, so the calls after it on the same workspace stay exact."""
    rng = np.random.default_rng(n)
    z = np.zeros(n, np.float32)
    z[rng.integers(0, n, n // 20)] = (rng.standard_normal(n // 20) * 0.05).astype(np.float32)
    c = np.full(n, -0.125, np.float32)
    normal = (rng.standard_normal(300_000) * 0.05).astype(np.float32)
    for _ in range(3):
        for x in (z, c, normal, z):
            outs, (r,) = eng.prune([_dev(x)], "haar", 0, 50.0)
            ref, rr = O.prune_tensor(x.copy(), "haar", 0, 50.0)
            _same(outs[0].cpu().numpy(), ref, r, rr)
            assert r["path"] != eng.MODE_FAULT


@pytest.mark.parametrize("ties", [3, 20, 60])
def test_slot_overflow_paths(eng, mode, ties):
    """k_resident's published bucket slots hold 14 keys in the granules every reader fetches, 30 in
    all: `ties` copies of the segment's median value inside ONE workgroup's chunk put that many
    keys into one slot of the ranks' bucket -- 3 fit the first granules, 20 take the second round
    trip, 60 overflow the slot (full scan).  Exact either way, and the next call on the workspace
    too."""
    n = 4 * RES_CHUNK
    rng = np.random.default_rng(ties)
    x = (rng.standard_normal(n) * 0.05).astype(np.float32)
    pos = RES_CHUNK + 100 + np.arange(ties)
    rest = np.delete(np.abs(x), pos)
    v = np.float32(np.sort(rest)[len(rest) // 2])
    x[pos] = v * np.where(rng.random(ties) < 0.5, -1, 1).astype(np.float32)
    for pct in (50.0, 49.99):
        outs, (r,) = eng.prune([_dev(x)], "haar", 0, pct)
        ref, rr = O.prune_tensor(x.copy(), "haar", 0, pct)
        _same(outs[0].cpu().numpy(), ref, r, rr)
        assert r["path"] != eng.MODE_FAULT
    y = (rng.standard_normal(n) * 0.05).astype(np.float32)
    outs, (r,) = eng.prune([_dev(y)], "haar", 0, 50.0)
    ref, rr = O.prune_tensor(y.copy(), "haar", 0, 50.0)
    _same(outs[0].cpu().numpy(), ref, r, rr)
