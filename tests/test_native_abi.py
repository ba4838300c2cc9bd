"""CPU checks of the C-ABI library: it loads without a GPU, exports every symbol that
include/wtprune.h declares, and its host-side logic (wavelet table, max level, packed shape,
validation in the reference's order) matches the oracle / golden fixtures.  No kernel runs."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O
from tests import golden_io as G
from wavelettransforms_amd import _native as N


def test_library_exports_every_declared_symbol():
    L = N.lib()
    declared = N.exported_symbols()
    assert len(declared) >= 18
    for name in declared:
        assert hasattr(L, name), name


def test_wavelet_table_matches_oracle():
    L = N.lib()
    assert L.wtp_wavelet_count() == 106
    for wid in range(106):
        name = L.wtp_wavelet_name(wid).decode()
        assert O.wavelet_id(name) == wid
        assert L.wtp_dec_len(wid) == O.dec_len(name)
    assert L.wtp_wavelet_id(b"nosuchwavelet") == -1


def test_max_level_matches_pywt_table():
    z = np.load(G.GOLDEN + "/max_level.npz")
    L = N.lib()
    for i, F in enumerate(z["F"]):
        got = [L.wtp_max_level(n, int(F)) for n in range(z["table"].shape[0])]
        assert got == list(z["table"][:, i])


def test_packed_shape_matches_golden():
    L = N.lib()
    m = G.manifest()["cases"]
    for name, rec in m.items():
        if "error" in rec or len(rec["shape"]) < 2:
            continue
        pr, pc = ctypes.c_int64(), ctypes.c_int64()
        H, W = rec["shape"][-2:]
        assert L.wtp_packed_shape(H, W, rec["eff_level"], ctypes.byref(pr), ctypes.byref(pc)) == 0
        assert [pr.value, pc.value] == rec["coeff_shape"][-2:], name


def _desc(shapes):
    arr = (N.WtpTensor * len(shapes))()
    for i, s in enumerate(shapes):
        arr[i].in_ = 0x1000
        arr[i].out = 0x1000
        arr[i].ndim = len(s)
        for j, v in enumerate(s):
            arr[i].shape[j] = v
    return arr


@pytest.mark.parametrize("shapes,wavelet,level,pct,code", [
    ([(4, 4, 3, 3)], "nosuch", 1, 50.0, N.WTP_EBADWAVELET),
    ([(16,)], "nosuch", 1, 50.0, None),                     # 1-D path never looks the wavelet up
    ([(4, 4, 3, 3)], "haar", -1, 50.0, N.WTP_EBADLEVEL),
    ([(4, 4, 3, 3)], "haar", 1, 100.5, N.WTP_EBADPCT),
    ([(4, 4, 3, 3)], "haar", 1, float("nan"), N.WTP_EBADPCT),
    ([(0,)], "haar", 1, 50.0, N.WTP_EEMPTY),
    ([(33, 17)], "db4", 2, 50.0, N.WTP_ECROP),
    ([(2, 2, 2, 18, 33)], "db2", 1, 50.0, N.WTP_ECROP),
    ([(16,), (33, 17)], "db4", 2, 50.0, N.WTP_ECROP),        # second tensor fails, index reported
])
def test_validation_errors_before_any_device_work(shapes, wavelet, level, pct, code):
    L = N.lib()
    wid = L.wtp_wavelet_id(wavelet.encode())
    d = _desc(shapes)
    if code is None:
        assert L.wtp_workspace_size(d, len(shapes), wid, level) > 0
        return
    rc = L.wtp_prune_f32(d, len(shapes), wid, level, pct, None, 0, 0x1000, None)
    assert rc == code
    assert L.wtp_last_error_tensor() == len(shapes) - 1
    assert N.last_error()


def test_workspace_size_covers_both_level_modes():
    L = N.lib()
    d = _desc([(4, 4, 3, 3), (2, 64, 64)])
    wid = L.wtp_wavelet_id(b"haar")
    assert L.wtp_workspace_size(d, 2, wid, 5) >= L.wtp_workspace_size(_desc([(2, 64, 64)]), 1, wid, 5)


def test_workspace_footprint_cfg5():
    """the level temps are sized per level kernel and shared by the launch
    groups (one set per group slot), so cfg5's workspace (64 x 4096^2, db8 L5) stays under 1.5x its
    weights (round 5: ~4x), and a call of 24 or fewer tensors still holds its own temps"""
    L = N.lib()
    wid = L.wtp_wavelet_id(b"db8")
    w = 4 * 4096 * 4096
    big = L.wtp_workspace_size_ex(_desc([(4096, 4096)] * 64), 64, wid, 5, 0)
    assert 0 < big <= 1.5 * 64 * w, big / (64 * w)
    one_group = L.wtp_workspace_size_ex(_desc([(4096, 4096)] * 24), 24, wid, 5, 0)
    # P of every tensor, plus 24 slots of three 2048^2 temps (level 1's approximation)
    assert one_group >= 24 * w + 24 * 3 * (w // 4)
    # the 40 extra blocks add their P and candidate buckets (the three-launch selection's, ~12 % of
    # P), not temps; with more than one group the fused selection's slot areas come in two sets
    # (24 x ~6.5 MB more)
    assert 40 * w <= big - one_group < 40 * w * 1.2


def test_mode_switches_validate_and_return_the_previous_mode():
    """wtp_set_resident / wtp_set_pipeline / wtp_set_fused_select (0 or 1): the previous mode returned,
    anything else rejected with WTP_EARG and the mode left as it was (host logic only, no device
    work)."""
    L = N.lib()
    for setter, top in ((L.wtp_set_resident, 1), (L.wtp_set_pipeline, 1), (L.wtp_set_fused_select, 1)):
        prev = setter(0)
        assert prev in range(top + 1)
        assert setter(1) == 0
        assert setter(top + 1) < 0 and setter(-1) < 0
        assert setter(top) == 1  # unchanged by the rejected calls
        assert setter(1) == top
        setter(prev)


def test_interior_mode_clamps_and_returns_the_previous_mode():
    """wtp_set_interior: 0 / 1 / 2 / 3, values outside clamped, the previous mode returned (host
    logic only: the mode is read at the next filter-bank launch)."""
    L = N.lib()
    prev = L.wtp_set_interior(2)
    assert prev in (0, 1, 2, 3)
    assert L.wtp_set_interior(0) == 2
    assert L.wtp_set_interior(1) == 0
    assert L.wtp_set_interior(7) == 1
    assert L.wtp_set_interior(-3) == 3
    assert L.wtp_set_interior(prev) == 0


def test_integration_stub_is_the_documented_block():
    """INTEGRATION.md section 2's code block is exactly tests/integration_stub.py's body (the GPU
    suite runs that file: tests/test_gpu_integration_stub.py)."""
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    doc = open(os.path.join(root, "INTEGRATION.md")).read()
    i = doc.index("```python\nimport ctypes, torch") + len("```python\n")
    block = doc[i:doc.index("```\n", i)]
    src = open(os.path.join(root, "tests", "integration_stub.py")).read()
    a = src.index("# --- begin INTEGRATION.md block ---\n") + len("# --- begin INTEGRATION.md block ---\n")
    body = src[a:src.index("# --- end INTEGRATION.md block ---")]
    assert body == block


def test_fused_selection_slot_areas_in_the_workspace():
    """The fused selection's wave slots (k_fwd_int: one 64-word slot per wave of every forward
    tile, FR x FC = 16 x 56 outputs a tile, 4 waves) plus a 512-byte head per tensor are reserved
    for a tensor that qualifies (>= 2^22 packed coefficients, tight, images >= 128^2, <= 6 levels,
    every level with interior tiles) and not for one that does not; a call of more than one launch
    group holds two sets (group parity) and k_fwin's per-segment histograms."""
    L = N.lib()
    wid = L.wtp_wavelet_id(b"db8")

    def ws(shapes, level):
        return L.wtp_workspace_size_ex(_desc(shapes), len(shapes), wid, level, 0)

    def slots(R, C, level):
        tot = 0
        for _ in range(level):
            Ro, Co = R // 2, C // 2
            tot += -(-Ro // 16) * -(-Co // 56) * 4
            R, C = Ro, Co
        return tot

    head, hist = 512, 24 * 4128 * 4  # FslHeader; SEG_PER_LAUNCH x FWIN_HW words
    # the same packed size, not fused: level 5's last level (a 128 x 128 input) has no interior tile
    assert ws([(2048, 2048)], 4) - ws([(2048, 2048)], 5) == 4 * slots(2048, 2048, 4) * 64 + head + hist
    # non-tight (2048 x 2040 at level 3: 2040 / 8 is not whole) -> nothing reserved
    assert ws([(2048, 2048)], 3) - ws([(2048, 2040)], 3) >= 4 * slots(2048, 2048, 3) * 64 + head + hist
    # two groups: two sets of 24 areas
    big, g1 = ws([(1024, 4096)] * 25, 4), ws([(1024, 4096)] * 24, 4)
    assert big - g1 >= 24 * (4 * slots(1024, 4096, 4) * 64 + head)
