"""Large analysis levels at shapes the golden cases do not reach: several tiles across and down,
odd extents (periodization's repeated last sample), partial last tiles, the right-edge split order,
batch dimensions and two depths.  Packed coefficients (pywt.wavedec2 + coeffs_to_array,
ResNet/dwt_pruning.py:67-72) and the pruned outputs must equal the oracle bit for bit for every
filter length the filter bank specialises."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests import golden_io as G
from wavelettransforms_amd import engine as eng

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"


# F = 2, 4, 6, 8, 10, 12, 16, 18: every specialised filter length
WAVELETS = ["haar", "db2", "rbio2.2", "bior3.3", "db5", "coif2", "db8", "db9"]
# odd extents (4-D, as the reference's crop needs), a last tile row of one output row (R = 130),
# a last tile a few columns wide
SHAPES = [(1, 1, 130, 1001), (2, 1, 255, 520), (1, 3, 301, 777), (512, 1024), (999, 600)]


@pytest.mark.parametrize("wavelet", WAVELETS)
def test_large_levels_equal_oracle(wavelet):
    for j, shp in enumerate(SHAPES):
        e = G.W.sigma_exponent((2.0 / (shp[-1] * shp[-2])) ** 0.5)
        host = G.W.synth_numpy(shp, 31, j, e)
        x = eng.synth(shp, 31, j, e)
        for level in (1, 3):
            P = eng.wavedec2_packed(x, wavelet, level).cpu().numpy()
            assert np.array_equal(P.view(np.uint32), O.wavedec2_packed(host, wavelet, level).view(np.uint32)), \
                (shp, level)
            if len(shp) == 2 and (shp[0] % 2 or shp[1] % 2):
                continue  # odd 2-D: the reference's crop raises (dwt_pruning.py:79-82)
            ref, rr = O.prune_tensor(host, wavelet, level, 37.5)
            outs, (r,) = eng.prune([x], wavelet, level, 37.5)
            assert np.array_equal(outs[0].cpu().numpy(), ref), (shp, level)
            assert r["zero_count"] == rr["zero_count"] and G.f64_bits_equal(r["thr64"], rr["thr64"])


@pytest.mark.parametrize("wavelet", WAVELETS)
def test_interior_kernels_equal_general(wavelet):
    """The interior filter-bank kernels (k_fwd_int / k_inv_int) with the frame of edge tiles in
    their EDGE form (mode 2; mode 3, the default, runs the small levels' every tile in the EDGE
    form), and in the general kernels (mode 1), against every tile
    in the general kernels (mode 0): packed coefficients and pruned outputs bit for bit, on shapes
    with an interior and a frame (odd extents, batches, partial last tiles, a 2-level and a 4-level
    tree; the deepest levels of the narrow shape fall back to the general frame; levels of 40-48
    coefficients, just wide enough for the EDGE frame, where a tile holds the level's last
    special / wrapped sites behind a partial extent -- the fix-up passes' densest case)."""
    shapes = [(1, 2, 700, 1100), (1, 1, 1031, 515), (800, 1600), (2, 1, 333, 4100), (1, 1, 170, 180),
              (1, 1, 680, 700)]
    prev = eng.set_interior(3)
    try:
        for j, shp in enumerate(shapes):
            e = G.W.sigma_exponent((2.0 / (shp[-1] * shp[-2])) ** 0.5)
            x = eng.synth(shp, 41, j, e)
            for level in (2, 4):
                res = []
                for mode in (3, 2, 1, 0):
                    eng.set_interior(mode)
                    P = eng.wavedec2_packed(x, wavelet, level).cpu().numpy().view(np.uint32)
                    outs, (r,) = eng.prune([x], wavelet, level, 61.8)
                    res.append((P, outs[0].cpu().numpy().view(np.uint32), r["zero_count"], r["thr64"]))
                Pg, og, zg, tg = res[-1]
                for m, (Pm, om, zm, tm) in zip((3, 2, 1), res[:3]):
                    assert np.array_equal(Pm, Pg), (shp, level, m)
                    assert np.array_equal(om, og), (shp, level, m)
                    assert zm == zg and G.f64_bits_equal(tm, tg), (shp, level, m)
    finally:
        eng.set_interior(prev)
