"""CPU: the oracle's 1-D flattened mode (oracle.prune_tensor_flat, WTP_FLATTEN) against the
PyWavelets 1.1.1 + NumPy 1.26.4 goldens of tools/gen_golden_flat.py (wavedec / coeffs_to_array
/ percentile / waverec of w.ravel()): values bit for bit, threshold bits, zero counts, the
packed coefficients and the coefficient-domain mask."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests import golden_io as G

FLAT = json.load(open(os.path.join(G.GOLDEN, "flat_manifest.json")))
ARR = dict(np.load(os.path.join(G.GOLDEN, "flat_cases.npz")))
NAMES = sorted(FLAT["cases"])


def flat_input(rec):
    return G.W.synth_numpy(tuple(rec["shape"]), *rec["synth"])


@pytest.mark.parametrize("name", NAMES)
def test_oracle_flat_matches_pywt(name):
    rec = FLAT["cases"][name]
    x = flat_input(rec)
    out, r, P = O.prune_tensor_flat(x, rec["wavelet"], rec["level_in"], rec["pct"], want_coeffs=True)
    assert r["eff_level"] == rec["eff_level"] and r["coeff_numel"] == rec["coeff_numel"]
    assert G.f64_bits_equal(r["thr64"], rec["thr64"])
    assert r["zero_count"] == rec["zero_count"]
    assert G.canon_hash(out) == rec["out_hash"]
    if name + "/out" in ARR:
        assert np.array_equal(out, ARR[name + "/out"])
    if "coeff_hash" in rec:
        assert G.canon_hash(P) == rec["coeff_hash"]
        mask = np.abs(P) < np.float32(r["thr64"])
        assert int(mask.sum()) == rec["mask_count"] and G.mask_hash(mask) == rec["mask_hash"]


def test_oracle_flat_level_carry():
    lvl = 9
    for j, rec in enumerate(FLAT["multi_db2_L9_p61.8"]):
        x = G.W.synth_numpy(tuple(rec["shape"]), *rec["synth"])
        out, r = O.prune_tensor_flat(x, "db2", lvl, 61.8)
        assert r["eff_level"] == rec["eff_level"]
        assert np.array_equal(out, ARR["multi/out%d" % j])
        if x.ndim >= 2:
            lvl = r["eff_level"]
