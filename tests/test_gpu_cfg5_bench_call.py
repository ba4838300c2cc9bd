"""cfg5 exactly as bench.py runs it (BASELINE configs[4]: 64 x 4096^2 blocks, db8 level 5, the
50th percentile) in ONE engine.prune call -- three launch groups of 24 / 24 / 16 blocks with the
selection pipeline on (each group's fused selection -- k_fwin, the forward's classification,
k_fslot_collect, k_mask_select and the retry launches -- on the library's side stream beside the
next group's forward) -- value-checked on the first and last block of every group against PyWavelets 1.1.1
goldens (tools/gen_golden.py --cfg5-groups: output hashes, float64 threshold bits, zero counts),
out of place and in place.  Reference path: dwt_pruning.py:53-89 per block."""
import pytest
import torch

from tests import golden_io as G

pytestmark = pytest.mark.gpu

NBLK = 64


@pytest.fixture(scope="module")
def eng():
    from wavelettransforms_amd import engine
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    prev = engine.set_pipeline(True)
    yield engine
    engine.set_pipeline(prev)


def _check(rec, o, r):
    assert r["eff_level"] == rec["eff_level"] == 5
    assert G.f64_bits_equal(r["thr64"], rec["thr64"]), (rec["index"], r["thr64"], rec["thr64"])
    assert int(r["thr32_bits"]) == int(rec["thr32_bits"])
    assert int(r["max_abs_bits"]) == int(rec["max_abs_bits"])
    assert r["zero_count"] == rec["zero_count"]
    assert r["coeff_numel"] == rec["coeff_numel"]
    assert G.canon_hash(o.cpu().numpy()) == rec["out_hash"], rec["index"]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("in_place", [False, True], ids=["out_of_place", "in_place"])
def test_cfg5_one_call_three_groups(eng, in_place):
    recs = G.manifest()["large"]["cfg5_db8_L5_groups"]
    blocks = G.W.block_tensors(NBLK)
    xs = [eng.synth(s, seed, tid, e) for _, s, seed, tid, e in blocks]
    outs, res = eng.prune(xs, "db8", 5, 50.0, outs=xs if in_place else None, carry_level=False)
    torch.cuda.synchronize()
    for rec in recs:
        i = rec["index"]
        if in_place:
            assert outs[i].data_ptr() == xs[i].data_ptr()
        _check(rec, outs[i], res[i])
    # every block carries a record of the full path (no fault, no missing record)
    assert all(r["eff_level"] == 5 and r["coeff_numel"] == 4096 * 4096 for r in res)
