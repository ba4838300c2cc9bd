"""The reference's own recorded outputs for this path (ResNet/StoredModels/*/selective_pruned/
log.csv and experiment_log.csv:739-786, copied into tests/golden/reference_logs.json by
tools/extract_reference_logs.py) pin the percentile semantics the oracle restates.

The real pretrained weights are not available offline, so the per-layer counts cannot be
re-derived value for value; what they pin is the rank arithmetic: with every ResNet-18
kernel clamped to DWT level 0, each layer prunes lo+1 = floor((n-1)q)+1 weights, or lo when
float32(threshold) rounds onto s[lo] (NumPy 1.x float32 compare) -- 4 such cases appear."""
import json
import math
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests import golden_io as G

LOGS = json.load(open(os.path.join(G.GOLDEN, "reference_logs.json")))


def _lo(n, threshold):
    pct = threshold * 100          # main_pruning.py:186 passes FLAGS.threshold * 100
    q = pct / 100                  # np.percentile divides by 100 (function_base.py:4279)
    return math.floor((n - 1) * q), q


def test_stored_selective_counts_follow_rank_rule():
    minus_one = []
    for run, phases in LOGS["stored_models"].items():
        for r in phases["selective_pruned"]:
            n, lo_q = r["n"], _lo(r["n"], r["threshold"])
            lo, q = lo_q
            assert r["nonzero"] + r["pruned"] == n
            if q >= 1.0:
                assert r["pruned"] == n - 1, (run, r)
            else:
                assert r["pruned"] in (lo, lo + 1), (run, r)
                if r["pruned"] == lo:
                    minus_one.append((r["threshold"], r["layer"]))
    assert sorted(minus_one) == sorted([
        (0.1, "resnet.encoder.stages.3.layers.0.layer.1.convolution"),
        (0.5, "resnet.encoder.stages.3.layers.0.layer.0.convolution"),
        (0.618, "resnet.encoder.stages.3.layers.1.layer.1.convolution"),
        (0.9, "resnet.encoder.stages.3.layers.0.layer.1.convolution"),
    ])


def test_experiment_log_totals_match_stored_layers():
    by_guid = {}
    for run, phases in LOGS["stored_models"].items():
        rows = phases["selective_pruned"]
        by_guid[rows[0]["wavelet"], rows[0]["threshold"]] = sum(r["pruned"] for r in rows)
    sel = [r for r in LOGS["experiment_log"] if r["phase"] == "selective"]
    for r in sel:
        if r["wavelet"] == "bior4.4":
            assert by_guid["bior4.4", r["threshold"]] == r["total_pruned"]
    # bior1.3 (F=6) and bior4.4 (F=10) both clamp every ResNet-18 kernel to level 0
    b13 = {r["threshold"]: r["total_pruned"] for r in sel if r["wavelet"] == "bior1.3"}
    b44 = {r["threshold"]: r["total_pruned"] for r in sel if r["wavelet"] == "bior4.4"}
    for t in b13:
        assert b13[t] == b44[t]
    for k in (1, 3, 7):
        assert O.dwt_max_level(k, O.dec_len("bior1.3")) == 0
        assert O.dwt_max_level(k, O.dec_len("bior4.4")) == 0


@pytest.mark.parametrize("threshold", [0.1, 0.236, 0.382, 0.5, 0.618, 0.786, 0.9, 1.0])
def test_oracle_reproduces_rule_on_resnet18_shapes(threshold):
    stored = next(p["selective_pruned"] for p in LOGS["stored_models"].values()
                  if p["selective_pruned"][0]["threshold"] == threshold)
    for (name, shape, seed, tid, e), row in zip(G.W.resnet18_tensors(0), stored):
        assert row["layer"] == name and row["n"] == int(np.prod(shape))
        x = G.W.synth_numpy(shape, seed, tid, e)
        out, res = O.prune_tensor(x, "bior4.4", 5, threshold * 100)
        lo, q = _lo(row["n"], threshold)
        assert res["eff_level"] == 0
        if q >= 1.0:
            assert res["zero_count"] <= row["n"] - 1
        else:
            assert res["zero_count"] in (lo, lo + 1)
