"""Min-weight pruning (ResNet/min_weight_pruning.py:66-139).

CPU: the oracle restatement against torch.topk (counts always; values where the k-th smallest
|w| is not tied), the k = int(n * p) rule against the reference's stored min_pruned logs, and the
log helpers of the mirror module.  GPU (marked): the HIP path against the oracle, bit for bit."""
import csv
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests import golden_io as G


def _torch_min_prune(x, p):
    t = torch.from_numpy(x.copy())
    v = t.view(-1)
    k = int(v.numel() * p)
    if k:
        _, idx = torch.topk(v.abs(), k, largest=False)
        v[idx] = 0
    return t.numpy(), k


@pytest.mark.parametrize("n,p,ties", [(1000, 0.3, True), (9408, 0.5, True), (36864, 0.618, False), (37, 1.0, True),
                                      (10, 0.0, True), (100, 0.999, False), (1, 0.5, False), (4099, 0.9, False)])
def test_oracle_vs_torch_topk(n, p, ties):
    rng = np.random.default_rng(n)
    x = (rng.integers(-20, 21, n).astype(np.float32) if ties else rng.standard_normal(n).astype(np.float32))
    out, z, t = O.min_prune(x, p)
    ref, k = _torch_min_prune(x, p)
    assert z == int((ref == 0).sum())                      # counts: exact whatever the tie order
    a = np.abs(x)
    if k and (a == t).sum() == 1 or k == 0:                # no tie at the boundary: identical values
        assert np.array_equal(out, ref)
    if k:                                                  # our rule: lowest indices among ties
        need = k - int((a < t).sum())
        eq = np.nonzero(a == t)[0]
        assert np.all(out[eq[:need]] == 0) and np.all(out[eq[need:]] == x[eq[need:]])
        assert np.all(out[a < t] == 0) and np.array_equal(out[a > t], x[a > t])


def test_oracle_k_out_of_range():
    with pytest.raises(RuntimeError):
        O.min_prune(np.ones(10, np.float32), 1.2)
    out, z, _ = O.min_prune(np.ones(10, np.float32), -0.05)   # int(-0.5) == 0: nothing pruned
    assert z == 0 and np.all(out == 1)


def test_reference_min_logs_follow_int_n_p():
    """The stored min_pruned logs: per layer pruned = int(n * p), p = the selective run's overall
    pruned fraction (min_weight_pruning.py:54-63,70) -- 160 rows over 8 runs."""
    runs = G.reference_logs()["stored_models"]
    rows = 0
    for run, phases in runs.items():
        if "min_pruned" not in phases:
            continue
        sel = phases["selective_pruned"]
        p = sum(r["pruned"] for r in sel) / sum(r["n"] for r in sel)
        for r in phases["min_pruned"]:
            rows += 1
            assert r["pruned"] == int(r["n"] * p) and r["nonzero"] == r["n"] - r["pruned"], (run, r["layer"])
    assert rows == 160


def test_log_helpers(tmp_path):
    from wavelettransforms_amd import min_weight_pruning as M
    from wavelettransforms_amd.utils import LAYER_LOG_FIELDS
    path = tmp_path / "log.csv"
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=LAYER_LOG_FIELDS)
        w.writeheader()
        for name, n, pr in [("a", 100, 40), ("b", 300, 110)]:
            w.writerow({"GUID": "g", "Wavelet": "haar", "Level": 1, "Threshold": 0.5, "DWT Phase": "selective",
                        "Original Parameter Count": n, "Non-zero Params": n - pr, "Total Pruned Count": pr,
                        "Layer Name": name})
    assert M.read_selective_pruning_log(str(path)) == {"a": 100, "b": 300}
    assert M.calculate_dwt_pruning_percentage(str(path)) == 150 / 400


# ------------------------------------------------------------------------------ GPU ---
@pytest.fixture(scope="module")
def eng():
    from wavelettransforms_amd import engine
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return engine


@pytest.mark.gpu
@pytest.mark.parametrize("n,p", [(1, 0.5), (7, 0.5), (4097, 0.25), (16384, 0.5), (16385, 0.999), (100_003, 0.1),
                                 (2 * 16384 + 4099, 0.75), (589_824, 0.5), (10, 0.0), (37, 1.0)])
def test_gpu_min_prune_vs_oracle(eng, n, p):
    rng = np.random.default_rng(n + 1)
    xs = [rng.integers(-30, 31, n).astype(np.float32) * np.float32(0.01),       # ties everywhere
          (rng.standard_normal(n) * 0.05).astype(np.float32)]
    dev = [torch.from_numpy(x).cuda() for x in xs]
    outs, recs = eng.min_prune(dev, p)
    for x, o, r in zip(xs, outs, recs):
        ref, z, t = O.min_prune(x, p)
        assert np.array_equal(o.cpu().numpy(), ref)
        assert r["zero_count"] == z and r["numel"] == n
        if int(n * p):
            assert np.float32(r["thr32"]) == np.float32(t)


@pytest.mark.gpu
def test_gpu_min_prune_resnet18_batch_in_place(eng):
    ts = G.W.resnet18_tensors(0)
    xs = [eng.synth(s, seed, tid, e) for _, s, seed, tid, e in ts]
    host = [x.cpu().numpy() for x in xs]
    p = 0.4999993
    outs, recs = eng.min_prune(xs, p, outs=xs)                  # in place, one launch sequence
    for (name, *_), h, o, r in zip(ts, host, outs, recs):
        ref, z, _ = O.min_prune(h, p)
        assert np.array_equal(o.cpu().numpy(), ref), name
        assert r["zero_count"] == z


@pytest.mark.gpu
def test_gpu_min_prune_special_values(eng):
    x = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-30, -1e-30, 3.0, -3.0, 0.5] * 50, np.float32)
    for p in (0.1, 0.35, 0.6, 0.9):
        (o,), (r,) = eng.min_prune([torch.from_numpy(x).cuda()], p)
        ref, z, _ = O.min_prune(x, p)
        assert np.array_equal(o.cpu().numpy(), ref, equal_nan=True) and r["zero_count"] == z


@pytest.mark.gpu
def test_gpu_percentage_min_pruning_mirror(eng):
    from wavelettransforms_amd.min_weight_pruning import percentage_min_pruning
    w = torch.from_numpy((np.random.default_rng(5).standard_normal((64, 32, 3, 3)) * 0.1).astype(np.float32))
    ref, _ = _torch_min_prune(w.numpy(), 0.3)
    wc = w.clone().cuda()
    out = percentage_min_pruning(wc, 0.3)
    assert out.shape == wc.shape and out.data_ptr() == wc.data_ptr()       # in place, like the view write
    assert np.array_equal(wc.cpu().numpy(), ref)                           # continuous weights: no ties
    wcpu = w.clone()
    percentage_min_pruning(wcpu, 0.3)                                       # CPU weights come back in place
    assert np.array_equal(wcpu.numpy(), ref)
    with pytest.raises(RuntimeError):
        percentage_min_pruning(w.clone().cuda(), 1.5)


@pytest.mark.gpu
def test_gpu_min_weight_pruning_driver(eng, tmp_path, capsys):
    """The baseline driver end to end on a small model: CSV rows and totals follow the rule
    pruned = int(n * p) the reference's stored logs show."""
    from wavelettransforms_amd import min_weight_pruning as M
    from wavelettransforms_amd.utils import LAYER_LOG_FIELDS
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Conv2d(3, 16, 3), torch.nn.ReLU(), torch.nn.Conv2d(16, 8, 3))
    sel = tmp_path / "sel.csv"
    with open(sel, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=LAYER_LOG_FIELDS)
        w.writeheader()
        for name, m in [("0", model[0]), ("2", model[2])]:
            n = m.weight.numel()
            w.writerow({"GUID": "abcd1234", "Wavelet": "haar", "Level": 1, "Threshold": 0.5,
                        "DWT Phase": "selective", "Original Parameter Count": n, "Non-zero Params": n // 2,
                        "Total Pruned Count": n - n // 2, "Layer Name": name})
    cwd = os.getcwd()
    work = tmp_path / "a" / "b"        # the reference writes to <cwd>/../../WaveletTransforms/ResNet/SavedModels
    work.mkdir(parents=True)
    os.chdir(work)
    try:
        M.min_weight_pruning(model, str(sel), "abcd1234", "haar", 1, 0.5, str(tmp_path / "exp.csv"))
    finally:
        os.chdir(cwd)
    p = M.calculate_dwt_pruning_percentage(str(sel))
    logs = list(csv.DictReader(open(next(tmp_path.rglob("min_pruned/log.csv")))))
    assert [r["Layer Name"] for r in logs] == ["0", "2"]
    for r, m in zip(logs, (model[0], model[2])):
        n = m.weight.numel()
        assert int(r["Total Pruned Count"]) == int(n * p) == int((m.weight == 0).sum())
    out = capsys.readouterr().out
    assert "Skipping layer:  (not in selective pruning log)" in out and "Pruned layer: 0," in out
