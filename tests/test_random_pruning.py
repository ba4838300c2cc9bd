"""Random pruning and the evaluation sparsity count (SURVEY.md 8f rank 4:
ResNet/random_pruning.py:49-56, testing_suite/eval_model.py:7-20).

Parity is unpinned for the positions: the reference draws torch.randperm (Philox), which is not
reproduced.  What IS pinned: the counts -- the reference's stored random_pruned logs hold
pruned == the selective run's pruned count for all 160 rows -- and the rule itself (k distinct
positions, Python slice semantics for k, count_nonzero afterwards), checked on the oracle here and
on the GPU path against the oracle bit for bit (both use the permutation of csrc/wt_perm.h)."""
import csv
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests import golden_io as G


@pytest.mark.parametrize("n,k", [(1, 1), (2, 1), (3, 2), (9408, 4704), (36864, 18432), (100, 0), (100, 100),
                                 (100, 250), (100, -30), (100, -250), (4097, 4096), (65537, 12345)])
def test_oracle_random_prune_counts(n, k):
    x = np.ones(n, np.float32)
    out, z = O.random_prune(x, k, seed=7, tensor_id=3)
    keff = len(range(n)[:k])                       # torch.randperm(n)[:k]: Python slicing
    assert z == keff == int((out == 0).sum())
    assert np.all(out[out != 0] == 1)


def test_oracle_permutation_is_a_bijection():
    for n in (1, 2, 3, 5, 16, 17, 1000, 4099):
        for tid in range(3):
            x = np.arange(1, n + 1, dtype=np.float32)
            out, z = O.random_prune(x, n, seed=11, tensor_id=tid)
            assert z == n and not out.any()
            half, _ = O.random_prune(x, n // 2, seed=11, tensor_id=tid)
            assert int((half == 0).sum()) == n // 2


def test_oracle_keys_and_spread():
    x = np.ones(10000, np.float32)
    a, _ = O.random_prune(x, 1000, seed=1, tensor_id=0)
    b, _ = O.random_prune(x, 1000, seed=1, tensor_id=0)
    c, _ = O.random_prune(x, 1000, seed=1, tensor_id=1)
    d, _ = O.random_prune(x, 1000, seed=2, tensor_id=0)
    assert np.array_equal(a, b) and not np.array_equal(a, c) and not np.array_equal(a, d)
    # uniform spread: every tenth of the tensor holds ~100 of the 1000 positions
    per = (a == 0).reshape(10, 1000).sum(axis=1)
    assert per.min() > 60 and per.max() < 140, per
    # the first k positions of a longer prefix contain the shorter prefix (randperm(n)[:k] nesting)
    e, _ = O.random_prune(x, 2000, seed=1, tensor_id=0)
    assert np.all(e[a == 0] == 0)


def test_oracle_random_prune_counts_existing_zeros_and_nan():
    x = np.array([0.0, -0.0, 1.0, np.nan, 2.0, 0.0, 3.0, -4.0] * 100, np.float32)
    for k in (0, 50, 400, 800):
        out, z = O.random_prune(x, k, seed=5, tensor_id=0)
        assert z == int((out == 0).sum())                           # NaN counts as non-zero
        assert int((out == 0).sum()) >= int((x == 0).sum())


def test_reference_random_logs_prune_the_selective_count():
    """The stored random_pruned logs: pruned == the selective run's pruned count of the layer
    (random_pruning.py:45,53-61 on weights without zeros) -- 160 rows over 8 runs."""
    rows = 0
    for run, phases in G.reference_logs()["stored_models"].items():
        sel = {r["layer"]: r for r in phases["selective_pruned"]}
        for r in phases.get("random_pruned", []):
            rows += 1
            assert r["pruned"] == sel[r["layer"]]["pruned"] and r["nonzero"] == r["n"] - r["pruned"], (run, r)
    assert rows == 160


# ------------------------------------------------------------------------------ GPU ---
@pytest.fixture(scope="module")
def eng():
    from wavelettransforms_amd import engine
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return engine


@pytest.mark.gpu
@pytest.mark.parametrize("inplace", [False, True])
def test_gpu_random_prune_vs_oracle(eng, inplace):
    cases = [(1, 1), (7, 3), (4097, 2048), (16384, 16384), (16385, 100), (100_003, 50_001), (589_824, 294_911),
             (2_359_296, 1_179_647), (1000, 0), (1000, 5000), (1000, -10)]
    rng = np.random.default_rng(3)
    xs = [(rng.standard_normal(n) * 0.05).astype(np.float32) for n, _ in cases]
    xs[3][::7] = 0.0                                                 # zeros already present
    dev = [torch.from_numpy(x).cuda() for x in xs]
    ks = [k for _, k in cases]
    outs, recs = eng.random_prune(dev, ks, seed=1234, outs=dev if inplace else None)
    for t, (x, o, r, k) in enumerate(zip(xs, outs, recs, ks)):
        ref, z = O.random_prune(x, k, 1234, t)
        assert np.array_equal(o.cpu().numpy(), ref), t
        assert r["zero_count"] == z and r["numel"] == x.size
        if inplace:
            assert o.data_ptr() == dev[t].data_ptr()


@pytest.mark.gpu
def test_gpu_random_prune_resnet18_batch(eng):
    ts = G.W.resnet18_tensors(0)
    xs = [eng.synth(s, seed, tid, e) for _, s, seed, tid, e in ts]
    host = [x.cpu().numpy() for x in xs]
    ks = [int(x.numel() // 2) for x in xs]
    outs, recs = eng.random_prune(xs, ks, seed=99, outs=xs)
    for t, ((name, *_), h, o, r) in enumerate(zip(ts, host, outs, recs)):
        ref, z = O.random_prune(h, ks[t], 99, t)
        assert np.array_equal(o.cpu().numpy(), ref), name
        assert r["zero_count"] == z


@pytest.mark.gpu
def test_gpu_random_pruning_driver(eng, tmp_path, capsys):
    """The baseline driver on a small model: CSV rows and totals follow the stored logs' rule
    (pruned == the selective count); a layer the model lacks is reported and skipped."""
    from wavelettransforms_amd import random_pruning as R
    from wavelettransforms_amd.utils import LAYER_LOG_FIELDS
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Conv2d(3, 16, 3), torch.nn.ReLU(), torch.nn.Conv2d(16, 8, 3))
    sel = tmp_path / "sel.csv"
    plan = [("0", model[0].weight.numel(), 200), ("2", model[2].weight.numel(), 500), ("9", 10, 5), ("1", 0, 0)]
    with open(sel, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=LAYER_LOG_FIELDS)
        w.writeheader()
        for name, n, pr in plan:
            w.writerow({"GUID": "abcd1234", "Wavelet": "haar", "Level": 1, "Threshold": 0.5,
                        "DWT Phase": "selective", "Original Parameter Count": n, "Non-zero Params": n - pr,
                        "Total Pruned Count": pr, "Layer Name": name})
    cwd = os.getcwd()
    work = tmp_path / "a" / "b"
    work.mkdir(parents=True)
    os.chdir(work)
    try:
        R.random_pruning(model, str(sel), "abcd1234", "haar", 1, 0.5, str(tmp_path / "exp.csv"))
    finally:
        os.chdir(cwd)
    logs = list(csv.DictReader(open(next(tmp_path.rglob("random_pruned/log.csv")))))
    assert [r["Layer Name"] for r in logs] == ["0", "2"]
    for r, m, (_, n, pr) in zip(logs, (model[0], model[2]), plan):
        assert int(r["Total Pruned Count"]) == pr == int((m.weight == 0).sum())
        assert int(r["Non-zero Params"]) == n - pr
    assert not model[0].weight.is_cuda                               # pruned where it lies
    exp = list(csv.reader(open(tmp_path / "exp.csv")))
    assert exp[1][4] == "random" and int(exp[1][5]) == 700
    out = capsys.readouterr().out
    assert "Processing layer: 0 with prune count: 200" in out
    assert "Layer not found or not a Conv2D layer: 9" in out and "Layer not found or not a Conv2D layer: 1" in out
    assert "Random pruning completed." in out


@pytest.mark.gpu
def test_gpu_calculate_sparsity(eng):
    from wavelettransforms_amd.eval_model import calculate_sparsity
    torch.manual_seed(1)
    model = torch.nn.Sequential(torch.nn.Conv2d(3, 16, 3), torch.nn.Linear(16, 4))
    with torch.no_grad():
        w = model[0].weight.view(-1)
        w[:100] = 0
        w[100:140] = torch.tensor(np.float32(1e-6)).item()              # exactly f32(1e-6): not < thr
        w[140:160] = float(np.nextafter(np.float32(1e-6), np.float32(0)))
        w[160:170] = float("nan")
        model[1].weight.view(-1)[:7] = -5e-7

    def ref(m, thr=1e-6):
        tot = near = 0
        for p in m.parameters():
            if p.dim() > 1:
                tot += p.numel()
                near += torch.sum(torch.abs(p) < thr).item()
        return near / tot
    assert calculate_sparsity(model) == ref(model)
    assert calculate_sparsity(model.cuda()) == ref(model.cpu())
    assert calculate_sparsity(model, threshold=0.05) == ref(model, 0.05)
    assert calculate_sparsity(torch.nn.ReLU()) == 0.0
