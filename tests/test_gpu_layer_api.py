"""The per-layer entry points of the drop-in module on the GPU:
prune_layer_weights and its north-star alias prune_conv_layer (ResNet/dwt_pruning.py:98-127) and
analyze_pruning (:16-22) -- printed lines, return tuple, the `.data` reassignment, the bias left
alone -- checked against the C oracle and the golden fixtures."""
import re

import numpy as np
import pytest
import torch
import torch.nn as nn

from oracle import oracle as O
from tests import golden_io as G
from wavelettransforms_amd import dwt_pruning as D

pytestmark = pytest.mark.gpu


def _conv(shape, seed, tid, device):
    o, i, kh, kw = shape
    m = nn.Conv2d(i, o, (kh, kw), bias=True).to(device)
    e = G.W.sigma_exponent(G.W.conv_sigma(shape))
    with torch.no_grad():
        m.weight.copy_(torch.from_numpy(G.W.synth_numpy(shape, seed, tid, e)))
        m.bias.copy_(torch.arange(o, dtype=torch.float32))
    return m, G.W.synth_numpy(shape, seed, tid, e)


@pytest.mark.parametrize("fn", [D.prune_layer_weights, D.prune_conv_layer], ids=["prune_layer_weights",
                                                                                "prune_conv_layer"])
@pytest.mark.parametrize("shape,wavelet,level,pct", [((64, 64, 3, 3), "haar", 5, 61.8),
                                                     ((64, 3, 7, 7), "haar", 5, 50.0),
                                                     ((128, 64, 3, 3), "bior3.3", 5, 23.599999999999998),
                                                     ((256, 128, 1, 1), "bior4.4", 5, 90.0)])
@pytest.mark.parametrize("device", ["cuda", "cpu"])
def test_prune_layer_weights(capsys, fn, shape, wavelet, level, pct, device):
    assert torch.cuda.is_available()
    m, host = _conv(shape, 3, 7, device)
    bias_before = m.bias.detach().clone()
    w_param = m.weight
    ret = fn(m, wavelet, level, pct)
    ref, rr = O.prune_tensor(host, wavelet, level, pct)
    nonzero = int(np.count_nonzero(ref))
    assert ret == (ref.size, nonzero, rr["zero_count"])
    assert isinstance(ret[0], int) and isinstance(ret[1], int) and isinstance(ret[2], int)
    # layer.weight.data = pruned[0]: the same Parameter object, new data, on the layer's device
    assert m.weight is w_param and m.weight.device.type == device and m.weight.shape == shape
    assert np.array_equal(m.weight.detach().cpu().numpy(), ref)
    assert torch.equal(m.bias.detach(), bias_before)
    out = capsys.readouterr().out.splitlines()
    assert out[-1] == "Original Param Count: %d, Non-zero Params: %d, Total Pruned Count: %d" % (
        ref.size, nonzero, rr["zero_count"])
    # :29-30 -- f-string of the np.float64 threshold and of the np.float32 max |coefficient| (an
    # f-string formats a NumPy float32 through Python float in NumPy 1.26 as in 2.x: 17 digits)
    thr_line = [l for l in out if l.startswith("Percentile: ")]
    assert thr_line and thr_line[0] == f"Percentile: {pct}, Threshold: {np.float64(rr['thr64'])}, " \
                                       f"Max Coeff: {np.float32(rr['max_abs'])}"


def test_analyze_pruning(capsys):
    """Per-Conv2d sparsity lines, in named_modules order, for a model pruned on the GPU."""
    model = nn.Sequential(nn.Conv2d(3, 64, 7), nn.ReLU(), nn.Conv2d(64, 64, 3), nn.Linear(4, 4),
                          nn.Conv2d(64, 128, 1)).cuda()
    for i, m in enumerate(model):
        if isinstance(m, nn.Conv2d):
            e = G.W.sigma_exponent(G.W.conv_sigma(tuple(m.weight.shape)))
            with torch.no_grad():
                m.weight.copy_(torch.from_numpy(G.W.synth_numpy(tuple(m.weight.shape), i, i, e)))
            D.prune_layer_weights(m, "haar", 5, 38.2)
    capsys.readouterr()
    D.analyze_pruning(model)
    lines = capsys.readouterr().out.splitlines()
    convs = [(n, m) for n, m in model.named_modules() if isinstance(m, nn.Conv2d)]
    assert len(lines) == len(convs)
    for line, (name, m) in zip(lines, convs):
        w = m.weight.detach()
        assert line == f"Layer {name}: Sparsity = {(w == 0).sum().item() / w.numel():.2%}"
        assert re.match(r"Layer \d+: Sparsity = \d+\.\d\d%$", line)


def test_multi_resolution_analysis_list_carry():
    """A list call carries the clamped level (dwt_pruning.py:64-65): the 3x3 tensor clamps haar L5
    to 1, and the 7x7 tensor after it then runs at level 1, not 2."""
    shapes = [(64, 64, 3, 3), (64, 3, 7, 7)]
    host = [G.W.synth_numpy(s, 1 + k, k, 26) for k, s in enumerate(shapes)]
    outs, zc = D.multi_resolution_analysis([torch.from_numpy(h).cuda() for h in host], "haar", 5, 50.0,
                                           verbose=False)
    lvl, total = 5, 0
    for h, o in zip(host, outs):
        ref, rr = O.prune_tensor(h, "haar", lvl, 50.0)
        lvl = min(lvl, rr["eff_level"])
        assert np.array_equal(o.cpu().numpy(), ref)
        total += rr["zero_count"]
    assert lvl == 1 and zc == total
