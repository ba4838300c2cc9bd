"""Workload definitions shared by bench.py, the tests and tools/gen_golden.py.

Dependency-free (NumPy + stdlib only) so that tools/gen_golden.py can load it under the
oracle interpreter (/opt/conda/bin/python3.9, no torch).

Configs follow BASELINE.json / SURVEY.md section 8(d):
  cfg1  (64,64,3,3) haar level 1                         (CPU-runnable reference case)
  cfg2  the 20 ResNet-18 Conv2d weights, bior3.3 level 5, percentile 50   <- headline
  cfg3  MNIST-MLP Linear weights (128,784),(10,128), rbio2.2 level 3
  cfg4  cfg2 sharded over ranks (LPT) + all-gather
  cfg5  4096x4096 fp32 blocks, db8 level 5 (one block = one tensor)
Synthetic values come from the splitmix64 / Irwin-Hall generator of csrc/wt_synth.h.
"""
import math

import numpy as np

# ResNet-18 Conv2d weights in HF `named_modules()` order; names and sizes match the
# reference's stored logs (ResNet/StoredModels/*/selective_pruned/log.csv).
RESNET18_CONVS = [
    ("resnet.embedder.embedder.convolution", (64, 3, 7, 7)),
    ("resnet.encoder.stages.0.layers.0.layer.0.convolution", (64, 64, 3, 3)),
    ("resnet.encoder.stages.0.layers.0.layer.1.convolution", (64, 64, 3, 3)),
    ("resnet.encoder.stages.0.layers.1.layer.0.convolution", (64, 64, 3, 3)),
    ("resnet.encoder.stages.0.layers.1.layer.1.convolution", (64, 64, 3, 3)),
    ("resnet.encoder.stages.1.layers.0.shortcut.convolution", (128, 64, 1, 1)),
    ("resnet.encoder.stages.1.layers.0.layer.0.convolution", (128, 64, 3, 3)),
    ("resnet.encoder.stages.1.layers.0.layer.1.convolution", (128, 128, 3, 3)),
    ("resnet.encoder.stages.1.layers.1.layer.0.convolution", (128, 128, 3, 3)),
    ("resnet.encoder.stages.1.layers.1.layer.1.convolution", (128, 128, 3, 3)),
    ("resnet.encoder.stages.2.layers.0.shortcut.convolution", (256, 128, 1, 1)),
    ("resnet.encoder.stages.2.layers.0.layer.0.convolution", (256, 128, 3, 3)),
    ("resnet.encoder.stages.2.layers.0.layer.1.convolution", (256, 256, 3, 3)),
    ("resnet.encoder.stages.2.layers.1.layer.0.convolution", (256, 256, 3, 3)),
    ("resnet.encoder.stages.2.layers.1.layer.1.convolution", (256, 256, 3, 3)),
    ("resnet.encoder.stages.3.layers.0.shortcut.convolution", (512, 256, 1, 1)),
    ("resnet.encoder.stages.3.layers.0.layer.0.convolution", (512, 256, 3, 3)),
    ("resnet.encoder.stages.3.layers.0.layer.1.convolution", (512, 512, 3, 3)),
    ("resnet.encoder.stages.3.layers.1.layer.0.convolution", (512, 512, 3, 3)),
    ("resnet.encoder.stages.3.layers.1.layer.1.convolution", (512, 512, 3, 3)),
]

MLP_LAYERS = [("fc1", (128, 784)), ("fc2", (10, 128))]

# FLAGS.threshold * 100 for the reference's sweep (main_pruning.py:185-186, experiment_log.csv)
REFERENCE_PCT_SWEEP = [t * 100 for t in (0.1, 0.236, 0.382, 0.5, 0.618, 0.786, 0.9, 1.0)]

SIGMA_Z = 2.0 ** 22 / math.sqrt(3.0)
_MASK64 = (1 << 64) - 1
_GAMMA = 0x9E3779B97F4A7C15


def sigma_exponent(sigma):
    """e such that ldexp(z, -e) has standard deviation ~sigma (z: the Irwin-Hall integer)."""
    return int(math.floor(math.log2(SIGMA_Z / sigma) + 0.5))


def conv_sigma(shape):
    # kaiming_normal_(mode='fan_out') as HF ResNet initialises Conv2d weights
    fan_out = shape[0] * int(np.prod(shape[2:])) if len(shape) > 2 else shape[0]
    return math.sqrt(2.0 / fan_out)


def _splitmix64(x):
    z = x + np.uint64(_GAMMA)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def synth_numpy(shape, seed, tensor_id, e):
    """NumPy restatement of wt_synth_value (csrc/wt_synth.h), element k in C order."""
    n = int(np.prod(shape)) if len(shape) else 1
    with np.errstate(over="ignore"):
        k = np.arange(n, dtype=np.uint64)
        key = np.uint64((seed << 40) & _MASK64) ^ np.uint64((tensor_id << 32) & _MASK64) ^ k
        z = np.zeros(n, np.int64)
        for i in range(4):
            h = _splitmix64(key + np.uint64((i * _GAMMA) & _MASK64))
            z += (h >> np.uint64(42)).astype(np.int64)
    z -= 1 << 23
    return (z.astype(np.float32) * np.float32(2.0 ** -e)).reshape(shape)


def resnet18_tensors(seed=0):
    """[(name, shape, seed, tensor_id, e)] for cfg2."""
    return [(name, shape, seed, i, sigma_exponent(conv_sigma(shape)))
            for i, (name, shape) in enumerate(RESNET18_CONVS)]


def mlp_tensors(seed=3):
    return [(name, shape, seed, i, sigma_exponent(1.0 / math.sqrt(shape[1])))
            for i, (name, shape) in enumerate(MLP_LAYERS)]


def block_tensors(nblocks, side=4096, seed=5):
    e = sigma_exponent(math.sqrt(2.0 / side))
    return [("block%d" % i, (side, side), seed, i, e) for i in range(nblocks)]


CONFIGS = {
    "cfg1": dict(wavelet="haar", level=1, pct=50.0,
                 tensors=lambda: [("conv", (64, 64, 3, 3), 1, 0, sigma_exponent(conv_sigma((64, 64, 3, 3))))]),
    "cfg2": dict(wavelet="bior3.3", level=5, pct=50.0, tensors=lambda: resnet18_tensors(0)),
    "cfg3": dict(wavelet="rbio2.2", level=3, pct=50.0, tensors=lambda: mlp_tensors(3)),
    "cfg5": dict(wavelet="db8", level=5, pct=50.0, tensors=lambda: block_tensors(64)),
}


def lpt_shard(sizes, world):
    """Longest-processing-time bin packing of tensors (by numel) onto `world` ranks.
    Deterministic: ties broken by tensor index; every rank computes the same table."""
    order = sorted(range(len(sizes)), key=lambda i: (-sizes[i], i))
    loads = [0] * world
    owner = [0] * len(sizes)
    for i in order:
        r = min(range(world), key=lambda j: (loads[j], j))
        owner[i] = r
        loads[r] += sizes[i]
    return owner, loads
