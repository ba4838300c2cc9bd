"""k_resident's sample positions (csrc/kernels.hip res_body P0, host csrc/api.hip res_step_fx):
group g of SAMPLE_GROUP contiguous keys starts at floor(g (n - 16) / 255), computed on the device
as floor(g * step_fx / 2^32) from a 32.32 fixed-point step the host rounds up.  Restated here
over many segment sizes: every start is the exact floor and every position lies in [0, n)."""
import numpy as np

RES_MS, SAMPLE_GROUP = 4096, 16
D = RES_MS // SAMPLE_GROUP - 1


def step_fx(n):  # csrc/api.hip: rounded up
    return (((n - SAMPLE_GROUP) << 32) + (D - 1)) // D


def positions(n):
    fx = step_fx(n)
    lo, hi = fx & 0xFFFFFFFF, fx >> 32
    g = np.arange(D + 1, dtype=np.uint64)
    start = ((g * np.uint64(lo)) >> np.uint64(32)) + g * np.uint64(hi)  # __umulhi(g, lo) + g * hi
    return start, g


def test_sample_starts_exact_and_in_range():
    rng = np.random.default_rng(3)
    sizes = list(range(RES_MS + 1, RES_MS + 600)) + [36864, 73728, 147456, 294912, 589824, 1179648, 2359296]
    sizes += [int(x) for x in rng.integers(RES_MS + 1, 1 << 31, 400)]
    sizes += [k * D + SAMPLE_GROUP for k in range(17, 60)]  # step exact in 32.32
    for n in sizes:
        start, g = positions(n)
        exact = (g.astype(object) * (n - SAMPLE_GROUP)) // D
        assert [int(x) for x in start] == list(exact), n
        assert int(start.max()) + SAMPLE_GROUP - 1 <= n - 1 and int(start.min()) >= 0, n
