"""Lab: the exact full-scan select on tied ranks -- a level-0 1x1 conv weight (k_mask_select: every
block selects) and a 4096^2 haar L1 tensor whose level-1 approximation holds half +-1.0 ties at
p90 (one select block per segment); prints path and ms per call (resident launch off)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from wavelettransforms_amd import engine  # noqa: E402

g = torch.Generator(device="cpu").manual_seed(9)


def tied(shape):
    xn = torch.randn(shape, generator=g) * 0.3
    tie = torch.rand(shape, generator=g) < 0.5
    xn[tie] = torch.where(torch.rand(int(tie.sum()), generator=g) < 0.5, 1.0, -1.0)
    return xn


engine.set_resident(False)
x0 = tied((1024, 4096, 1, 1)).cuda()
x2 = tied((2048, 2048)).repeat_interleave(2, 0).repeat_interleave(2, 1).mul_(0.5).cuda()
for name, x, wav, lv, pct in (("level0", x0, "haar", 3, 50.0), ("dwt", x2, "haar", 1, 90.0)):
    for fused in (False, True):
        engine.set_fused_select(fused)
        for rep in range(2):
            t0 = time.perf_counter()
            o, r = engine.prune([x], wav, lv, pct, carry_level=False)
            torch.cuda.synchronize()
            print(name, "fused" if fused else "unfused", "path", r[0]["path"], "%.2f ms" % ((time.perf_counter() - t0) * 1e3))
