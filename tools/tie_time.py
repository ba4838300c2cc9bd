"""Time one call on tie-heavy input (integer-valued floats in {-2..2}: the buckets overflow and the
select takes its exact full scan) -- 4 x 4096^2 db8 L5 p50, fused and unfused; prints ms per call
and the records' paths.  Lab: tools/gpu_tie.sh runs it against two libraries."""
import sys
import time

import torch

sys.path.insert(0, ".")
from wavelettransforms_amd import engine  # noqa: E402

g = torch.Generator(device="cpu").manual_seed(1)
xs = [torch.randint(-2, 3, (4096, 4096), generator=g).float().cuda() for _ in range(4)]
for fused in (True, False):
    engine.set_fused_select(fused)
    outs, res = engine.prune(xs, "db8", 5, 50.0, carry_level=False)
    torch.cuda.synchronize()
    t = []
    for _ in range(3):
        t0 = time.perf_counter()
        outs, res = engine.prune(xs, "db8", 5, 50.0, carry_level=False)
        torch.cuda.synchronize()
        t.append((time.perf_counter() - t0) * 1e3)
    print("fused" if fused else "unfused", "%.2f ms / call (min of 3)" % min(t), "paths", [r["path"] for r in res])
