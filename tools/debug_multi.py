import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from tests import golden_io as G
from wavelettransforms_amd import engine
from oracle import oracle as O
arrs = G.arrays()
recs = G.manifest()["multi"]["haar_L5_p50"]
xs = [torch.from_numpy(arrs["multi/in%d" % j]).cuda() for j in range(len(recs))]
outs, res = engine.prune(xs, "haar", 5, 50.0, carry_level=True)
for j in range(len(recs)):
    o1, r1 = engine.prune([xs[j]], "haar", recs[j]["eff_level"], 50.0)
    g = arrs["multi/out%d" % j]
    a = outs[j].cpu().numpy(); b = o1[0].cpu().numpy()
    print(j, xs[j].shape, "batch==golden", np.array_equal(a, g), "single==golden", np.array_equal(b, g),
          "thr batch", res[j]["thr64"], "single", r1[0]["thr64"], "golden", recs[j]["thr64"], "path", res[j]["path"], r1[0]["path"])
    if not np.array_equal(a, g):
        d = np.argwhere(a != g)
        print("  ndiff", len(d), d[:5], a[tuple(d[0])], g[tuple(d[0])])
