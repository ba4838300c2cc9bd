"""Per-segment phase summary of a tools/mb/reslab per-workgroup CSV (cfg2 layout, RES_CHUNK blocks)."""
import csv
import math
import sys

SHAPES = [(64, 3, 7, 7), (64, 64, 3, 3), (64, 64, 3, 3), (64, 64, 3, 3), (64, 64, 3, 3), (128, 64, 1, 1),
          (128, 64, 3, 3), (128, 128, 3, 3), (128, 128, 3, 3), (128, 128, 3, 3), (256, 128, 1, 1), (256, 128, 3, 3),
          (256, 256, 3, 3), (256, 256, 3, 3), (256, 256, 3, 3), (512, 256, 1, 1), (512, 256, 3, 3), (512, 512, 3, 3),
          (512, 512, 3, 3), (512, 512, 3, 3)]
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 49152
rows = list(csv.DictReader(open(sys.argv[1])))
seg = []
for t, s in enumerate(SHAPES):
    seg += [t] * (-(-math.prod(s) // chunk))
by = {}
for r in rows:
    by.setdefault(seg[int(r["wg"])], []).append(r)
for t in sorted(by):
    rs = by[t]
    mx = lambda k: max(float(x[k]) for x in rs)
    md = lambda k: sorted(float(x[k]) for x in rs)[len(rs) // 2]
    print("%2d %-16s %3d %-5s counted max %5.1f  arrive max %5.1f  pass med %5.1f  selected max %5.1f  stored max %5.1f"
          % (t, SHAPES[t], len(rs), "late" if rs[0]["late"] == "1" else "early", mx("counted"), mx("B1-arrive"),
             md("B1-pass"), mx("selected"), mx("stored")))
