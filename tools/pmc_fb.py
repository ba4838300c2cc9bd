"""Per-(kernel, grid) averages of the SQ counters collected by tools/pmc_fb.sh (lab)."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for p in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    with open(p) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if "wtp::" not in name:
                continue
            grid = int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"]))
            acc[(name, grid)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for p in sorted(glob.glob(os.path.join(d, "p*", "run_kernel_trace.csv"))):
    with open(p) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
            dur[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
for key in sorted(acc, key=lambda k: -sum(dur.get(k, [0])) / max(1, len(dur.get(k, [1])))):
    c = acc[key]
    us = sum(dur[key]) / len(dur[key]) if dur.get(key) else 0.0
    row = {k: sum(v) / len(v) for k, v in c.items()}
    print("%-32s wgs %6d  %8.1f us  " % (key[0][:32], key[1], us) +
          "  ".join("%s=%.3g" % (k.replace("SQ_", ""), v) for k, v in sorted(row.items())))
