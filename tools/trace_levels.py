"""Per-launch-shape summary of a rocprofv3 kernel trace (a lab tool): groups the dispatches of
a run_kernel_trace.csv by (kernel, grid size) and prints count, mean and total device time, so
the filter-bank levels of cfg5 (one grid size per level) can be told apart.
Usage: python tools/trace_levels.py gpurun_out/<dir>/run_kernel_trace.csv [--min-us X]"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    min_us = float(sys.argv[sys.argv.index("--min-us") + 1]) if "--min-us" in sys.argv else 0.0
    g = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
            g[(name, grid, r["VGPR_Count"], r["LDS_Block_Size"])].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    rows = sorted(g.items(), key=lambda kv: -sum(kv[1]))
    print("%-40s %8s %5s %6s %6s %10s %10s %10s" % ("kernel", "wgs", "vgpr", "lds", "n", "mean_us", "min_us", "total_ms"))
    for (name, grid, vg, lds), ds in rows:
        if sum(ds) / len(ds) < min_us:
            continue
        print("%-40s %8d %5s %6s %6d %10.1f %10.1f %10.3f" % (name[:40], grid, vg, lds, len(ds), sum(ds) / len(ds),
                                                            min(ds), sum(ds) / 1000.0))


if __name__ == "__main__":
    main()
