#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (tools/pmc_run.sh) into per-kernel bytes per launch.

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB per dispatch and count the L2's
memory-side (fabric) requests, Infinity-Cache hits included (MI355X_MICROARCH.md, HBM).
gfx950 correction from the same section: FETCH_SIZE counts 128-B read requests at 64 B, so it
is doubled for the wide (16 B/lane) streaming reads these kernels issue; WRITE_SIZE is exact
for 16-B streaming stores.

Usage: python tools/pmc_summary.py gpurun_out/pmc_TAG profiles/pmc_cfg2.json [label]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

KERNELS = ["k_resident", "k_small", "k_mask_select", "k_mask_inplace", "k_collect_t", "k_collect_retry", "k_window",
           "k_fwin", "k_fslot_collect", "k_fwd_level", "k_inv_level",
           "k_fwd_int", "k_inv_int", "k_dwt_cols", "k_dwt_rows",
           "k_idwt_rows", "k_idwt_cols", "k_copy_threshold"]


def short(name):
    for k in KERNELS:  # exact identifier match (k_mask_select is not k_mask)
        if re.search(r"(?<![A-Za-z0-9_])%s(?![A-Za-z0-9_])" % re.escape(k), name):
            return k
    return None


def main():
    src, dst = sys.argv[1], sys.argv[2]
    label = sys.argv[3] if len(sys.argv) > 3 else os.path.basename(src.rstrip("/"))
    acc = defaultdict(lambda: defaultdict(list))
    for path in sorted(glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True)):
        with open(path) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                if k:
                    acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {"source": label, "units": "bytes per launch (mean over launches)",
           "correction": "fetch = 2 x FETCH_SIZE (gfx950 128-B requests tallied at 64 B); write = WRITE_SIZE",
           "note": "memory-side L2 requests: Infinity-Cache hits are included", "kernels": {}}
    for k, ctrs in acc.items():
        d = {}
        mean = lambda v: sum(v) / len(v)
        if "FETCH_SIZE" in ctrs:
            d["fetch_size_kib_raw"] = mean(ctrs["FETCH_SIZE"])
            d["fetch_bytes_per_launch"] = 2.0 * 1024.0 * d["fetch_size_kib_raw"]
        if "WRITE_SIZE" in ctrs:
            d["write_size_kib_raw"] = mean(ctrs["WRITE_SIZE"])
            d["write_bytes_per_launch"] = 1024.0 * d["write_size_kib_raw"]
        for c in ("TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT",
                  "SQ_WAIT_INST_LDS", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAVES"):
            if c in ctrs:
                d[c] = mean(ctrs[c])
        if "fetch_bytes_per_launch" in d and "write_bytes_per_launch" in d:
            d["hbm_bytes_per_launch"] = d["fetch_bytes_per_launch"] + d["write_bytes_per_launch"]
        d["launches"] = max(len(v) for v in ctrs.values())
        out["kernels"][k] = d
    # a filter-bank stage runs as interior and frame dispatches (k_*_int, the frame in k_*_int's
    # edge instance or in the general k_*_level): bench.py names the stage "k_fwd_int+k_fwd_level"
    # and averages over every dispatch of either, so the combined entry is the per-dispatch mean
    for a, b in (("k_fwd_int", "k_fwd_level"), ("k_inv_int", "k_inv_level")):
        parts = [k for k in (out["kernels"].get(a), out["kernels"].get(b)) if k and "hbm_bytes_per_launch" in k]
        if parts:
            n = sum(k["launches"] for k in parts)
            tot = sum(k["hbm_bytes_per_launch"] * k["launches"] for k in parts)
            out["kernels"][a + "+" + b] = {"hbm_bytes_per_launch": tot / n, "launches": n,
                                           "note": "every interior and frame dispatch of the stage, per dispatch"}
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    for k, d in sorted(out["kernels"].items()):
        print("%-24s fetch %10.0f B  write %10.0f B  launches %d" % (k, d.get("fetch_bytes_per_launch", -1),
                                                                   d.get("write_bytes_per_launch", -1), d["launches"]))


if __name__ == "__main__":
    main()
