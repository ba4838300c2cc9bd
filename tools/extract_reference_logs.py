"""Copy the reference's own recorded outputs for this path into a committed fixture.

The reference publishes what its DWT-pruning path produced on the real ResNet-18 weights
(which are not available offline): per-layer counts in
  ResNet/StoredModels/<wavelet>_threshold-<t>_level-<L>_guid-<g>/{selective,min,random}_pruned/log.csv
(schema utils.py:55-58) and run totals in ResNet/experiment_log.csv:739-786 (schema
utils.py:127-128).  This script reads those CSV data files and writes
tests/golden/reference_logs.json.  Run here (the GPU box has no /root/reference):
    python3 tools/extract_reference_logs.py
"""
import csv
import glob
import json
import os

REF = "/root/reference/ResNet"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    out = {"stored_models": {}, "experiment_log": []}
    for d in sorted(glob.glob(os.path.join(REF, "StoredModels", "*"))):
        run = os.path.basename(d)
        out["stored_models"][run] = {}
        for phase in ("selective_pruned", "min_pruned", "random_pruned"):
            p = os.path.join(d, phase, "log.csv")
            if not os.path.exists(p):
                continue
            with open(p, newline="") as fh:
                rows = list(csv.DictReader(fh))
            out["stored_models"][run][phase] = [
                {"layer": r["Layer Name"], "n": int(r["Original Parameter Count"]),
                 "nonzero": int(r["Non-zero Params"]), "pruned": int(r["Total Pruned Count"]),
                 "threshold": float(r["Threshold"]), "wavelet": r["Wavelet"], "level": int(r["Level"])}
                for r in rows]
    with open(os.path.join(REF, "experiment_log.csv"), newline="") as fh:
        lines = list(csv.reader(fh))
    for lineno in range(739, 787):  # 1-based line numbers of the bior1.3 / bior4.4 L5 sweep
        r = lines[lineno - 1]
        out["experiment_log"].append({"line": lineno, "guid": r[0], "wavelet": r[1], "level": int(r[2]),
                                      "threshold": float(r[3]), "phase": r[4],
                                      "total_pruned": int(r[5]), "total_nonzero": int(r[6])})
    with open(os.path.join(ROOT, "tests", "golden", "reference_logs.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
