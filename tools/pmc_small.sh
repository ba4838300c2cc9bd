#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_small
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_IFETCH" "SQC_ICACHE_MISSES SQC_ICACHE_HITS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$ROOT/bench.py" --config cfg3 --steps 20 --warmup 3 --no-cpu --no-cold --no-rocprof --no-graph > "$OUT/p$i.log" 2>&1 \
      || { echo "pass $i ($grp) failed"; tail -5 "$OUT/p$i.log"; }
done
python3 - <<'PY'
import csv, glob, collections, os
root = os.environ.get("GRAFT_REPO_ROOT", ".") + "/gpurun_out/pmc_small"
for f in sorted(glob.glob(root + "/p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "k_small" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        print(k, len(v), sum(v) / max(1, len(v)))
PY
