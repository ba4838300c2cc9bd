#!/bin/bash
# cfg5 filter-bank profile: kernel trace + stats of the bench loop with the interior kernels on and
# off, then one PMC pass (SQ counters) over the interior-on run.
# Usage: gpurun --timeout 900 -- bash tools/gpu_fbprof.sh TAG
set -o pipefail
TAG=${1:-fbp}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for v in int gen; do
  F=""; [ $v = gen ] && F=--no-interior
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/fbp_${TAG}_$v -o run --output-format csv -- python3 $ROOT/bench.py --config cfg5 --steps 4 --warmup 1 --replays 2 --stage-reps 2 --no-cpu --no-cold --no-rocprof --no-graph $F > $OUT/fbp_${TAG}_$v.log 2>&1 || { echo "rocprof $v failed"; tail -20 $OUT/fbp_${TAG}_$v.log; exit 1; }
  echo "== $v"; head -14 $OUT/fbp_${TAG}_$v/run_kernel_stats.csv | cut -d, -f1-8 | cut -c1-220
done
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY --kernel-trace --output-format csv -d $OUT/fbp_${TAG}_pmc -o run -- python3 $ROOT/bench.py --config cfg5 --steps 2 --warmup 1 --replays 1 --stage-reps 1 --no-cpu --no-cold --no-rocprof --no-graph > $OUT/fbp_${TAG}_pmc.log 2>&1 || { echo "pmc failed"; tail -20 $OUT/fbp_${TAG}_pmc.log; exit 1; }
python3 - <<PY
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob("$OUT/fbp_${TAG}_pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        n = r["Kernel_Name"]
        k = next((x for x in ("k_inv_int", "k_inv_level", "k_fwd_int", "k_fwd_level", "k_collect_t") if x in n), None)
        if k:
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
