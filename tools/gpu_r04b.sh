#!/bin/bash
# Round-4 measurement, part 2: rocprofv3 kernel trace of the cfg5 loop (levels split by launch),
# then the PMC passes of cfg2, cfg3 and cfg5 (tools/pmc_run.sh) and their summaries.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_r04b.sh TAG
set -o pipefail
TAG=${1:-r04}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== cfg5 rocprofv3"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_cfg5_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg5 --steps 4 --warmup 1 --replays 2 --stage-reps 2 --no-cpu --no-cold --no-rocprof --no-graph > "$OUT/bench_prof_cfg5_$TAG.log" 2>&1 || { echo rocprof cfg5 failed; tail -30 "$OUT/bench_prof_cfg5_$TAG.log"; exit 1; }
head -8 "$OUT/prof_cfg5_$TAG/run_kernel_stats.csv" | cut -d, -f1-4 | cut -c1-160
cd "$ROOT"
for c in cfg2 cfg3 cfg5; do
  echo "== pmc $c"
  timeout -k 10 700 bash tools/pmc_run.sh "${c}_$TAG" --config $c > "$OUT/pmc_${c}_$TAG.log" 2>&1 || { echo "pmc $c failed"; tail -20 "$OUT/pmc_${c}_$TAG.log"; exit 1; }
  python3 tools/pmc_summary.py "$OUT/pmc_${c}_$TAG" "$OUT/pmc_${TAG}_$c.json" "$TAG" || exit 1
done
echo done
