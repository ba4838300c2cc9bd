#!/bin/bash
# Round-4 end, cfg5 only: rocprofv3 kernel trace of the bench loop and the PMC passes.
# Usage: gpurun --timeout 1100 -- bash tools/gpu_r04e.sh TAG
set -o pipefail
TAG=${1:-r04e}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_cfg5_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg5 --steps 4 --warmup 1 --replays 2 --stage-reps 2 --no-cpu --no-cold --no-rocprof --no-graph > "$OUT/bench_prof_cfg5_$TAG.log" 2>&1 || { echo rocprof cfg5 failed; tail -30 "$OUT/bench_prof_cfg5_$TAG.log"; exit 1; }
cd "$ROOT"
timeout -k 10 700 bash tools/pmc_run.sh "cfg5_$TAG" --config cfg5 > "$OUT/pmc_cfg5_$TAG.log" 2>&1 || { echo "pmc cfg5 failed"; tail -20 "$OUT/pmc_cfg5_$TAG.log"; exit 1; }
python3 tools/pmc_summary.py "$OUT/pmc_cfg5_$TAG" "$OUT/pmc_${TAG}_cfg5.json" "$TAG" || exit 1
echo done
