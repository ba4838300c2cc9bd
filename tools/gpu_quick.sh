#!/bin/bash
# Quick GPU iteration: resident parity tests, the full GPU suite, bench in both level-0 forms.
# Usage: gpurun --timeout 900 -- bash tools/gpu_quick.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-q}
K=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== resident tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -v --timeout 120 --timeout-method thread ${K:+-k "$K"} > "$OUT/res_$TAG.log" 2>&1 || { echo resident tests failed; tail -60 "$OUT/res_$TAG.log"; exit 1; }
tail -3 "$OUT/res_$TAG.log"
echo "== all gpu tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_$TAG.log" 2>&1 || { echo gpu tests failed; tail -60 "$OUT/gpu_$TAG.log"; exit 1; }
tail -3 "$OUT/gpu_$TAG.log"
echo "== bench resident"
timeout -k 10 300 python bench.py --no-cpu > "$OUT/bench_res_$TAG.log" 2>&1 || { echo bench failed; tail -30 "$OUT/bench_res_$TAG.log"; exit 1; }
tail -1 "$OUT/bench_res_$TAG.log"
echo "== bench three-launch"
timeout -k 10 300 python bench.py --no-cpu --no-resident > "$OUT/bench_3l_$TAG.log" 2>&1 || { echo bench failed; tail -30 "$OUT/bench_3l_$TAG.log"; exit 1; }
tail -1 "$OUT/bench_3l_$TAG.log"
echo "== rocprof"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 100 --warmup 5 --no-cpu --stage-reps 5 > "$OUT/bench_prof_$TAG.log" 2>&1 || { echo rocprof failed; tail -30 "$OUT/bench_prof_$TAG.log"; exit 1; }
head -5 "$OUT/prof_$TAG/run_kernel_stats.csv"
