#!/bin/bash
# k_resident iteration: resident parity tests, the phase lab, the cfg2 bench and a kernel trace.
# Usage: gpurun --timeout 600 -- bash tools/gpu_res.sh TAG
set -o pipefail
TAG=${1:-res}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== resident tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -q --timeout 120 --timeout-method thread > "$OUT/res_$TAG.log" 2>&1 || { echo resident tests failed; tail -60 "$OUT/res_$TAG.log"; exit 1; }
tail -2 "$OUT/res_$TAG.log"
echo "== reslab"
timeout -k 10 120 ./tools/mb/reslab 50 "$OUT/reslab_$TAG.csv" > "$OUT/reslab_$TAG.log" 2>&1 || { echo reslab failed; tail -20 "$OUT/reslab_$TAG.log"; exit 1; }
grep -v "184466" "$OUT/reslab_$TAG.log"
echo "== rocprof cfg2"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 200 --warmup 5 --no-cpu --no-cold --no-rocprof --stage-reps 2 > "$OUT/bench_prof_$TAG.log" 2>&1 || { echo rocprof failed; tail -30 "$OUT/bench_prof_$TAG.log"; exit 1; }
head -3 "$OUT/prof_$TAG/run_kernel_stats.csv" | cut -c1-200
tail -1 "$OUT/bench_prof_$TAG.log" | cut -c1-400
