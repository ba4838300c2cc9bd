#!/bin/bash
# Round-4 measurement, part 1: smoke, the -m gpu suite, the bench lines (cfg2 default, cfg3, cfg5)
# and a rocprofv3 kernel trace of the cfg2 and cfg3 loops.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_r04a.sh TAG
set -o pipefail
TAG=${1:-r04}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 || { echo smoke failed; tail -30 "$OUT/smoke_$TAG.log"; exit 1; }
tail -2 "$OUT/smoke_$TAG.log"
echo "== pytest -m gpu"; timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1 || { echo gpu tests failed; grep -E "^FAILED|passed|failed" "$OUT/pytest_gpu_$TAG.log" | tail; exit 1; }
tail -1 "$OUT/pytest_gpu_$TAG.log"
for c in cfg2 cfg3 cfg5; do
  timeout -k 10 400 python bench.py --config $c > "$OUT/bench_${c}_$TAG.log" 2>&1 || { echo "bench $c failed"; tail -30 "$OUT/bench_${c}_$TAG.log"; exit 1; }
  tail -1 "$OUT/bench_${c}_$TAG.log" | cut -c1-300
done
for c in cfg2 cfg3; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${c}_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config $c --steps 100 --warmup 5 --no-cpu --no-cold --no-rocprof --stage-reps 5 > "$OUT/bench_prof_${c}_$TAG.log" 2>&1 || { echo "rocprof $c failed"; tail -30 "$OUT/bench_prof_${c}_$TAG.log"; exit 1; }
  head -4 "$OUT/prof_${c}_$TAG/run_kernel_stats.csv" | cut -d, -f1-4 | cut -c1-160
done
echo done
