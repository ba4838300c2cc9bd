#!/bin/bash
# One GPU round: smoke, GPU parity tests, the benches (cfg2 / cfg3 / cfg5), rocprofv3 kernel traces
# and PMC passes of cfg2 and cfg5.
# Usage (from this container): gpurun --timeout 1200 -- bash tools/gpu_check.sh [tag]
set -o pipefail
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 || { echo smoke failed; tail -30 "$OUT/smoke_$TAG.log"; exit 1; }
tail -2 "$OUT/smoke_$TAG.log"
echo "== pytest -m gpu"; timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu_$TAG.log" 2>&1 || { echo gpu tests failed; tail -40 "$OUT/pytest_gpu_$TAG.log"; exit 1; }
tail -3 "$OUT/pytest_gpu_$TAG.log"
echo "== bench"; timeout -k 10 600 python bench.py > "$OUT/bench_$TAG.log" 2>&1 || { echo bench failed; tail -30 "$OUT/bench_$TAG.log"; exit 1; }
tail -1 "$OUT/bench_$TAG.log"
echo "== rocprofv3"; cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 100 --warmup 5 --no-cpu --stage-reps 5 > "$OUT/bench_prof_$TAG.log" 2>&1 || { echo rocprof failed; tail -30 "$OUT/bench_prof_$TAG.log"; exit 1; }
find "$OUT/prof_$TAG" -name "*stats*" | head
echo "== pmc"; cd "$ROOT" && timeout -k 10 900 bash tools/pmc_run.sh "$TAG" > "$OUT/pmc_$TAG.log" 2>&1 || { echo pmc failed; tail -20 "$OUT/pmc_$TAG.log"; exit 1; }
python3 tools/pmc_summary.py "$OUT/pmc_$TAG" "$OUT/pmc_${TAG}_cfg2.json" "$TAG" || exit 1
echo "== cfg3 / cfg5 benches"
for c in cfg3 cfg5; do
  timeout -k 10 300 python bench.py --config $c > "$OUT/bench_${c}_$TAG.log" 2>&1 || { echo "bench $c failed"; tail -30 "$OUT/bench_${c}_$TAG.log"; exit 1; }
  tail -1 "$OUT/bench_${c}_$TAG.log"
done
echo "== cfg5 rocprofv3"; cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_cfg5_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg5 --steps 20 --warmup 3 --no-cpu > "$OUT/bench_prof_cfg5_$TAG.log" 2>&1 || { echo rocprof cfg5 failed; tail -30 "$OUT/bench_prof_cfg5_$TAG.log"; exit 1; }
echo "== cfg5 pmc"; cd "$ROOT" && timeout -k 10 900 bash tools/pmc_run.sh "cfg5_$TAG" --config cfg5 > "$OUT/pmc_cfg5_$TAG.log" 2>&1 || { echo pmc cfg5 failed; tail -20 "$OUT/pmc_cfg5_$TAG.log"; exit 1; }
python3 tools/pmc_summary.py "$OUT/pmc_cfg5_$TAG" "$OUT/pmc_${TAG}_cfg5.json" "$TAG" || exit 1
echo done
