#!/bin/bash
# One GPU verification pass: smoke, the whole -m gpu suite, the PMC passes (cfg2 / cfg3 / cfg5,
# copied into the box's profiles/ so the bench lines below cite this run's counters), the benches
# (cfg2 default line, cfg3, cfg5), a 2-rank rehearsal of the N > 1 path, and kernel traces.
# PART=a: smoke, tests and PMC only; PART=b: benches and traces only (two calls under gpurun's limit).
# Usage: gpurun --timeout 1200 -- bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-r}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${PART:-ab}" != b ]; then
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 || { echo smoke failed; tail -30 "$OUT/smoke_$TAG.log"; exit 1; }
tail -1 "$OUT/smoke_$TAG.log"
echo "== pytest -m gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1 || { echo gpu tests failed; tail -60 "$OUT/pytest_gpu_$TAG.log"; exit 1; }
tail -2 "$OUT/pytest_gpu_$TAG.log"
echo "== pmc cfg2"; cd "$ROOT" && timeout -k 10 600 bash tools/pmc_run.sh "$TAG" > "$OUT/pmc_$TAG.log" 2>&1 || { echo pmc failed; tail -20 "$OUT/pmc_$TAG.log"; exit 1; }
python3 tools/pmc_summary.py "$OUT/pmc_$TAG" "$OUT/pmc_${TAG}_cfg2.json" "$TAG" || exit 1
echo "== pmc cfg3"; timeout -k 10 600 bash tools/pmc_run.sh "${TAG}c3" --config cfg3 > "$OUT/pmc_${TAG}c3.log" 2>&1 || { echo pmc cfg3 failed; tail -20 "$OUT/pmc_${TAG}c3.log"; exit 1; }
python3 tools/pmc_summary.py "$OUT/pmc_${TAG}c3" "$OUT/pmc_${TAG}_cfg3.json" "${TAG}c3" || exit 1
echo "== pmc cfg5"; timeout -k 10 900 bash tools/pmc_run.sh "${TAG}c5" --config cfg5 --steps 3 --warmup 1 > "$OUT/pmc_${TAG}c5.log" 2>&1 || { echo pmc cfg5 failed; tail -20 "$OUT/pmc_${TAG}c5.log"; exit 1; }
python3 tools/pmc_summary.py "$OUT/pmc_${TAG}c5" "$OUT/pmc_${TAG}_cfg5.json" "${TAG}c5" || exit 1
for c in 2 3 5; do [ -f "$OUT/pmc_${TAG}_cfg$c.json" ] && cp "$OUT/pmc_${TAG}_cfg$c.json" "$ROOT/profiles/pmc_cfg$c.json"; done
cd "$ROOT"
fi
if [ "${PART:-ab}" != a ]; then
cd "$ROOT"
echo "== bench cfg2"; timeout -k 10 300 python bench.py > "$OUT/bench_cfg2_$TAG.log" 2>&1 || { echo bench failed; tail -30 "$OUT/bench_cfg2_$TAG.log"; exit 1; }
tail -1 "$OUT/bench_cfg2_$TAG.log"
echo "== bench cfg3"; timeout -k 10 300 python bench.py --config cfg3 > "$OUT/bench_cfg3_$TAG.log" 2>&1 || { echo bench cfg3 failed; tail -30 "$OUT/bench_cfg3_$TAG.log"; exit 1; }
tail -1 "$OUT/bench_cfg3_$TAG.log" | cut -c1-600
echo "== bench cfg5"; WTP_BENCH_TRACE_DIR="$OUT/trace5_$TAG" timeout -k 10 400 python bench.py --config cfg5 --steps 20 --warmup 3 > "$OUT/bench_cfg5_$TAG.log" 2>&1 || { echo bench cfg5 failed; tail -30 "$OUT/bench_cfg5_$TAG.log"; exit 1; }
tail -1 "$OUT/bench_cfg5_$TAG.log" | cut -c1-600
echo "== rehearsal --gpus 2"; WTP_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --steps 40 --warmup 5 > "$OUT/bench_n2_$TAG.log" 2>&1 || { echo rehearsal failed; tail -30 "$OUT/bench_n2_$TAG.log"; exit 1; }
grep '"metric"' "$OUT/bench_n2_$TAG.log" | cut -c1-400
echo "== rehearsal --gpus 2 --exchange allgather"; WTP_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --steps 40 --warmup 5 --exchange allgather > "$OUT/bench_n2ag_$TAG.log" 2>&1 || { echo rehearsal allgather failed; tail -30 "$OUT/bench_n2ag_$TAG.log"; exit 1; }
grep '"metric"' "$OUT/bench_n2ag_$TAG.log" | cut -c1-400
echo "== rocprof cfg2"; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 400 --warmup 5 --no-cpu --no-cold --no-rocprof > "$OUT/bench_prof_$TAG.log" 2>&1 || { echo rocprof failed; tail -30 "$OUT/bench_prof_$TAG.log"; exit 1; }
head -3 "$OUT/prof_$TAG/run_kernel_stats.csv" | cut -c1-200
echo "== rocprof cfg3"; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof3_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg3 --steps 400 --warmup 5 --no-cpu --no-cold --no-rocprof > "$OUT/bench_prof3_$TAG.log" 2>&1 || { echo rocprof cfg3 failed; tail -30 "$OUT/bench_prof3_$TAG.log"; exit 1; }
head -3 "$OUT/prof3_$TAG/run_kernel_stats.csv" | cut -c1-200
fi
echo done
