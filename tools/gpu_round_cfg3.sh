#!/bin/bash
# cfg3 refresh after a k_small change: smoke, the whole GPU suite, cfg3 PMC (copied into the box's profiles/), the cfg3 bench line and kernel trace.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_round_cfg3.sh TAG
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r05c}
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 || { tail -20 "$OUT/smoke_$TAG.log"; exit 1; }
tail -1 "$OUT/smoke_$TAG.log"
echo "== pytest -m gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1 || { tail -40 "$OUT/pytest_gpu_$TAG.log"; exit 1; }
tail -1 "$OUT/pytest_gpu_$TAG.log"
echo "== pmc cfg3"; timeout -k 10 600 bash tools/pmc_run.sh "${TAG}c3" --config cfg3 > "$OUT/pmc_${TAG}c3.log" 2>&1 || { tail -20 "$OUT/pmc_${TAG}c3.log"; exit 1; }
python3 tools/pmc_summary.py "$OUT/pmc_${TAG}c3" "$OUT/pmc_${TAG}_cfg3.json" "${TAG}c3" || exit 1
cp "$OUT/pmc_${TAG}_cfg3.json" "$ROOT/profiles/pmc_cfg3.json"
echo "== bench cfg3"; timeout -k 10 300 python bench.py --config cfg3 > "$OUT/bench_cfg3_$TAG.log" 2>&1 || { tail -20 "$OUT/bench_cfg3_$TAG.log"; exit 1; }
tail -1 "$OUT/bench_cfg3_$TAG.log" | cut -c1-300
echo "== rocprof cfg3"; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof3_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg3 --steps 400 --warmup 5 --no-cpu --no-cold --no-rocprof > "$OUT/bench_prof3_$TAG.log" 2>&1 || { tail -20 "$OUT/bench_prof3_$TAG.log"; exit 1; }
head -3 "$OUT/prof3_$TAG/run_kernel_stats.csv" | cut -c1-200
