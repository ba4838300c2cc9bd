#!/bin/bash
# Cold-Infinity-Cache profiles of the cfg2 prune (tools/cold_run.py): one kernel trace with stats
# and the FETCH_SIZE / WRITE_SIZE PMC passes.  Usage: gpurun -- bash tools/gpu_cold.sh TAG
set -o pipefail
TAG=${1:-cold}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT/pmc_$TAG"
export TMPDIR=/tmp
cd /tmp
echo "== kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- python3 "$ROOT/tools/cold_run.py" --steps 60 > "$OUT/cold_$TAG.log" 2>&1 || { echo trace failed; tail -20 "$OUT/cold_$TAG.log"; exit 1; }
grep -E "Name|k_resident|Fill" "$OUT/prof_$TAG/run_kernel_stats.csv" | cut -c1-200
echo "== kernel trace, read flush"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${TAG}_rd" -o run --output-format csv -- python3 "$ROOT/tools/cold_run.py" --steps 60 --flush read > "$OUT/cold_${TAG}_rd.log" 2>&1 || { echo trace failed; tail -20 "$OUT/cold_${TAG}_rd.log"; exit 1; }
grep -E "Name|k_resident" "$OUT/prof_${TAG}_rd/run_kernel_stats.csv" | cut -c1-200
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/pmc_$TAG/p$i" -o run -- python3 "$ROOT/tools/cold_run.py" --steps 20 > "$OUT/pmc_$TAG/p$i.log" 2>&1 || { echo "pmc $grp failed"; tail -20 "$OUT/pmc_$TAG/p$i.log"; exit 1; }
done
cd "$ROOT" && python3 tools/pmc_summary.py "$OUT/pmc_$TAG" "$OUT/pmc_${TAG}_cfg2.json" "$TAG" && echo done
