#!/bin/bash
# Round-4 measurement, part 3: the cfg5 bench line again (its PMC traffic now read from the
# committed summary) and a 2-rank rehearsal of the N > 1 path.
# Usage: gpurun --timeout 900 -- bash tools/gpu_r04c.sh TAG
set -o pipefail
TAG=${1:-r04c}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== bench cfg5"; timeout -k 10 400 python bench.py --config cfg5 --steps 20 --warmup 3 > "$OUT/bench_cfg5_$TAG.log" 2>&1 || { echo bench cfg5 failed; tail -30 "$OUT/bench_cfg5_$TAG.log"; exit 1; }
tail -1 "$OUT/bench_cfg5_$TAG.log" | cut -c1-300
echo "== rehearsal --gpus 2"; WTP_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --steps 40 --warmup 5 > "$OUT/bench_n2_$TAG.log" 2>&1 || { echo rehearsal failed; tail -30 "$OUT/bench_n2_$TAG.log"; exit 1; }
grep '"metric"' "$OUT/bench_n2_$TAG.log" | cut -c1-400
echo done
