#!/bin/bash
# A/B of k_resident variants (env knobs read by launch_resident): resident parity tests under
# each variant, then the cfg2 bench per variant (ms/step and the k_resident stage time).
# Usage: gpurun --timeout 900 -- bash tools/gpu_ab.sh TAG "OPTS:SIGMA" ["OPTS:SIGMA" ...]
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in "$@"; do
  export WTP_RES_OPTS=${v%%:*} WTP_RES_SIGMA=${v##*:}
  timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -q --timeout 120 --timeout-method thread \
      > "$OUT/ab_${TAG}_$v.log" 2>&1 || { echo "tests failed for $v"; tail -40 "$OUT/ab_${TAG}_$v.log"; exit 1; }
  echo "$v tests: $(tail -1 "$OUT/ab_${TAG}_$v.log")"
done
for rep in 1 2; do
  for v in "$@"; do
    export WTP_RES_OPTS=${v%%:*} WTP_RES_SIGMA=${v##*:}
    timeout -k 10 300 python bench.py --no-cpu --steps 1000 > "$OUT/abb_${TAG}_$v.log" 2>&1 || { echo "bench failed for $v"; tail -20 "$OUT/abb_${TAG}_$v.log"; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'ms/step %.5f'%d['ms_per_step'], 'stage', {k: round(v,2) for k,v in d['stage_us'].items()})" "$OUT/abb_${TAG}_$v.log" "$v"
  done
done
