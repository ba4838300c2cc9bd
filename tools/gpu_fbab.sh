#!/bin/bash
# Filter-bank A/B: GPU parity of the default build, then the cfg5 / cfg3 stage breakdown for
# each lab build named on the command line (wavelettransforms_amd/_lib/<name>.so via WTP_LIB_PATH).
# Usage: gpurun --timeout 900 -- bash tools/gpu_fbab.sh TAG name [name ...]   (CFGS="cfg2 cfg5" to choose configs)
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/fbab_pytest_$TAG.log" 2>&1 \
    || { echo gpu tests failed; tail -40 "$OUT/fbab_pytest_$TAG.log"; exit 1; }
tail -1 "$OUT/fbab_pytest_$TAG.log"
for v in "$@"; do
  for c in ${CFGS:-cfg5 cfg3}; do
    WTP_LIB_PATH=$ROOT/wavelettransforms_amd/_lib/$v.so timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu \
        > "$OUT/fbab_${TAG}_${v}_$c.log" 2>&1 || { echo "bench $v $c failed"; tail -20 "$OUT/fbab_${TAG}_${v}_$c.log"; exit 1; }
    tail -1 "$OUT/fbab_${TAG}_${v}_$c.log" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$v $c ms/step %.4f' % d['ms_per_step'], {k: round(v,1) for k,v in d['stage_us'].items()})"
  done
done
