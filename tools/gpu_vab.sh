#!/bin/bash
# A/B of lab library variants on cfg2 (k_resident): resident parity tests per variant, then the
# cfg2 bench per variant, alternated twice.  A variant is NAME or NAME:ENV=VAL (extra env for it);
# NAME "prod" is the product library.
# Usage: gpurun --timeout 900 -- bash tools/gpu_vab.sh TAG v1 v2 ...
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/vab_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run_env() { # $1 = variant spec; prints the env assignments
  local n=${1%%:*} e=""
  [ "$n" != "$1" ] && e=${1#*:}
  if [ "$n" = prod ]; then echo "$e"; else echo "WTP_LIB_PATH=$ROOT/tools/mb/libwtprune_$n.so $e"; fi
}
for v in "$@"; do
  env $(run_env "$v") timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -q --timeout 120 --timeout-method thread \
      > "$OUT/t_${v//[:=]/_}.log" 2>&1 || { echo "tests failed for $v"; tail -40 "$OUT/t_${v//[:=]/_}.log"; exit 1; }
  echo "$v tests: $(tail -1 "$OUT/t_${v//[:=]/_}.log")"
done
for rep in 1 2; do
  for v in "$@"; do
    f="$OUT/b_${v//[:=]/_}_$rep.log"
    env $(run_env "$v") timeout -k 10 300 python bench.py --no-cpu --no-cold --steps 200 > "$f" 2>&1 || { echo "bench failed for $v"; tail -20 "$f"; exit 1; }
    python3 -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']
print(sys.argv[2], 'us/step %.2f' % (d['ms_per_step']*1e3), r['kernel'], 'rocprof %.2f' % r['avg_launch_us'], 'stamps %s' % r.get('avg_launch_us_stamps'), 'valid', d.get('valid', True))" "$f" "$v"
  done
done
