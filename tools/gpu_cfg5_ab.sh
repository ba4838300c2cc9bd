#!/bin/bash
# cfg5 A/B on one box: the filter-bank parity tests, then the cfg5 bench line per bench-flag
# variant (alternated twice).  Usage: gpurun --timeout 1200 -- bash tools/gpu_cfg5_ab.sh TAG "" "--frame-apart" ...
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${PARITY:-tests/test_gpu_large_levels.py tests/test_gpu_cfg5_bench_call.py} -x -q --timeout 300 --timeout-method thread > $OUT/c5par_$TAG.log 2>&1 || { echo parity failed; tail -30 $OUT/c5par_$TAG.log; exit 1; }
tail -1 $OUT/c5par_$TAG.log
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    timeout -k 10 400 python bench.py --config cfg5 --steps 10 --warmup 2 --replays 10 --no-cpu --no-cold $v > $OUT/c5_${TAG}_$i.log 2>&1 || { tail -20 $OUT/c5_${TAG}_$i.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']
print(repr(sys.argv[2]), 'ms/step %.3f' % d['ms_per_step'], 'stages', {k: round(v,1) for k,v in d['stage_us'].items()}, r['kernel'], round(r['avg_launch_us'],1), 'launches', r['launches_per_stage'])" $OUT/c5_${TAG}_$i.log "$v"
  done
done
