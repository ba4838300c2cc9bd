#!/bin/bash
# filter-bank iteration: GPU parity tests + cfg5/cfg3 bench stage breakdown
set -o pipefail
TAG=${1:-fb}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for c in cfg5 cfg3; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_${c}_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_${c}_$TAG.log; exit 1; }
  tail -1 gpurun_out/bench_${c}_$TAG.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$c ms/step %.4f' % d['ms_per_step'], {k: round(v,1) for k,v in d['stage_us'].items()})"
done
