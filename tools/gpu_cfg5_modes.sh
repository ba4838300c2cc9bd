#!/bin/bash
# cfg5 pipeline modes and graph vs eager on one box (round 5: the lane-stream and graph-fill
# investigations).  Runs the pipeline tests, then the cfg5 bench per variant, then (TRACE=1) the
# graph and eager kernel traces that profiles/r05_cfg5_graph_fill.txt was read from.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_cfg5_modes.sh TAG ["variant" ...]
#   default variants: "--pipeline 0" "" "--pipeline 2" "--no-graph" "--pipeline 2 --no-graph"
set -o pipefail
TAG=${1:-m}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; mkdir -p gpurun_out
[ $# -gt 0 ] || set -- "--pipeline 0" "" "--pipeline 2" "--no-graph" "--pipeline 2 --no-graph"
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -q --timeout 300 --timeout-method thread \
  > gpurun_out/pipe_$TAG.log 2>&1 || { tail -20 gpurun_out/pipe_$TAG.log; exit 1; }
tail -1 gpurun_out/pipe_$TAG.log
for v in "$@"; do
  timeout -k 10 400 python bench.py --config cfg5 --steps 10 --warmup 2 --replays 10 --no-cpu --no-cold --no-rocprof $v \
    > gpurun_out/c5_$TAG.log 2>&1 || { tail -5 gpurun_out/c5_$TAG.log; exit 1; }
  python3 - "$v" gpurun_out/c5_$TAG.log <<'PY' || exit 1
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][-1])
print(repr(sys.argv[1]), 'ms/step %.3f' % d['ms_per_step'], 'timed_region %.3f' % d['timed_region']['ms_per_step'])
PY
done
if [ "${TRACE:-0}" = 1 ]; then
  for form in graph eager; do
    X=""; [ $form = eager ] && X="--no-graph"
    WTP_BENCH_TRACE_DIR=gpurun_out/trace_${form}_$TAG timeout -k 10 400 python bench.py --config cfg5 --steps 10 \
      --warmup 2 --replays 10 --no-cpu --no-cold $X > gpurun_out/c5_t${form}_$TAG.log 2>&1 \
      || { tail -5 gpurun_out/c5_t${form}_$TAG.log; exit 1; }
    grep -c Fill gpurun_out/trace_${form}_$TAG/run_kernel_trace.csv || true
  done
fi
