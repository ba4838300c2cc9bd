#!/bin/bash
# Filter-bank frame kernels: the parity tests that cover the levels, then cfg5 with the frame of edge
# tiles in k_fwd_int/k_inv_int's EDGE form (default) and in the general kernels (--frame-general),
# alternating on one box, then a rocprofv3 kernel trace of the default cfg5 bench.
# Usage: gpurun --timeout 1100 -- bash tools/gpu_fbedge.sh TAG
set -o pipefail
TAG=${1:-fe}
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
echo "== filter-bank parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_levels.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_cfg5_bench_call.py tests/test_gpu_flat.py -x -q --timeout 300 --timeout-method thread > $OUT/fep_$TAG.log 2>&1 || { echo parity failed; grep -E "FAIL|Error|assert|error" $OUT/fep_$TAG.log | head -40; tail -30 $OUT/fep_$TAG.log; exit 1; }
tail -1 $OUT/fep_$TAG.log
for v in edge gen edge gen; do
  F=""; [ $v = gen ] && F=--frame-general
  timeout -k 10 300 python bench.py --config cfg5 --steps 10 --warmup 2 --replays 10 --no-cpu --no-cold --no-rocprof $F > $OUT/b5_${TAG}_$v.log 2>&1 || { tail -20 $OUT/b5_${TAG}_$v.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$OUT/b5_${TAG}_$v.log') if l.startswith('{')][-1]); print('$v', round(d['ms_per_step'],4), 'ms/step', {k: round(x,1) for k,x in d.get('stage_us',{}).items()})"
done
echo "== rocprof cfg5"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof5_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 4 --warmup 1 --replays 2 --stage-reps 2 --no-cpu --no-cold --no-rocprof --no-graph > $GRAFT_REPO_ROOT/$OUT/prof5_$TAG.log 2>&1 || { echo rocprof failed; tail -20 $GRAFT_REPO_ROOT/$OUT/prof5_$TAG.log; exit 1; }
head -12 $GRAFT_REPO_ROOT/$OUT/prof5_$TAG/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-200
