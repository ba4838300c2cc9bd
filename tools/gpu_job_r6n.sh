#!/bin/bash
# round 6: pipelined fused selection: its tests + the cfg5 goldens, the cfg5 bench lines fused /
# unfused alternated, then the per-launch trace of the fused form.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_select.py tests/test_gpu_cfg5_bench_call.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|assert" $OUT/t.log | head -30; tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for v in fused unfused fused unfused; do
  X=""; [ $v = unfused ] && X="--no-fused-select"
  timeout -k 10 300 python bench.py --config cfg5 --no-cpu --no-cold --steps 10 --warmup 2 --replays 10 $X > $OUT/b_$v.log 2>&1 || { tail -20 $OUT/b_$v.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$OUT/b_$v.log') if l.startswith('{')][-1]); r=d['roofline']
print('$v', round(d['ms_per_step']*1e3,1), 'us/step', r.get('kernel'), round(r.get('avg_launch_us') or -1,2), 'frac', round(r.get('frac') or -1,3))"
done
VARIANTS=cur bash tools/gpu_cfg5_vartrace.sh n
