#!/bin/bash
# round 6: fused selection -- its GPU tests, the cfg5 golden test, then cfg5 fused against
# unfused (wtp_set_fused_select), alternated twice, and a rocprofv3 kernel-stats pass of each.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6l
mkdir -p $OUT
export TMPDIR=/tmp
echo "== fused tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_select.py -x -v --timeout 300 --timeout-method thread > $OUT/t_fused.log 2>&1 || { echo fused tests failed; grep -E "FAIL|Error|assert|passed|failed" $OUT/t_fused.log | head -30; tail -40 $OUT/t_fused.log; exit 1; }
grep -E "passed|failed" $OUT/t_fused.log | tail -1
timeout -k 10 400 python -u -m pytest tests/test_gpu_cfg5_bench_call.py -x -q --timeout 300 --timeout-method thread > $OUT/t_cfg5.log 2>&1 || { echo cfg5 test failed; tail -30 $OUT/t_cfg5.log; exit 1; }
tail -1 $OUT/t_cfg5.log
for v in fused unfused fused unfused; do
  X=""; [ $v = unfused ] && X="--no-fused-select"
  timeout -k 10 300 python bench.py --config cfg5 --no-cpu --no-cold --steps 10 --warmup 2 --replays 10 $X > $OUT/b_$v.log 2>&1 || { tail -20 $OUT/b_$v.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$OUT/b_$v.log') if l.startswith('{')][-1]); r=d['roofline']
print('$v', round(d['ms_per_step']*1e3,1), 'us/step', r.get('kernel'), round(r.get('avg_launch_us') or -1,2), 'frac', round(r.get('frac') or -1,3))"
done
for v in fused unfused; do
  X=""; [ $v = unfused ] && X="--no-fused-select"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run -- python bench.py --config cfg5 --no-cpu --no-cold --no-rocprof --steps 10 --warmup 2 --replays 10 $X > $OUT/p_$v.log 2>&1 || { tail -20 $OUT/p_$v.log; exit 1; }
  f=$(find $OUT/prof_$v -name "*kernel_stats.csv" | head -1); cp $f $OUT/stats_$v.csv
  cut -d, -f1-4 $OUT/stats_$v.csv | head -14
done
