set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -q --timeout 300 --timeout-method thread > gpurun_out/pipe_r5e.log 2>&1 || { tail -20 gpurun_out/pipe_r5e.log; exit 1; }
tail -1 gpurun_out/pipe_r5e.log
for c in cfg2 cfg5; do
  X=""; [ $c = cfg5 ] && X="--steps 20 --warmup 3"
  WTP_BENCH_TRACE_DIR=gpurun_out/trace_$c timeout -k 10 400 python bench.py --config $c $X --no-cpu --no-cold > gpurun_out/b_r5e_$c.log 2>&1 || { tail -5 gpurun_out/b_r5e_$c.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/b_r5e_$c.log') if l.startswith('{')][-1]); r=d['roofline']
print('$c', 'ms/step %.5f' % d['ms_per_step'], 'timed_region %.5f' % d['timed_region']['ms_per_step'], r['kernel'], round(r['avg_launch_us'],2), 'frac %.3f' % r['frac'])"
  grep -c Fill gpurun_out/trace_$c/run_kernel_trace.csv || true
done
