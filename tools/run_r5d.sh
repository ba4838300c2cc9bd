set -o pipefail
cd $GRAFT_REPO_ROOT
for v in "--pipeline 0" "--pipeline 0 --no-graph" "" "--no-graph"; do
  timeout -k 10 400 python bench.py --config cfg5 --steps 10 --warmup 2 --replays 10 --no-cpu --no-cold --no-rocprof $v > gpurun_out/c5_r5d.log 2>&1 || { tail -5 gpurun_out/c5_r5d.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/c5_r5d.log') if l.startswith('{')][-1])
print(repr(sys.argv[1]), 'ms/step %.3f' % d['ms_per_step'], 'timed_region %.3f' % d['timed_region']['ms_per_step'])" "$v"
done
echo "== traces"
WTP_BENCH_TRACE_DIR=gpurun_out/trace_graph timeout -k 10 400 python bench.py --config cfg5 --steps 10 --warmup 2 --replays 10 --no-cpu --no-cold > gpurun_out/c5_tg.log 2>&1 || { tail -5 gpurun_out/c5_tg.log; exit 1; }
WTP_BENCH_TRACE_DIR=gpurun_out/trace_eager timeout -k 10 400 python bench.py --config cfg5 --steps 10 --warmup 2 --replays 10 --no-cpu --no-cold --no-graph > gpurun_out/c5_te.log 2>&1 || { tail -5 gpurun_out/c5_te.log; exit 1; }
ls -la gpurun_out/trace_graph gpurun_out/trace_eager
