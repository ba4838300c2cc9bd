set -o pipefail
cd $GRAFT_REPO_ROOT
echo skip-diag
echo "== pipeline tests"
timeout -k 10 600 python -X faulthandler -u -m pytest tests/test_gpu_pipeline.py -q --timeout 300 --timeout-method thread > gpurun_out/pipe_r5c.log 2>&1 || { tail -20 gpurun_out/pipe_r5c.log; exit 1; }
tail -1 gpurun_out/pipe_r5c.log
for v in "" "--pipeline 2" "--no-graph" "--pipeline 2 --no-graph" "" "--pipeline 2"; do
  timeout -k 10 400 python bench.py --config cfg5 --steps 10 --warmup 2 --replays 10 --no-cpu --no-cold --no-rocprof $v > gpurun_out/c5_r5c.log 2>&1 || { tail -5 gpurun_out/c5_r5c.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/c5_r5c.log') if l.startswith('{')][-1])
print(repr(sys.argv[1]), 'ms/step %.3f' % d['ms_per_step'], 'timed_region %.3f' % d['timed_region']['ms_per_step'])" "$v"
done
