set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -q --timeout 120 --timeout-method thread > $O/res.log 2>&1 || { echo resident tests failed; tail -30 $O/res.log; exit 1; }
tail -1 $O/res.log
for v in ${VARS:-fsel0 fsel2 fsel0 fsel2}; do
  WTP_LIB_PATH=$GRAFT_REPO_ROOT/tools/ab/libwtprune_$v.so timeout -k 10 300 python bench.py --no-cpu --no-cold > $O/b_$v.log 2>&1 || { tail -20 $O/b_$v.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/b_$v.log') if l.startswith('{')][-1]); r=d['roofline']; print('$v', round(d['ms_per_step']*1e3,2), 'us/step', r['kernel'], round(r['avg_launch_us'],2), 'rocprof', round(r['avg_launch_us_stamps'],2), 'stamps')"
done
