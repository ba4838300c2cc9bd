# A/B of lab library variants (tools/ab/libwtprune_VARIANT.so): parity subset + one bench line each.
# Usage: VARIANTS="a b" PYK="large or window" CFG=cfg5 gpurun -- bash tools/lib_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab
mkdir -p $O
CFG=${CFG:-cfg5}
for v in $VARIANTS; do
  L=$GRAFT_REPO_ROOT/tools/ab/libwtprune_$v.so
  WTP_LIB_PATH=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_levels.py -x -q --timeout 300 --timeout-method thread -k "$PYK" > $O/p_$v.log 2>&1 || { echo "$v parity FAILED"; tail -15 $O/p_$v.log; exit 1; }
  echo "$v parity: $(tail -1 $O/p_$v.log)"
  WTP_LIB_PATH=$L timeout -k 10 300 python bench.py --config $CFG --steps 10 --warmup 2 --no-cpu --no-cold > $O/v_$v.log 2>&1 || { tail -20 $O/v_$v.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/v_$v.log') if l.startswith('{')][-1]); print('$v', round(d['ms_per_step'],4), {k: round(x,1) for k,x in d['stage_us'].items()}, d['roofline']['kernel'], round(d['roofline']['avg_launch_us'],1))"
done
