#!/bin/bash
# One bench line per lab library variant, alternating twice: VARIANTS="new base x" CFG=cfg2
# (new = the in-tree library, X = tools/mb/libwtprune_X.so).  Optional PYTEST=<file> parity first.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/vb; mkdir -p $OUT
export TMPDIR=/tmp
CFG=${CFG:-cfg2}
for v in $VARIANTS; do
  [ -z "$PYTEST" ] && break
  L=""; [ $v != new ] && L=$(pwd)/tools/mb/libwtprune_$v.so
  WTP_LIB_PATH=$L timeout -k 10 300 python -u -m pytest $PYTEST -x -q --timeout 120 --timeout-method thread > $OUT/p_$v.log 2>&1 || { echo "$v parity FAILED"; tail -15 $OUT/p_$v.log; exit 1; }
  echo "$v parity: $(tail -1 $OUT/p_$v.log)"
done
for rep in 1 2; do for v in $VARIANTS; do
  L=""; [ $v != new ] && L=$(pwd)/tools/mb/libwtprune_$v.so
  WTP_LIB_PATH=$L timeout -k 10 300 python bench.py --config $CFG --no-cpu --no-cold $BARGS > $OUT/b_${v}_$rep.log 2>&1 || { tail -20 $OUT/b_${v}_$rep.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$OUT/b_${v}_$rep.log') if l.startswith('{')][-1]); r=d['roofline']; print('$v', round(d['ms_per_step']*1e3,2), 'us/step', r['kernel'], round(r['avg_launch_us'],2), 'rocprof', round(r['avg_launch_us_stamps'] or -1,2), 'stamps', {k: round(x,1) for k,x in d.get('stage_us',{}).items()})"
done; done
