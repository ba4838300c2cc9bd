#!/bin/bash
# k_resident A/B: resident parity tests + phase lab on the in-tree library, then cfg2 bench lines
# alternating the in-tree library and tools/ab/libwtprune_base.so (tools/build_base.sh: HEAD before the change).
# Usage: gpurun --timeout 900 -- bash tools/gpu_resab.sh TAG
set -o pipefail
TAG=${1:-ab}
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
echo "== resident tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -v --timeout 120 --timeout-method thread > $OUT/res_$TAG.log 2>&1 || { echo resident tests failed; grep -E "PASS|FAIL|Error|assert" $OUT/res_$TAG.log | tail -40; exit 1; }
tail -1 $OUT/res_$TAG.log
echo "== reslab"
timeout -k 10 120 ./tools/mb/reslab 50 $OUT/reslab_$TAG.csv > $OUT/reslab_$TAG.log 2>&1 || { echo reslab failed; tail -20 $OUT/reslab_$TAG.log; exit 1; }
grep -v "184466" $OUT/reslab_$TAG.log
for v in new base new base; do
  L=""; [ $v = base ] && L=$(pwd)/tools/ab/libwtprune_base.so
  WTP_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu --no-cold > $OUT/b_${TAG}_$v.log 2>&1 || { tail -20 $OUT/b_${TAG}_$v.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$OUT/b_${TAG}_$v.log') if l.startswith('{')][-1]); r=d['roofline']; print('$v', round(d['ms_per_step']*1e3,2), 'us/step', r['kernel'], round(r['avg_launch_us'],2), 'rocprof', round(r['avg_launch_us_stamps'] or -1,2), 'stamps frac', round(r['frac'],3))"
done
