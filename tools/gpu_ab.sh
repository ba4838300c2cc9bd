#!/bin/bash
# A/B on one box: parity of the changed paths, then each config's bench line with the
# working tree's library ("new") and tools/ab/libwtprune_base.so ("base", tools/build_base.sh),
# alternated twice; the k_resident phase lab last.  NEW_LIB / BASE_LIB override either library
# (e.g. a lab build under tools/ab/); PARITY="" skips the parity step.
# Usage: gpurun --timeout 1100 -- bash tools/gpu_ab.sh TAG [configs]
set -o pipefail
TAG=${1:-ab}
CFGS=${2:-"cfg2 cfg3 cfg5"}
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
PARITY=${PARITY-tests/test_gpu_resident.py tests/test_gpu_small.py tests/test_gpu_large_levels.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_cfg5_bench_call.py}
if [ -n "$PARITY" ]; then
  echo "== parity"
  timeout -k 10 700 python -u -m pytest $PARITY -x -q --timeout 300 --timeout-method thread > $OUT/par_$TAG.log 2>&1 || { echo parity failed; grep -E "FAIL|Error|assert" $OUT/par_$TAG.log | head -30; tail -30 $OUT/par_$TAG.log; exit 1; }
  tail -1 $OUT/par_$TAG.log
fi
for c in $CFGS; do
  X=""; [ $c = cfg5 ] && X="--steps 10 --warmup 2 --replays 10"
  for v in new base new base; do
    L=${NEW_LIB:-}; [ $v = base ] && L=${BASE_LIB:-$(pwd)/tools/ab/libwtprune_base.so}
    NC="--no-cold"; [ -n "$COLD" ] && NC=""
    WTP_LIB_PATH=$L timeout -k 10 300 python bench.py --config $c --no-cpu $NC $X > $OUT/b_${TAG}_${c}_$v.log 2>&1 || { tail -20 $OUT/b_${TAG}_${c}_$v.log; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('$OUT/b_${TAG}_${c}_$v.log') if l.startswith('{')][-1]); r=d['roofline']
cm=d.get('cold_mall') or {}; cr=cm.get('after_read_flush') or {}
print('$c', '$v', round(d['ms_per_step']*1e3,2), 'us/step', r.get('kernel'), round(r.get('avg_launch_us') or -1,2), 'frac', round(r.get('frac') or -1,3),
      'cold(write) %.2f us/step span %.2f | cold(read) %.2f span %.2f' % (1e3*cm.get('ms_per_step_p50',0), cm.get(r.get('kernel','')+'_us',0), 1e3*cr.get('ms_per_step_p50',0), cr.get(r.get('kernel','')+'_us',0)) if cm else '')"
  done
done
if [ -n "$RESLAB" ]; then
  echo "== reslab"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I wavelettransforms_amd/csrc tools/mb/reslab.hip -o /tmp/reslab || exit 1
  timeout -k 10 120 /tmp/reslab 50 $OUT/reslab_$TAG.csv > $OUT/reslab_$TAG.log 2>&1 || { echo reslab failed; tail -20 $OUT/reslab_$TAG.log; exit 1; }
  grep -v "184466" $OUT/reslab_$TAG.log | head -30
fi
