#!/bin/bash
# Bench A/B of several library builds on one box: tools/ab/libwtprune_<v>.so for each v in VARIANTS
# ("cur" = the in-tree wavelettransforms_amd/_lib/libwtprune.so), ROUNDS passes in alternation, one
# bench.py line each (graph p50 + the rocprofv3 child's kernel average).
# Build variants with tools/mb/build_variant.sh or tools/resvar_lib.sh.
# Usage: VARIANTS="cur a b" CFG=cfg2 ROUNDS=2 gpurun -- bash tools/gpu_libvars.sh TAG
set -o pipefail
TAG=${1:-lv}
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/lv_$TAG; mkdir -p $OUT
export TMPDIR=/tmp
CFG=${CFG:-cfg2}
X=""; [ $CFG = cfg5 ] && X="--steps 10 --warmup 2 --replays 10"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-cur}; do
    L=""; [ $v != cur ] && L=$(pwd)/tools/ab/libwtprune_$v.so
    WTP_LIB_PATH=$L timeout -k 10 300 python bench.py --config $CFG --no-cpu ${COLD:---no-cold} $X > $OUT/b_${v}_$r.log 2>&1 || { echo "$v failed"; tail -20 $OUT/b_${v}_$r.log; exit 1; }
    python3 - $OUT/b_${v}_$r.log $v $r <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r = d['roofline']
cm = d.get('cold_mall') or {}
print("%-12s rep %s  %8.2f us/step  %s %7.2f us  frac %.3f%s" % (sys.argv[2], sys.argv[3], d['ms_per_step'] * 1e3, r.get('kernel'),
      r.get('avg_launch_us') or -1, r.get('frac') or -1, ("  cold(write) span %.2f" % cm.get(r.get('kernel') + '_us', 0)) if cm else ""))
PY
  done
done
