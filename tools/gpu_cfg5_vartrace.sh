#!/bin/bash
# cfg5 per-launch trace (pipeline 0, eager) of several library builds: the rows of the selection
# kernels and the level-1/2 forward.  Usage: VARIANTS="cur a b" gpurun -- bash tools/gpu_cfg5_vartrace.sh TAG
set -o pipefail
TAG=${1:-vt}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; mkdir -p gpurun_out
for v in ${VARIANTS:-cur}; do
  L=""; [ $v != cur ] && L=$ROOT/tools/ab/libwtprune_$v.so
  d=gpurun_out/vt_${TAG}_$v
  WTP_LIB_PATH=$L WTP_BENCH_TRACE_DIR=$d timeout -k 10 400 python bench.py --config cfg5 --steps 10 --warmup 2 --no-cpu --no-cold \
    --no-graph --pipeline 0 $X > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  echo "== $v $(python3 -c "import json,sys; d=json.loads([l for l in open('$d.log') if l.startswith('{')][-1]); print('ms/step %.3f' % d['ms_per_step'])")"
  python3 tools/trace_levels.py $d/run_kernel_trace.csv --min-us 5 | grep -E "k_fwin|k_fslot|k_mask|k_fwd_int<16, false>" || exit 1
done
