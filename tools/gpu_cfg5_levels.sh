#!/bin/bash
# cfg5 per-level kernel trace with the selections serialised (pipeline 0, eager), so no level
# shares the GPU with k_collect: the clean per-launch time of every filter-bank level.
# Usage: gpurun --timeout 900 -- bash tools/gpu_cfg5_levels.sh TAG ["variant" ...]   (default: "" "--frame-apart")
set -o pipefail
TAG=${1:-l}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; mkdir -p gpurun_out
[ $# -gt 0 ] || set -- "" "--frame-apart"
i=0
for v in "$@"; do
  d=gpurun_out/lv_${TAG}_$i
  WTP_BENCH_TRACE_DIR=$d timeout -k 10 400 python bench.py --config cfg5 --steps 10 --warmup 2 --no-cpu --no-cold \
    --no-graph --pipeline 0 $v > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  echo "== variant '$v'"
  python3 - $d.log <<'PY' || exit 1
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('ms/step %.3f' % d['ms_per_step'], 'stages', {k: round(v, 1) for k, v in d['stage_us'].items()})
PY
  python3 tools/trace_levels.py $d/run_kernel_trace.csv --min-us 5 || exit 1
  i=$((i+1))
done
