#!/bin/bash
# The full GPU suite on the in-tree library, then k_collect's cost split on cfg5: the bench's
# stage times with lab variants of the library (tools/ab/libwtprune_cxN.so, WTP_CX knob in
# kernels.hip: 1 no scatter, 2 no reservation, 3 counters only, 4 loads + max) -- their
# selections are wrong by construction, only k_collect's own time is read.
# Usage: gpurun --timeout 1100 -- bash tools/gpu_cx.sh TAG
set -o pipefail
TAG=${1:-cx}
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out
mkdir -p $O


echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pyt_$TAG.log 2>&1 || { echo gpu tests failed; grep -E "^FAILED|passed|failed" $O/pyt_$TAG.log | tail -10; }
tail -1 $O/pyt_$TAG.log
for v in new ${VARIANTS:-np} new ${VARIANTS:-np}; do
  L=""; [ $v != new ] && L=$(pwd)/tools/ab/libwtprune_$v.so
  WTP_LIB_PATH=$L timeout -k 10 300 python bench.py --config cfg5 --steps 6 --warmup 2 --replays 4 --no-cpu --no-cold --no-rocprof > $O/cx_${TAG}_$v.log 2>&1 || { tail -20 $O/cx_${TAG}_$v.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/cx_${TAG}_$v.log') if l.startswith('{')][-1]); print('$v', round(d['ms_per_step'],4), {k: round(x,1) for k,x in d['stage_us'].items()})"
done
