#!/bin/bash
# round 6 end: smoke, the whole GPU suite, the cfg5 bench line and its kernel trace (final tree).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r6o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo gpu tests failed; tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
WTP_BENCH_TRACE_DIR=$OUT/trace5 timeout -k 10 400 python bench.py --config cfg5 --steps 20 --warmup 3 > $OUT/bench_cfg5.log 2>&1 || { echo bench cfg5 failed; tail -30 $OUT/bench_cfg5.log; exit 1; }
tail -1 $OUT/bench_cfg5.log | cut -c1-300
