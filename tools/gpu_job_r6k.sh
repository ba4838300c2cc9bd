#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
for v in cur head; do
  L=""; [ $v != cur ] && L=$(pwd)/tools/ab/libwtprune_$v.so
  WTP_LIB_PATH=$L WTP_BENCH_TRACE_DIR=$(pwd)/gpurun_out/tr_$v timeout -k 10 300 python bench.py --config cfg5 --steps 10 --warmup 2 --replays 10 --no-cpu --no-cold > gpurun_out/tr_$v.log 2>&1 || { tail -20 gpurun_out/tr_$v.log; exit 1; }
  python3 tools/trace_levels.py gpurun_out/tr_$v/run_kernel_trace.csv | head -14
done
