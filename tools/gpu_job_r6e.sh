#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
for v in fc54 fc52; do
  WTP_LIB_PATH=$(pwd)/tools/ab/libwtprune_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_large_levels.py tests/test_gpu_cfg5_bench_call.py -x -q --timeout 300 --timeout-method thread > gpurun_out/par_r6e_$v.log 2>&1 || { echo "parity $v failed"; grep -E "FAIL|Error|assert" gpurun_out/par_r6e_$v.log | head -20; tail -20 gpurun_out/par_r6e_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/par_r6e_$v.log)"
done
VARIANTS="cur fc54 fc52" CFG=cfg5 ROUNDS=2 bash tools/gpu_libvars.sh fc
