#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_levels.py tests/test_gpu_cfg5_bench_call.py tests/test_gpu_pipeline.py tests/test_gpu_flat.py -x -q --timeout 300 --timeout-method thread > gpurun_out/par_r6i.log 2>&1 || { echo "parity failed"; grep -E "FAIL|Error|assert" gpurun_out/par_r6i.log | head -20; tail -20 gpurun_out/par_r6i.log; exit 1; }
echo "parity: $(tail -1 gpurun_out/par_r6i.log)"
WTP_LIB_PATH=$(pwd)/tools/ab/libwtprune_fdnt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_cfg5_bench_call.py tests/test_gpu_large_levels.py -x -q --timeout 300 --timeout-method thread > gpurun_out/par_r6i_fdnt.log 2>&1 || { echo "parity fdnt failed"; tail -20 gpurun_out/par_r6i_fdnt.log; exit 1; }
echo "parity fdnt: $(tail -1 gpurun_out/par_r6i_fdnt.log)"
VARIANTS="cur noalt fdnt noalt_fdnt" CFG=cfg5 ROUNDS=2 bash tools/gpu_libvars.sh alt
