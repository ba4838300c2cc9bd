#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_parity.py tests/test_gpu_layer_api.py -x -q --timeout 300 --timeout-method thread > gpurun_out/par_r6g.log 2>&1 || { echo "parity failed"; grep -E "FAIL|Error|assert" gpurun_out/par_r6g.log | head -20; tail -20 gpurun_out/par_r6g.log; exit 1; }
echo "parity: $(tail -1 gpurun_out/par_r6g.log)"
VARIANTS="cur head" CFG=cfg3 ROUNDS=3 bash tools/gpu_libvars.sh sm1
