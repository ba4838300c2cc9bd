#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py tests/test_gpu_sharding.py tests/test_gpu_integration_stub.py -x -q --timeout 300 --timeout-method thread > gpurun_out/par_r6h.log 2>&1 || { echo "parity failed"; grep -E "FAIL|Error|assert" gpurun_out/par_r6h.log | head -20; tail -20 gpurun_out/par_r6h.log; exit 1; }
echo "parity: $(tail -1 gpurun_out/par_r6h.log)"
VARIANTS="cur nolast" CFG=cfg2 ROUNDS=3 COLD=" " bash tools/gpu_libvars.sh last1
