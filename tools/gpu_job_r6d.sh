#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_levels.py tests/test_gpu_cfg5_bench_call.py tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/par_r6d.log 2>&1 || { echo parity failed; grep -E "FAIL|Error|assert" gpurun_out/par_r6d.log | head -20; tail -20 gpurun_out/par_r6d.log; exit 1; }
tail -1 gpurun_out/par_r6d.log
VARIANTS="cur head cnt fnt int" CFG=cfg5 ROUNDS=2 bash tools/gpu_libvars.sh nt5
