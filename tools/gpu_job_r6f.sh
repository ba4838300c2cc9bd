#!/bin/bash
# parity (resident tests) then cfg2 bench A/B of k_resident window variants (tools/resvar/*.sed)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS}; do
  [ $v = cur ] && continue
  WTP_LIB_PATH=$(pwd)/tools/ab/libwtprune_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py -x -q --timeout 300 --timeout-method thread > gpurun_out/par_r6f_$v.log 2>&1 || { echo "parity $v failed"; grep -E "FAIL|Error|assert" gpurun_out/par_r6f_$v.log | head -20; tail -20 gpurun_out/par_r6f_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/par_r6f_$v.log)"
done
VARIANTS="$VARIANTS" CFG=cfg2 ROUNDS=${ROUNDS:-2} bash tools/gpu_libvars.sh ${TAG:-r6f}
