#!/bin/bash
# A/B of cfg5 and cfg3 (tools/gpu_r4ab.sh), then k_small's phase timeline (tools/probe_small.py on
# the -DWTP_SM_PROBE build in tools/ab/).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_r4ab.sh ${1:-r4f} "${2:-cfg5 cfg3}" || exit 1
echo "== k_small phases"
PROBE_OUT=$(pwd)/tools/ab/libwtprune_probe.so timeout -k 10 200 python tools/probe_small.py > gpurun_out/probe_small_${1:-r4f}.log 2>&1 || { tail -20 gpurun_out/probe_small_${1:-r4f}.log; exit 1; }
cat gpurun_out/probe_small_${1:-r4f}.log | tail -32
