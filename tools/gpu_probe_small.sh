#!/bin/bash
# k_small phase probes (tools/probe_small.py) for one or more probe libraries under tools/ab/
# (built with PROBE_OUT=tools/ab/libwtprune_probe_NAME.so python tools/probe_small.py --build).
# Lab variants whose results are wrong by construction run with PROBE_NOCHECK=1.
# Usage: gpurun -- bash tools/gpu_probe_small.sh TAG NAME[:nocheck] ...
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; mkdir -p gpurun_out
for v in "$@"; do
  n=${v%%:*}; nc=""; [ "$n" != "$v" ] && nc=1
  echo "== $n"
  PROBE_NOCHECK=$nc PROBE_OUT=$ROOT/tools/ab/libwtprune_probe_$n.so timeout -k 10 300 python tools/probe_small.py \
    > gpurun_out/probe_${TAG}_$n.txt 2>&1 || { tail -5 gpurun_out/probe_${TAG}_$n.txt; exit 1; }
  grep -E "span|arrived 1|barrier 1|slots in|ranks|I start|drained" gpurun_out/probe_${TAG}_$n.txt
done
