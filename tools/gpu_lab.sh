#!/bin/bash
# Build a tools/mb lab on the box (the binaries are gpurun-ignored) and run it under a time limit.
# Usage: gpurun --timeout 600 -- bash tools/gpu_lab.sh NAME TAG [args...]
set -o pipefail
N=$1; TAG=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/mb/$N.hip -o /tmp/$N 2> gpurun_out/lab_${N}_$TAG.build.log || { tail -20 gpurun_out/lab_${N}_$TAG.build.log; exit 1; }
timeout -k 10 240 /tmp/$N "$@" > gpurun_out/lab_${N}_$TAG.log 2>&1 || { echo "lab $N failed"; tail -30 gpurun_out/lab_${N}_$TAG.log; exit 1; }
cat gpurun_out/lab_${N}_$TAG.log
