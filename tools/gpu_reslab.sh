#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I wavelettransforms_amd/csrc tools/mb/reslab.hip -o /tmp/reslab && timeout -k 10 120 /tmp/reslab 50 gpurun_out/reslab_$1.csv > gpurun_out/reslab_$1.log 2>&1 || { tail -20 gpurun_out/reslab_$1.log; exit 1; }
grep -v "184466" gpurun_out/reslab_$1.log
