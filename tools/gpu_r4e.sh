#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_r4ab.sh r4e "cfg5" && bash tools/gpu_fbprof.sh r4e
