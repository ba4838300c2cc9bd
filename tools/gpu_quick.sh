set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/mb/lab 2>&1 | grep -v maskv
timeout -k 10 600 bash tools/gpu_check.sh "${1:-r01c}"
