set -o pipefail
cd $GRAFT_REPO_ROOT
VARIANTS="cur pct0 pct30 pct45 pct75" ROUNDS=2 bash tools/gpu_libvars.sh pct1 && bash tools/gpu_job_r6b.sh
