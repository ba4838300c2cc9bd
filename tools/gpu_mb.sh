set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 ./tools/mb/stream_mb > gpurun_out/stream_mb.log 2>&1; cat gpurun_out/stream_mb.log
timeout -k 10 900 bash tools/pmc_run.sh r01
