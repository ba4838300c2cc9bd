#!/bin/bash
# cfg5: bench line with the rocprof child's kernel trace kept (per-level times), then the PMC
# passes of tools/pmc_run.sh over the cfg5 step.  Usage: gpurun --timeout 1200 -- bash tools/gpu_cfg5prof.sh TAG
set -o pipefail
TAG=${1:-c5}
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
WTP_BENCH_TRACE_DIR=$R/gpurun_out/trace5_$TAG timeout -k 10 500 python bench.py --config cfg5 --steps 20 --warmup 3 --no-cpu --no-cold > gpurun_out/bench_cfg5_$TAG.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench_cfg5_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_cfg5_$TAG.log | cut -c1-600
python3 tools/trace_levels.py gpurun_out/trace5_$TAG/run_kernel_trace.csv --min-us 5 | head -30
[ -n "$2" ] && exit 0
timeout -k 10 900 bash tools/pmc_run.sh c5$TAG --config cfg5 && python3 tools/pmc_summary.py gpurun_out/pmc_c5$TAG gpurun_out/pmc_cfg5_$TAG.json c5$TAG && cat gpurun_out/pmc_cfg5_$TAG.json | head -60
