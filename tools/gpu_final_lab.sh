set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export TMPDIR=/tmp
WTP_BENCH_TRACE_DIR=$(pwd)/gpurun_out/trace5_r03k timeout -k 10 500 python bench.py --config cfg5 --steps 20 --warmup 3 --no-cpu --no-cold > gpurun_out/bench_cfg5_tr.log 2>&1 || { tail -20 gpurun_out/bench_cfg5_tr.log; exit 1; }
python3 tools/trace_levels.py gpurun_out/trace5_r03k/run_kernel_trace.csv --min-us 5 > gpurun_out/levels_r03k.txt && cat gpurun_out/levels_r03k.txt
timeout -k 10 120 ./tools/mb/reslab 50 gpurun_out/reslab_r03k.csv > gpurun_out/reslab_r03k.log 2>&1 || { tail -5 gpurun_out/reslab_r03k.log; exit 1; }
grep -v 184466 gpurun_out/reslab_r03k.log
