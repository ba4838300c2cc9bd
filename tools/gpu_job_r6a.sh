set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/pytest_j1.log 2>&1 || { echo FAIL; grep -E "FAIL|Error|assert" gpurun_out/pytest_j1.log | head -20; tail -20 gpurun_out/pytest_j1.log; exit 1; }
tail -2 gpurun_out/pytest_j1.log; grep -E "two concurrent|beside 8" gpurun_out/pytest_j1.log
echo "== rehearsal allgather"
WTP_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --steps 40 --warmup 5 --exchange allgather > gpurun_out/bench_n2_ag.log 2>&1 || { echo rehearsal failed; tail -30 gpurun_out/bench_n2_ag.log; exit 1; }
grep '"metric"' gpurun_out/bench_n2_ag.log | cut -c1-300
echo "== coop variant"
VARIANTS="base coop" MODES="0" bash tools/gpu_resvar.sh coop
