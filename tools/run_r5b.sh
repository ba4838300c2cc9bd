set -o pipefail
cd $GRAFT_REPO_ROOT
PARITY="tests/test_gpu_resident.py tests/test_gpu_parity.py tests/test_gpu_large_levels.py tests/test_gpu_cfg5_bench_call.py" bash tools/gpu_ab.sh r5b "cfg2 cfg5" || exit 1
echo "== pipeline mode 2 eager (bench, no graph)"
timeout -k 10 300 python -X faulthandler bench.py --config cfg5 --steps 6 --warmup 2 --no-cpu --no-cold --no-graph --no-rocprof --pipeline 2 > gpurun_out/c5_lanes_eager.log 2>&1; echo "rc=$?"; tail -3 gpurun_out/c5_lanes_eager.log | cut -c1-400
echo "== pipeline tests"
timeout -k 10 600 python -X faulthandler -u -m pytest tests/test_gpu_pipeline.py -v --timeout 300 --timeout-method thread > gpurun_out/pipe_m2.log 2>&1; echo "rc=$?"; grep -E 'PASS|FAIL|Fatal|Error' gpurun_out/pipe_m2.log | head -30
