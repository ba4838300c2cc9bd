#!/bin/bash
# round 6: parity of the workspace / LDS-pitch changes, cfg5 A/B against HEAD's library, and one SQ
# PMC pass of the cfg5 step (the forward kernels' LDS bank conflicts)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_levels.py tests/test_gpu_cfg5_bench_call.py tests/test_gpu_pipeline.py tests/test_gpu_flat.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/par_r6b.log 2>&1 || { echo parity failed; grep -E "FAIL|Error|assert" gpurun_out/par_r6b.log | head -20; tail -20 gpurun_out/par_r6b.log; exit 1; }
tail -1 gpurun_out/par_r6b.log
echo "== cfg5 A/B"
PARITY="" bash tools/gpu_ab.sh r6b cfg5 || exit 1
echo "== SQ pmc cfg5 (new)"
cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_r6b_sq -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 3 --warmup 1 --no-cpu --no-cold --no-rocprof --stage-reps 0 --no-graph > $GRAFT_REPO_ROOT/gpurun_out/pmc_r6b_sq.log 2>&1 || { echo pmc failed; tail -10 $GRAFT_REPO_ROOT/gpurun_out/pmc_r6b_sq.log; exit 1; }
echo done
