#!/bin/bash
# Round-4 check: the new tests (solo overflow, the documented ctypes stub, cfg5 as the bench runs
# it), then the whole GPU suite and the default bench line.
# Usage: gpurun --timeout 1100 -- bash tools/gpu_r4.sh TAG
set -o pipefail
TAG=${1:-r4}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== new tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py::test_solo_overflow_then_reuse tests/test_gpu_integration_stub.py tests/test_gpu_cfg5_bench_call.py -x -v --timeout 300 --timeout-method thread > "$OUT/new_$TAG.log" 2>&1 || { echo new tests failed; tail -60 "$OUT/new_$TAG.log"; exit 1; }
tail -3 "$OUT/new_$TAG.log"
echo "== all gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_$TAG.log" 2>&1 || { echo gpu tests failed; tail -60 "$OUT/gpu_$TAG.log"; exit 1; }
tail -3 "$OUT/gpu_$TAG.log"
echo "== bench"
timeout -k 10 400 python bench.py > "$OUT/bench_$TAG.log" 2>&1 || { echo bench failed; tail -30 "$OUT/bench_$TAG.log"; exit 1; }
tail -1 "$OUT/bench_$TAG.log" | cut -c1-600
