#!/bin/bash
# Round-2 crash reproduction: rocprofv3 --kernel-trace over the cfg5 bench's graph loop, with a
# fault handler and a memory-map snapshot (WTP_CRASH_DIAG) so the native frames can be named.
# Usage: gpurun --timeout 600 -- bash tools/prof5_repro.sh TAG
set -o pipefail
TAG=${1:-p5}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof5_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
WTP_CRASH_DIAG=$OUT timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg5 --steps 10 --warmup 2 --no-cpu --no-cold --no-rocprof > "$OUT/run.log" 2>&1
rc=$?
echo "rc=$rc"
grep -m3 "SIGSEGV\|PC:" "$OUT/run.log"
tail -1 "$OUT/run.log" | cut -c1-200
exit 0
