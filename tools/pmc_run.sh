#!/bin/bash
# rocprofv3 PMC passes over a short bench run (one counter group per pass, kernel trace only).
# --stage-reps 0: only the step's own launches are counted (the stage leg runs the call as ONE
# launch group, whose larger launches would skew the per-launch means bench.py multiplies by the
# step's launch count).
# Usage: gpurun -- bash tools/pmc_run.sh TAG [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu --no-cold --no-rocprof --stage-reps 0 --no-graph "$@" > "$OUT/p$i.log" 2>&1 \
      || { echo "pass $i ($grp) failed"; tail -20 "$OUT/p$i.log"; exit 1; }
done
echo pmc done
