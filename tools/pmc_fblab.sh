#!/bin/bash
# PMC passes over the filter-bank lab (one counter group per pass, kernel trace only)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_fblab
mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- "$ROOT/tools/mb/fblab" 8 > "$OUT/p$i.log" 2>&1 \
      || { echo "pass $i ($grp) failed"; tail -20 "$OUT/p$i.log"; exit 1; }
done
echo pmc done
