#!/bin/bash
# k_small A/B: parity of each variant library on the golden + cfg3 cases, then its phase probe.
# Usage: gpurun -- bash tools/gpu_small_ab.sh VARIANT...   (tools/mb/libwtprune_VARIANT{,_probe}.so)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
for v in "$@"; do
  echo "== $v"
  WTP_LIB_PATH=$ROOT/tools/mb/libwtprune_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
      --timeout 120 --timeout-method thread -k "golden_case or cfg3 or grouped" > "$OUT/ab_$v.log" 2>&1 \
      || { echo "parity failed"; tail -30 "$OUT/ab_$v.log"; exit 1; }
  tail -1 "$OUT/ab_$v.log"
  PROBE_OUT=$ROOT/tools/mb/libwtprune_${v}_probe.so timeout -k 10 120 python -u tools/probe_small.py > "$OUT/probe_$v.log" 2>&1 \
      || { echo "probe failed"; tail -20 "$OUT/probe_$v.log"; exit 1; }
  grep -v amdgpu.ids "$OUT/probe_$v.log"
done
if [ -n "$SM_TILES_SWEEP" ]; then
  for n in $SM_TILES_SWEEP; do
    echo "== tiles $n"
    WTP_SM_TILES=$n PROBE_OUT=$ROOT/tools/mb/libwtprune_${1}_probe.so timeout -k 10 120 python -u tools/probe_small.py > "$OUT/probe_t$n.log" 2>&1 || { echo "probe failed"; exit 1; }
    grep -E "workgroups|arrived|digit 3|stores" "$OUT/probe_t$n.log"
  done
fi
if [ -n "$SM_COST_SWEEP" ]; then
  for c in $SM_COST_SWEEP; do
    echo "== tile cost $c"
    WTP_SM_TILES=128 WTP_SM_TILECOST=$c PROBE_OUT=$ROOT/tools/mb/libwtprune_probe.so timeout -k 10 120 python -u tools/probe_small.py > "$OUT/probe_c$c.log" 2>&1 || { echo "probe failed"; exit 1; }
    grep -E "workgroups|L0 loaded|arrived 0|barrier|ranks|I start|stores" "$OUT/probe_c$c.log"
  done
fi
