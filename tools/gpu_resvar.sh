#!/bin/bash
# k_resident source variants A/B on one box, warm and cold: each variant is a copy of csrc/ with sed
# edits (tools/resvar/<name>.sed, one "FILE<TAB>sed-expression" a line; "base" = the tree as is),
# built into the unstamped reslab harness (tools/mb/reslab.hip -DRESLAB_NOPROBE), then for each
# flush mode (0 warm, 1 write 512 MiB, 2 read 512 MiB) a rocprofv3 kernel trace of 60 calls.
# Usage: VARIANTS="base ntl" MODES="0 1 2" gpurun -- bash tools/gpu_resvar.sh TAG
set -o pipefail
TAG=${1:-rv}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
OUT=$ROOT/gpurun_out/resvar_$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off"
for v in ${VARIANTS:-base}; do
  rm -rf /tmp/rv_$v; mkdir -p /tmp/rv_$v/w /tmp/rv_$v/include; cp include/*.h /tmp/rv_$v/include/
  D=/tmp/rv_$v/w/csrc; cp -r wavelettransforms_amd/csrc $D
  if [ "$v" != base ]; then
    while IFS=$'\t' read -r f e; do [ -z "$f" ] && continue
      cp $D/$f $D/$f.orig; sed -i "$e" $D/$f
      cmp -s $D/$f $D/$f.orig && { echo "variant $v: '$e' changed nothing in $f"; exit 1; }
    done < tools/resvar/$v.sed
  fi
  $H -I $D -DRESLAB_NOPROBE tools/mb/reslab.hip -o /tmp/rvbin_$v || { echo "build $v failed"; exit 1; }
done
for r in 1 2; do
for v in ${VARIANTS:-base}; do
  for m in ${MODES:-0 1 2}; do
    cd /tmp
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/p_${v}_${m}_$r" -o run --output-format csv -- /tmp/rvbin_$v 60 /dev/null $m > "$OUT/l_${v}_${m}_$r.log" 2>&1 || { echo "run $v $m failed"; tail -5 "$OUT/l_${v}_${m}_$r.log"; exit 1; }
    cd "$ROOT"
    grep "k_resident cfg2" "$OUT/l_${v}_${m}_$r.log" | sed "s/^/  $v flush $m rep $r event-timed: /"
    python3 - "$OUT/p_${v}_${m}_$r/run_kernel_stats.csv" "$v" "$m" "$r" <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[1])):
    if "k_resident" in row["Name"]:
        print("%-10s flush %s rep %s  k_resident %7.2f us avg over %s (min %.2f)" % (sys.argv[2], sys.argv[3], sys.argv[4], float(row["AverageNs"]) / 1e3, row["Calls"], float(row["MinNs"]) / 1e3))
PY
  done
done
done
echo done
