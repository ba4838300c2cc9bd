#!/bin/bash
# Round 6 cold study: k_resident's phases and times with a warm Infinity Cache and after three
# flushes (write 512 MiB / read 512 MiB / write then read) -- the stamped lab (tools/mb/reslab.hip)
# and the unstamped product kernel (RESLAB_NOPROBE), then rocprofv3 kernel traces of the product
# library under tools/cold_run.py for each flush.  Usage: gpurun -- bash tools/gpu_cold6.sh TAG
set -o pipefail
TAG=${1:-c6}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
export TMPDIR=/tmp
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off"
$H -I wavelettransforms_amd/csrc tools/mb/reslab.hip -o /tmp/reslab && $H -I wavelettransforms_amd/csrc -DRESLAB_NOPROBE tools/mb/reslab.hip -o /tmp/reslab_np || exit 1
for m in 0 1 2 3; do
  echo "== stamped, flush $m"
  timeout -k 10 120 /tmp/reslab 60 $OUT/reslab_${TAG}_f$m.csv $m > $OUT/reslab_${TAG}_f$m.log 2>&1 || { tail -20 $OUT/reslab_${TAG}_f$m.log; exit 1; }
  grep -v "184466" $OUT/reslab_${TAG}_f$m.log | grep -E "median|selector 2(31|39)" | head -24
  echo "== unstamped, flush $m"
  timeout -k 10 120 /tmp/reslab_np 60 /dev/null $m > $OUT/reslabnp_${TAG}_f$m.log 2>&1 || { tail -20 $OUT/reslabnp_${TAG}_f$m.log; exit 1; }
  grep "k_resident cfg2" $OUT/reslabnp_${TAG}_f$m.log
done
cd /tmp
for f in write read clean; do
  echo "== rocprofv3 cold_run --flush $f"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${TAG}_$f" -o run --output-format csv -- python3 "$ROOT/tools/cold_run.py" --steps 60 --flush $f > "$OUT/cold_${TAG}_$f.log" 2>&1 || { echo trace failed; tail -20 "$OUT/cold_${TAG}_$f.log"; exit 1; }
  grep -E "k_resident|Fill|reduce" "$OUT/prof_${TAG}_$f/run_kernel_stats.csv" | cut -c1-160
done
echo done
