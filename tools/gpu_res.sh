#!/bin/bash
# k_resident iteration: resident parity tests, the phase lab, then the cfg2 bench.
# Usage: gpurun --timeout 900 -- bash tools/gpu_res.sh TAG [full]
set -o pipefail
TAG=${1:-res}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== resident tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -v --timeout 120 --timeout-method thread > "$OUT/res_$TAG.log" 2>&1 || { echo resident tests failed; grep -E "PASS|FAIL|Error|assert" "$OUT/res_$TAG.log" | tail -40; exit 1; }
tail -1 "$OUT/res_$TAG.log"
echo "== reslab"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I wavelettransforms_amd/csrc tools/mb/reslab.hip -o /tmp/reslab && timeout -k 10 120 /tmp/reslab 50 "$OUT/reslab_$TAG.csv" > "$OUT/reslab_$TAG.log" 2>&1 || { echo reslab failed; tail -20 "$OUT/reslab_$TAG.log"; exit 1; }
grep -v "184466\|select" "$OUT/reslab_$TAG.log"
if [ -n "$2" ]; then
echo "== all gpu tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_$TAG.log" 2>&1 || { echo gpu tests failed; tail -40 "$OUT/gpu_$TAG.log"; exit 1; }
tail -1 "$OUT/gpu_$TAG.log"
fi
echo "== bench cfg2"
timeout -k 10 300 python bench.py --no-cpu > "$OUT/bench_$TAG.log" 2>&1 || { echo bench failed; tail -30 "$OUT/bench_$TAG.log"; exit 1; }
tail -1 "$OUT/bench_$TAG.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('ms/step %.5f value %.4g frac %.3f avg_launch_us %.2f stamps %.2f cold %s' % (d['ms_per_step'], d['value'], r['frac'], r['avg_launch_us'], r['avg_launch_us_stamps'] or -1, (d.get('cold_mall') or {}).get('k_resident_us')))"
