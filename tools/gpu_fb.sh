#!/bin/bash
# cfg5 iteration: the whole GPU suite, then the cfg5 bench (its rocprofv3 child included).
# Usage: gpurun --timeout 1200 -- bash tools/gpu_fb.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-fb5}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$2" ]; then
echo "== all gpu tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_$TAG.log" 2>&1 || { echo gpu tests failed; tail -40 "$OUT/gpu_$TAG.log"; exit 1; }
tail -1 "$OUT/gpu_$TAG.log"
fi
echo "== bench cfg5"
timeout -k 10 500 python bench.py --config cfg5 --steps 20 --warmup 3 --no-cpu --no-cold > "$OUT/bench_cfg5_$TAG.log" 2>&1 || { echo bench failed; tail -30 "$OUT/bench_cfg5_$TAG.log"; exit 1; }
tail -1 "$OUT/bench_cfg5_$TAG.log" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('ms/step %.3f value %.4g' % (d['ms_per_step'], d['value']), 'stages', {k: round(v,1) for k,v in d['stage_us'].items()})
print('roofline kernel %s frac %.3f valu_frac %s achieved %.0f GB/s launches %.1f us/step %.1f traffic/launch %s' % (r['kernel'], r['frac'], r['valu_frac'], r['achieved'], r['launches_per_stage'], r['us_per_step'], r['traffic']))
print('valu_roof', d.get('valu_roof'))"
