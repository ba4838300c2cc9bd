# per-kernel trace of cfg5 with each lab library (ablations: results may be wrong, timing only)
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in $VARIANTS; do
  cd /tmp && WTP_LIB_PATH=$ROOT/tools/mb/libwtprune_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/tv_$v -o run -- python3 $ROOT/bench.py --config cfg5 --steps 2 --warmup 1 --no-cpu --no-cold --no-rocprof --no-graph > $ROOT/gpurun_out/tv_$v.log 2>&1 || { echo "$v failed"; tail -5 $ROOT/gpurun_out/tv_$v.log; exit 1; }
  cd $ROOT && echo "== $v" && python3 tools/trace_levels.py gpurun_out/tv_$v/run_kernel_trace.csv --min-us 100 | grep -i "collect\|kernel"
done
