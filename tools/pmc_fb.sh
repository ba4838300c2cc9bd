# SQ counters of the cfg5 filter-bank kernels (lab): one pass, a short bench run.
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/pmcfb
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $O/p1 -o run -- python3 $ROOT/bench.py --config cfg5 --steps 2 --warmup 1 --no-cpu --no-cold --no-rocprof --stage-reps 1 --no-graph > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/p2 -o run -- python3 $ROOT/bench.py --config cfg5 --steps 2 --warmup 1 --no-cpu --no-cold --no-rocprof --stage-reps 1 --no-graph > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
cd $ROOT && python3 tools/pmc_fb.py $O
