#!/bin/bash
# rocprofv3 kernel-trace + stats of the bench command, then PMC passes (each its own run,
# --kernel-trace only, no sys/runtime tracing).  Usage (on the GPU box):
#   tools/profile_bench.sh <outdir> [bench args]
set -o pipefail
OUT=${1:-$GRAFT_REPO_ROOT/gpurun_out/prof}
shift || true
ARGS=${@:---steps 4 --warmup 1 --no-cpu --no-extra}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/bench_under_trace.json 2> $OUT/trace.err || { echo "trace failed"; tail $OUT/trace.err; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > /dev/null 2>$OUT/p$i.err || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.err; exit 1; }
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt
find $OUT/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
cat $OUT/pmc_summary.txt
