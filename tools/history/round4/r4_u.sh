#!/bin/bash
# Round 4: kernel statistics and HBM traffic of the wide-field NTT line on the final library
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/wide_prof
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/wide_prof/trace -o run -- python3 $R/bench.py --no-ntt --extra wide --no-cpu --steps 8 > $R/gpurun_out/wide_prof/bench.json 2> $R/gpurun_out/wide_prof/trace.err || { echo TRACE FAILED; tail -5 $R/gpurun_out/wide_prof/trace.err; exit 1; }
cd $R && bash tools/pmc_line.sh wide_prof/pmc "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" -- --no-ntt --extra wide --steps 4 > gpurun_out/wide_prof/pmc.txt 2>&1 || { echo PMC FAILED; tail -10 gpurun_out/wide_prof/pmc.txt; exit 1; }
find gpurun_out/wide_prof/trace -name "*kernel_stats.csv" | head -1
