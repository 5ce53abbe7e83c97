#!/bin/bash
# rocprofv3 kernel trace + stats of selected bench lines (run on the GPU box via gpurun)
# usage: tools/trace_line.sh <outname> <bench args...>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --no-cpu "$@" > $OUT/bench.json 2> $OUT/trace.err || { echo "trace failed"; tail $OUT/trace.err; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
cut -d, -f1-8 $OUT/kernel_stats.csv | head -20
