#!/bin/bash
# kernel-trace + stats of the headline bench command (run on the GPU box via gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu --no-extra > $OUT/bench.json 2>$OUT/bench.err || { echo BENCH FAILED; tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu --no-extra --steps 5 > $OUT/bench_traced.json 2> $OUT/trace.err || { echo TRACE FAILED; tail $OUT/trace.err; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
head -8 $OUT/kernel_stats.csv
