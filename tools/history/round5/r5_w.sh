#!/bin/bash
# Round 5: configs[4] / configs[2] commit timelines on the final library: the product DAG, and the
# experiments build on one stream (RINGO_JINDO_SPLIT=0), whose kernels run alone
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for line in j16 j14; do
  for mode in dag one; do
    OUT=$R/gpurun_out/r5w_${line}_$mode
    mkdir -p $OUT
    if [ $mode = one ]; then export RINGO_LIB=$R/ringo-snark_amd/lib/libringo_exp.so RINGO_JINDO_SPLIT=0; else unset RINGO_LIB RINGO_JINDO_SPLIT; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 $R/bench.py --no-cpu --no-ntt --extra $line --steps 4 --warmup 1 > $OUT/bench.json 2> $OUT/trace.err || { echo "trace $line $mode failed"; tail -5 $OUT/trace.err; exit 1; }
    f=$(find $OUT -name "*kernel_trace.csv" | head -1)
    echo "== $line $mode"; python3 $R/tools/trace_batch.py $f
  done
done
