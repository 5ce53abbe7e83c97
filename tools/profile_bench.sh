#!/bin/bash
# Profiles of the bench (run on the GPU box via gpurun):
#   1. rocprofv3 --kernel-trace --stats of the default bench command (every line)
#   2. per line (ntt, l4, j14, j16), separate --pmc passes (each its own run, --kernel-trace
#      only: no sys/runtime tracing), then tools/kernel_counters.py -> kernel_counters.json
#      (per-line HBM bytes and VALU instruction counts that bench.py reports for THIS .so)
# usage: tools/profile_bench.sh <outdir>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=${1:-$R/gpurun_out/prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --no-cpu --steps 10 --warmup 2 > $OUT/bench_under_trace.json 2> $OUT/trace.err || { echo "trace failed"; tail $OUT/trace.err; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
for line in ntt l4 j14 j16; do
  if [ $line = ntt ]; then LA="--no-extra"; else LA="--no-ntt --extra $line"; fi
  i=0
  mkdir -p $OUT/pmc/$line
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/pmc/$line/p$i -o run -- python3 $R/bench.py $LA --no-cpu --no-prewarm --steps 4 --warmup 1 > $OUT/pmc/$line/bench.json 2>$OUT/pmc/$line/p$i.err || { echo "pmc $line pass $i failed"; tail -5 $OUT/pmc/$line/p$i.err; exit 1; }
    echo "pmc $line pass $i ok"
  done
done
python3 $R/tools/kernel_counters.py $OUT/pmc $OUT/kernel_counters.json $R/ringo-snark_amd/lib/libringo.so
head -12 $OUT/kernel_stats.csv
