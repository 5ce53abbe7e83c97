#!/bin/bash
# kernel-trace stats of the j16 line for the default library and each lib/var<n> variant
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in base "$@"; do
  OUT=$R/gpurun_out/var_$v
  mkdir -p $OUT
  if [ $v = base ]; then unset RINGO_LIB; else export RINGO_LIB=$R/ringo-snark_amd/vlib/var$v/libringo.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --no-cpu --no-ntt --extra j16 --steps 4 --warmup 1 > $OUT/bench.json 2> $OUT/trace.err || { echo "variant $v failed"; tail -5 $OUT/trace.err; exit 1; }
  f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
  echo "== $v"; grep -E "noise_kernel|uniform_elems" $f | cut -d, -f1-4
done
