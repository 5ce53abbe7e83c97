#!/bin/bash
# A/B of the headline NTT line between the in-tree libringo.so (base) and ringo-snark_amd/vlib variants:
#   tools/ab_ntt.sh "base prio base prio"
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for v in $1; do
  if [ $v = base ]; then unset RINGO_LIB; else export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so; fi
  timeout -k 10 240 python3 $R/bench.py --no-extra --no-cpu --steps 50 --warmup 5 > $R/gpurun_out/abn_$v.json 2> $R/gpurun_out/abn_$v.err || { echo "bench $v failed"; tail -5 $R/gpurun_out/abn_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$R/gpurun_out/abn_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],4))"
done
