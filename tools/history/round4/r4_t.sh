#!/bin/bash
# Round 4: the commit's two halves staggered (the second starts after the first half's samplers)
# vs started together -- Jindo / sampler parity, then the A/B on the experiments build
# (RINGO_JINDO_SPLIT=2: together; 1: staggered, the product's choice).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_samplers.py tests/test_gpu_jindo_2e16.py > gpurun_out/t_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/t_tests.log; exit 1; }
tail -1 gpurun_out/t_tests.log
out=gpurun_out/split_ab.txt
: > $out
for rep in 1 2; do
  for v in 2 1; do
    RINGO_LIB=$R/ringo-snark_amd/lib/libringo_exp.so RINGO_JINDO_SPLIT=$v timeout -k 10 300 python3 bench.py --no-ntt --extra j14,j16 --no-cpu > gpurun_out/sab_$v.json 2> gpurun_out/sab_$v.err || { echo "$v FAILED"; tail -5 gpurun_out/sab_$v.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/sab_$v.json'))
print('split=$v', ' | '.join('%s %.1f ms %.3f' % (k, d[k]['value'], d[k]['ms_per_batch']) for k in ('jindo_commit','jindo_commit_2e16')))" | tee -a $out
  done
done
