#!/bin/bash
# Round 4: prep256 without per-stage reductions (NC) -- Jindo parity on the product library
# (including the NC vs per-stage form comparison), then the one-box A/B of the commit lines on the
# experiments build: RINGO_JINDO_PREP=canon (per-stage form) vs the default (NC).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_jindo.py > gpurun_out/l_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/l_tests.log; exit 1; }
tail -1 gpurun_out/l_tests.log
out=gpurun_out/prep_nc_ab.txt
: > $out
for rep in 1 2; do
  for v in canon nc; do
    RINGO_LIB=$R/ringo-snark_amd/lib/libringo_exp.so RINGO_JINDO_PREP=$v timeout -k 10 300 python3 bench.py --no-ntt --extra j14,j16 --no-cpu > gpurun_out/pab_$v.json 2> gpurun_out/pab_$v.err || { echo "$v FAILED"; tail -5 gpurun_out/pab_$v.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/pab_$v.json'))
print('$v', ' | '.join('%s %.1f ms %.3f' % (k, d[k]['value'], d[k]['ms_per_batch']) for k in ('jindo_commit','jindo_commit_2e16')))" | tee -a $out
  done
done
