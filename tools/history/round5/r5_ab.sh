#!/bin/bash
# Round 5: L = 4 variant parity (tests/test_gpu_ntt.py) and the l4 bench line A/B
#   r5_ab.sh "<variants>" "<order>"
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for v in $1; do
  RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ntt.py tests/test_gpu_buckler.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5ab_tests_$v.txt 2>&1 || { echo "tests $v failed"; tail -30 gpurun_out/r5ab_tests_$v.txt; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r5ab_tests_$v.txt)"
done
for v in $2; do
  if [ $v = base ]; then unset RINGO_LIB; else export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so; fi
  timeout -k 10 240 python3 bench.py --no-ntt --extra l4 --no-cpu > gpurun_out/abl4_$v.json 2> gpurun_out/abl4_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/abl4_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/abl4_$v.json')); x=d['l4_ntt']; print('$v', round(x['value']), round(x.get('ms_per_step',0),4))"
done
