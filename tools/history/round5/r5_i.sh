#!/bin/bash
# Round 5: the DAG with the encode prep split (TwinCDT rows after cdt2, COSAC rows after cosac2),
# parity on it (COSAC groups of 8), A/B x2 vs the plain DAG and with stream priorities, its timeline
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_split.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_jindo.py tests/test_gpu_jindo_2e16.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5i_tests.txt 2>&1 || { echo "dag tests failed"; tail -30 gpurun_out/r5i_tests.txt; exit 1; }
tail -2 gpurun_out/r5i_tests.txt
: > gpurun_out/r5i_ab.txt
for rep in 1 2; do
for v in dagg8 split splitprio; do
  if [ $v = base ]; then unset RINGO_LIB; else export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so; fi
  timeout -k 10 300 python3 bench.py --no-ntt --extra j14,j16 --no-cpu > gpurun_out/r5i_$v.json 2> gpurun_out/r5i_$v.err || { echo "bench $v failed"; tail -3 gpurun_out/r5i_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5i_$v.json')); print('$v', round(d['jindo_commit']['value']), round(d['jindo_commit_2e16']['value']))" | tee -a gpurun_out/r5i_ab.txt
done
done
export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_split.so
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r5i_tr -o run -- python3 $R/bench.py --no-ntt --extra j14 --no-cpu --steps 4 --warmup 1 > $R/gpurun_out/r5i_tr.json 2> $R/gpurun_out/r5i_tr.err || { echo "trace failed"; exit 1; }
