#!/bin/bash
# Round 5: commit DAG refinements, A/B x2 at configs[2] / configs[4]: g8 (DAG, COSAC groups of 8),
# mlprio (MLWE stream at the highest priority), mlg256 (MLWE samplers on 256 workgroups),
# tail1 / tail2 (cdt2's last 1 / 2 rounds of chunks one polynomial each); sampler parity on tail2
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_tail2.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_jindo.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5j_tests.txt 2>&1 || { echo "tail2 tests failed"; tail -30 gpurun_out/r5j_tests.txt; exit 1; }
tail -1 gpurun_out/r5j_tests.txt
: > gpurun_out/r5j_ab.txt
for rep in 1 2; do
for v in g8 mlprio mlg256 tail1 tail2; do
  export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so
  timeout -k 10 300 python3 bench.py --no-ntt --extra j14,j16 --no-cpu > gpurun_out/r5j_$v.json 2> gpurun_out/r5j_$v.err || { echo "bench $v failed"; tail -3 gpurun_out/r5j_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5j_$v.json')); print('$v', round(d['jindo_commit']['value']), round(d['jindo_commit_2e16']['value']))" | tee -a gpurun_out/r5j_ab.txt
done
done
