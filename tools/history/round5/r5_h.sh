#!/bin/bash
# Round 5: the three-stream commit DAG (vlib/libringo_dag.so): sampler / Jindo parity on it,
# then A/B x2 against the product library at configs[2] and configs[4], and its j14 timeline
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_dag.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_jindo.py tests/test_gpu_jindo_2e16.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5h_tests.txt 2>&1 || { echo "dag tests failed"; tail -30 gpurun_out/r5h_tests.txt; exit 1; }
tail -2 gpurun_out/r5h_tests.txt
: > gpurun_out/r5h_ab.txt
for rep in 1 2; do
for v in base dag dagg8 dagg4; do
  if [ $v = base ]; then unset RINGO_LIB; else export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so; fi
  timeout -k 10 300 python3 bench.py --no-ntt --extra j14,j16 --no-cpu > gpurun_out/r5h_$v.json 2> gpurun_out/r5h_$v.err || { echo "bench $v failed"; tail -3 gpurun_out/r5h_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5h_$v.json')); print('$v', round(d['jindo_commit']['value']), round(d['jindo_commit_2e16']['value']))" | tee -a gpurun_out/r5h_ab.txt
done
done
export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_dag.so
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r5h_tr -o run -- python3 $R/bench.py --no-ntt --extra j14 --no-cpu --steps 4 --warmup 1 > $R/gpurun_out/r5h_tr.json 2> $R/gpurun_out/r5h_tr.err || { echo "trace failed"; exit 1; }
