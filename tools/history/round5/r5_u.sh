#!/bin/bash
# Round 5: index splits through the double unit (idx_div) in digits, MLWE and MustSetRandom kernels (idx)
# vs the product: Jindo / sampler parity on idx, A/B x2 at configs[2] / configs[4], kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_idx.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_jindo.py tests/test_gpu_jindo_2e16.py tests/test_gpu_verify.py tests/test_gpu_samplers.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5u_tests.txt 2>&1 || { echo "idx tests failed"; tail -30 gpurun_out/r5u_tests.txt; exit 1; }
tail -1 gpurun_out/r5u_tests.txt
: > gpurun_out/r5u_ab.txt
for rep in 1 2; do
for v in base idx; do
  if [ $v = base ]; then unset RINGO_LIB; else export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so; fi
  timeout -k 10 300 python3 bench.py --no-ntt --extra j14,j16 --no-cpu > gpurun_out/r5u_$v.json 2> gpurun_out/r5u_$v.err || { echo "bench $v failed"; tail -3 gpurun_out/r5u_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5u_$v.json')); print('$v', round(d['jindo_commit']['value']), round(d['jindo_commit_2e16']['value']))" | tee -a gpurun_out/r5u_ab.txt
done
done
bash tools/lib_kstats.sh "base idx" j16 2>&1 | grep -e "==" -e digits -e mlwe -e uniform | tee -a gpurun_out/r5u_ab.txt
