#!/bin/bash
# Round 5: MFMA MAC epilogue rows rotated (macrot: 4-way instead of 32-way LDS bank conflicts)
# vs the product: Jindo / sampler parity on idx, A/B x2 at configs[2] / configs[4], kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_macrot.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_jindo.py tests/test_gpu_jindo_2e16.py tests/test_gpu_verify.py tests/test_gpu_samplers.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5v_tests.txt 2>&1 || { echo "macrot tests failed"; tail -30 gpurun_out/r5v_tests.txt; exit 1; }
tail -1 gpurun_out/r5v_tests.txt
: > gpurun_out/r5v_ab.txt
for rep in 1 2; do
for v in base macrot; do
  if [ $v = base ]; then unset RINGO_LIB; else export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so; fi
  timeout -k 10 300 python3 bench.py --no-ntt --extra j14,j16 --no-cpu > gpurun_out/r5v_$v.json 2> gpurun_out/r5v_$v.err || { echo "bench $v failed"; tail -3 gpurun_out/r5v_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5v_$v.json')); print('$v', round(d['jindo_commit']['value']), round(d['jindo_commit_2e16']['value']))" | tee -a gpurun_out/r5v_ab.txt
done
done
bash tools/lib_kstats.sh "base macrot" j14 2>&1 | grep -e "==" -e mac_mfma | tee -a gpurun_out/r5v_ab.txt
