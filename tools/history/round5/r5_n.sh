#!/bin/bash
# Round 5: COSAC centres ahead of cdt2 (cenfirst), + data-row digits beside MustSetRandom (digsplit):
# Jindo parity on digsplit,
# A/B x2 at configs[2] / configs[4], and its configs[4] timeline
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_digsplit.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_jindo.py tests/test_gpu_samplers.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5n_tests.txt 2>&1 || { echo "digsplit tests failed"; tail -30 gpurun_out/r5n_tests.txt; exit 1; }
tail -1 gpurun_out/r5n_tests.txt
: > gpurun_out/r5n_ab.txt
for rep in 1 2; do
for v in base cenfirst digsplit; do
  if [ $v = base ]; then unset RINGO_LIB; else export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so; fi
  timeout -k 10 300 python3 bench.py --no-ntt --extra j14,j16 --no-cpu > gpurun_out/r5n_$v.json 2> gpurun_out/r5n_$v.err || { echo "bench $v failed"; tail -3 gpurun_out/r5n_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5n_$v.json')); print('$v', round(d['jindo_commit']['value']), round(d['jindo_commit_2e16']['value']))" | tee -a gpurun_out/r5n_ab.txt
done
done
export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_digsplit.so
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r5n_tr16 -o run -- python3 $R/bench.py --no-ntt --extra j16 --no-cpu --steps 4 --warmup 1 > $R/gpurun_out/r5n_tr16.json 2> $R/gpurun_out/r5n_tr16.err || { echo "trace failed"; exit 1; }
