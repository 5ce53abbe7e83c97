#!/bin/bash
# Round 4, call c: the whole -m gpu suite on the current library, the default bench line, and the
# Evaluate A/B (dot_split_kernel vs mac_kernel via the experiments build) on the j16 line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/c_tests.log; exit 1; }
tail -2 gpurun_out/c_tests.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/c_bench.json 2> gpurun_out/c_bench.err || { echo BENCH FAILED; tail -5 gpurun_out/c_bench.err; exit 1; }
cat gpurun_out/c_bench.json
RINGO_LIB=$R/ringo-snark_amd/lib/libringo_exp.so RINGO_JINDO_EVAL=mac timeout -k 10 300 python3 bench.py --no-ntt --extra j16 --no-cpu > gpurun_out/c_bench_evalmac.json 2> gpurun_out/c_bench_evalmac.err || { echo AB FAILED; tail -5 gpurun_out/c_bench_evalmac.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/c_bench_evalmac.json')); print('eval on mac_kernel:', d['jindo_evaluate_2e16'])"
