#!/bin/bash
# Round-3 call: the N = 2^15 ntt256 path (q255 NTT tests, Buckler encode), then the l4 bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ntt.py tests/test_gpu_buckler.py > gpurun_out/l4_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/l4_tests.log; exit 1; }
tail -2 gpurun_out/l4_tests.log
timeout -k 10 300 python -u bench.py --no-ntt --extra l4 --no-cpu --steps 10 --warmup 2 > gpurun_out/bench_l4.json 2> gpurun_out/bench_l4.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_l4.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_l4.json'))['l4_ntt']
print('l4', d['value'], json.dumps(d['bigpoly_ops'].get('buckler')))"
