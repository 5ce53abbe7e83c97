#!/bin/bash
# Round 4: 28-bit-digit wide product -- wide parity (NTT + Buckler) on the product library, then
# the one-box A/B against the 32-bit-digit product (tools/wide_ab.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ntt.py tests/test_gpu_buckler.py > gpurun_out/i_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/i_tests.log; exit 1; }
tail -1 gpurun_out/i_tests.log
bash tools/wide_ab.sh d32 d28
