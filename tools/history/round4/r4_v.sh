#!/bin/bash
# Round 4: the 14-limb forward wide pass at 3 waves/SIMD -- wide parity, then the one-box A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ntt.py tests/test_gpu_buckler.py > gpurun_out/v_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/v_tests.log; exit 1; }
tail -1 gpurun_out/v_tests.log
bash tools/wide_ab.sh lb2 lb3
