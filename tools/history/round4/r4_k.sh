#!/bin/bash
# Round 4: dot_split_kernel with 2 lk per lane (16-byte loads) -- Jindo (Evaluate) parity on the
# product library, then the one-box A/B of the configs[4] line (lpl1 = 8-byte form, lpl2 = 16-byte,
# lpl2u1 = 16-byte without the x2 term unroll).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_jindo.py > gpurun_out/k_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/k_tests.log; exit 1; }
tail -1 gpurun_out/k_tests.log
bash tools/lib_ab.sh j16 lpl1 lpl2 lpl2u1
