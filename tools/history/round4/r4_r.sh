#!/bin/bash
# Round 4: MustSetRandom's whole-word draws on uniform_whole_kernel (+ fix-up) -- sampler and Jindo
# parity (fix-up path included), then the one-box A/B of the commit lines (u0 = general kernel only).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_samplers.py tests/test_gpu_jindo.py > gpurun_out/r_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r_tests.log; exit 1; }
tail -1 gpurun_out/r_tests.log
bash tools/lib_ab.sh j14,j16 u0 u1
