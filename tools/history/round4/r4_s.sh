#!/bin/bash
# Round 4: Harvey butterflies in the workgroup LDS NTTs (round_kernel, verifier kernels) -- Jindo,
# verifier and sampler parity, then the one-box A/B of the commit lines (lz0 = fully reduced).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_jindo.py tests/test_gpu_jindo_2e16.py tests/test_gpu_verify.py tests/test_gpu_samplers.py > gpurun_out/s_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/s_tests.log; exit 1; }
tail -1 gpurun_out/s_tests.log
bash tools/lib_ab.sh j14,j16 lz0 lz1
