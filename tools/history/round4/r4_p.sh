#!/bin/bash
# Round 4: cosac2_noise_kernel groups from one grid counter -- Jindo + sampler parity on the product library,
# then the one-box A/B of the commit lines (k0 = fixed per-wave COSAC queues, k1 = refilled 4 jobs at a time from a counter).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_jindo.py tests/test_gpu_samplers.py tests/test_gpu_jindo_2e16.py > gpurun_out/p_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/p_tests.log; exit 1; }
tail -1 gpurun_out/p_tests.log
bash tools/lib_ab.sh j14,j16 k0 k1
