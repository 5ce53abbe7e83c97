#!/bin/bash
# Round 4: mlwe_noise split into table / rounded kernels -- Jindo + sampler parity, then the
# one-box A/B of the commit lines (mlwe1 = one kernel, mlwe2 = split).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_jindo.py tests/test_gpu_samplers.py > gpurun_out/j_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/j_tests.log; exit 1; }
tail -1 gpurun_out/j_tests.log
bash tools/lib_ab.sh j14,j16 mlwe1 mlwe2
