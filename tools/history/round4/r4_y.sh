#!/bin/bash
# Round 4: cdt2 queue chunks of 4 polynomials vs 8 (one-box A/B, both commit lines)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_cd4.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_samplers.py > gpurun_out/y_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/y_tests.log; exit 1; }
tail -1 gpurun_out/y_tests.log
bash tools/lib_ab.sh j14,j16 cd8 cd4
