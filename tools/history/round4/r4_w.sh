#!/bin/bash
# Round 4: Evaluate's dot kernel with 2 / 4 / 8 columns per workgroup (one-box A/B, configs[4] line)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for v in nc2 nc8; do
  RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_jindo.py -k evaluate > gpurun_out/w_tests_$v.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 gpurun_out/w_tests_$v.log; exit 1; }
  tail -1 gpurun_out/w_tests_$v.log
done
bash tools/lib_ab.sh j16 nc4 nc2 nc8
