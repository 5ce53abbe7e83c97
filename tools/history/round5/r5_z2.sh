#!/bin/bash
# Round 5: commit-library variant parity (tests/test_gpu_jindo.py on each variant) + j14/j16 A/B
#   r5_z2.sh "<variants>"   (A/B against the in-tree product, vlib/libringo_base.so)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for v in $1; do
  RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_jindo.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5z2_tests_$v.txt 2>&1 || { echo "tests $v failed"; tail -30 gpurun_out/r5z2_tests_$v.txt; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r5z2_tests_$v.txt)"
done
bash tools/lib_ab.sh j14,j16 base $1
