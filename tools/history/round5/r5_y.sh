#!/bin/bash
# Round 5: NTT variant parity (tests/test_gpu_ntt.py on each ringo-snark_amd/vlib variant), then the
# headline A/B.  usage: r5_y.sh "<variants>" "<ab order>"
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for v in $1; do
  RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ntt.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5y_tests_$v.txt 2>&1 || { echo "tests $v failed"; tail -30 gpurun_out/r5y_tests_$v.txt; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r5y_tests_$v.txt)"
done
bash tools/ab_ntt.sh "$2"
