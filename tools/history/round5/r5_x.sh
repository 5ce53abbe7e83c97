#!/bin/bash
# Round 5: the ROW pass with cross-lane exchanges (DPP row_shr/row_shl with bank masks,
# v_permlane16_swap, quad_perm) instead of LDS: parity of each variant on the NTT tests, then
# the headline line A/B (xl1: H<->M by swaps; xl2: + M<->L; xl3: + the store / load transposes)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for v in xl1 xl2 xl3; do
  RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ntt.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5x_tests_$v.txt 2>&1 || { echo "tests $v failed"; tail -30 gpurun_out/r5x_tests_$v.txt; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r5x_tests_$v.txt)"
done
bash tools/ab_ntt.sh "base xl1 xl2 xl3 base xl1 xl2 xl3 base xl1"
