#!/bin/bash
# Round 5: the pipelined persistent NTT pass (ntt16_pipe: LDS-DMA of the next tile during the
# current one, 2 workgroups per CU): NTT parity on it, A/B x3 of the headline line vs the product,
# and its per-pass kernel times
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_pipe.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_ntt.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5q_tests.txt 2>&1 || { echo "pipe tests failed"; tail -30 gpurun_out/r5q_tests.txt; exit 1; }
tail -1 gpurun_out/r5q_tests.txt
bash tools/ab_ntt.sh "base pipe base pipe base pipe" 2>&1 | tee gpurun_out/r5q_ab.txt
bash tools/ntt_kstats.sh "pipe" 2>&1 | tee gpurun_out/r5q_kstats.txt
