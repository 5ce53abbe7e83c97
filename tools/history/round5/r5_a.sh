#!/bin/bash
# Round 5: wave-local NTT exchanges. NTT parity on the new product library, then A/B x3 of the
# headline line: r4 (round-4 library) / base (wave-local, this build) / wl_noltw / wl0 (barriers)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ntt.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5a_ntt_tests.txt 2>&1 || { echo "ntt tests failed"; tail -30 gpurun_out/r5a_ntt_tests.txt; exit 1; }
tail -2 gpurun_out/r5a_ntt_tests.txt
bash tools/ab_ntt.sh "r4 base wl_noltw wl0 r4 base wl_noltw wl0 r4 base wl_noltw wl0" 2>&1 | tee gpurun_out/r5a_ab.txt
