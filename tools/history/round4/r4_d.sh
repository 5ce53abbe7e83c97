#!/bin/bash
# Round 4, call d: wide NTT (one sub-transform per workgroup at L = 7) parity + bench, then the
# MFMA MAC key-in-registers A/B (tools/mfma_kr.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/r4_wide.sh > gpurun_out/r4_wide.out 2>&1; rw=$?
tail -4 gpurun_out/r4_wide.out
[ $rw -eq 0 ] || exit $rw
bash tools/mfma_kr.sh > gpurun_out/mfma_kr.txt 2>&1; rc=$?
cat gpurun_out/mfma_kr.txt
exit $rc
