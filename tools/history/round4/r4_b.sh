#!/bin/bash
# Round 4, call b: wide-field NTT parity + bench (tools/r4_wide.sh), then the MFMA MAC stage A/B
# (tools/mfma_ct.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/r4_wide.sh || exit 1
bash tools/mfma_ct.sh > gpurun_out/mfma_ct.txt 2>&1; rc=$?
cat gpurun_out/mfma_ct.txt
exit $rc
