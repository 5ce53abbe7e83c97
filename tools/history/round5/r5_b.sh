#!/bin/bash
# Round 5: per-pass times of round-4 / wave-local (both passes, ROW only, COL only) NTT libraries
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/ntt_kstats.sh "r4 base wlrow wlcol r4 base wlrow wlcol" 2>&1 | tee gpurun_out/r5b_kstats.txt
