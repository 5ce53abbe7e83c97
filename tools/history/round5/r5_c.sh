#!/bin/bash
# Round 5: NTT A/B x2 -- barriers (wl0) / ROW wave-local (wlrow), each with waves 4-7 at s_setprio 1 / 2
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/ab_ntt.sh "wl0 wlrow wl0p1 wl1p1 wl0p2 wl1p2 wl0 wlrow wl0p1 wl1p1 wl0p2 wl1p2" 2>&1 | tee gpurun_out/r5c_ab.txt
