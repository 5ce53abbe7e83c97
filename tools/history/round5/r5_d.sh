#!/bin/bash
# Round 5: NTT A/B x3 -- barriers (wl0) vs first-generation workgroups started out of phase
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/ab_ntt.sh "wl0 stag127 stag64 wl0 stag127 stag64 wl0 stag127 stag64" 2>&1 | tee gpurun_out/r5d_ab.txt
