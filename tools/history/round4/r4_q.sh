#!/bin/bash
# Round 4: chunk sizes of the sampler queues (cdt2: 32 / 16 / 8 polynomials; cosac2: 4 / 2 / 8 jobs)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/lib_ab.sh j14,j16 base cd16 cd8 ck2 ck8
