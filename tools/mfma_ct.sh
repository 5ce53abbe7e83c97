#!/bin/bash
# (the RG_MFMA_CT / RG_MFMA_KEYREG variants exist only with tools/experiments/mac_mfma_stage_keyreg.patch applied)
# Round 4 MFMA MAC A/B: chunks per ring stage (RG_MFMA_CT) x ring depth (RG_MFMA_STAGES), each
# variant checked for correctness (NB = 5 / 6 / 8, odd chunk counts) and timed at the configs[4]
# inner-MAC half batch (T 545, J 16, 2304 columns) and the configs[2] one.  Binaries are built
# in the container (tools/ubench/mmc/).
cd $GRAFT_REPO_ROOT
for v in tools/ubench/mmc/mmc_*; do
  echo "== $v"
  timeout -k 5 60 $v 68719484929 33 32 10 37 | tail -1 || exit 1
  timeout -k 5 60 $v 1099511630849 30 0 6 37 | tail -1 || exit 1
  timeout -k 5 60 $v 288230376151736833 41 32 16 37 | tail -1 || exit 1
  timeout -k 5 120 $v 288230376151748609 513 32 16 2304 512 20 || exit 1
  timeout -k 5 120 $v 288230376151748609 513 32 16 2304 512 20 || exit 1
  timeout -k 5 120 $v 68719484929 129 32 10 1152 512 20 || exit 1
done
