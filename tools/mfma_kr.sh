#!/bin/bash
# (the RG_MFMA_CT / RG_MFMA_KEYREG variants exist only with tools/experiments/mac_mfma_stage_keyreg.patch applied)
# Round 4 MFMA MAC A/B: key chunks by LDS-DMA (mmc_kr0: the library's kernel) vs plain loads into a
# register ring (mmc_kr1_s*: mac_mfma_kr_kernel, S opening stages), correctness at NB = 5 / 6 / 8
# with odd chunk counts, then the configs[4] / configs[2] inner half-batch timings, each twice.
cd $GRAFT_REPO_ROOT
for v in tools/ubench/mmc/mmc_kr*; do
  echo "== $v"
  timeout -k 5 60 $v 68719484929 33 32 10 37 | tail -1 || exit 1
  timeout -k 5 60 $v 1099511630849 30 0 6 37 | tail -1 || exit 1
  timeout -k 5 60 $v 288230376151736833 41 32 16 37 | tail -1 || exit 1
  timeout -k 5 60 $v 288230376151736833 513 32 16 19 | tail -1 || exit 1
  for r in 1 2; do timeout -k 5 120 $v 288230376151748609 513 32 16 2304 512 20 || exit 1; done
  timeout -k 5 120 $v 68719484929 129 32 10 1152 512 20 || exit 1
done
