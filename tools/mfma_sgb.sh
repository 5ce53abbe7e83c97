#!/bin/bash
# (mmc_sgb0 / mmc_sgb1 are built from tools/experiments/mac_mfma_sched_interleave.patch applied)
# Round 4 MFMA MAC A/B: the round-3 kernel (mmc_base) vs the term strides pinned in registers with
# hipcc's MFMA burst left alone (mmc_sgb0) or interleaved with the VALU that forms the next A
# operand (mmc_sgb1, sched_group_barrier); correctness, then configs[4] / configs[2] timings.
cd $GRAFT_REPO_ROOT
for v in tools/ubench/mmc/mmc_base tools/ubench/mmc/mmc_sgb0 tools/ubench/mmc/mmc_sgb1; do
  echo "== $v"
  timeout -k 5 60 $v 68719484929 33 32 10 37 | tail -1 || exit 1
  timeout -k 5 60 $v 1099511630849 30 0 6 37 | tail -1 || exit 1
  timeout -k 5 60 $v 288230376151736833 41 32 16 37 | tail -1 || exit 1
  timeout -k 5 60 $v 288230376151736833 513 32 16 19 | tail -1 || exit 1
  for r in 1 2; do timeout -k 5 120 $v 288230376151748609 513 32 16 2304 512 20 || exit 1; done
  timeout -k 5 120 $v 68719484929 129 32 10 1152 512 20 || exit 1
done
