#!/bin/bash
# MFMA MAC variants (tools/ubench/mmc_*): correctness at a small shape, then the configs[4] half-batch timing
cd $GRAFT_REPO_ROOT
for b in tools/ubench/mmc_*; do
  timeout -k 5 60 $b 288230376151736833 33 32 16 37 | tail -1
  timeout -k 5 120 $b 288230376151748609 513 32 16 2304 512 10 || { echo "$b timing failed"; exit 1; }
done
