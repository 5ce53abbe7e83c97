#!/bin/bash
# MFMA MAC one vs two column tiles per wave: correctness at NB = 5 / 6 / 8, configs[2] half-batch timing
cd $GRAFT_REPO_ROOT
for b in tools/ubench/mmc_nt1 tools/ubench/mmc_nt2; do
  echo "== $b"
  timeout -k 5 60 $b 68719484929 33 32 10 37 | tail -1
  timeout -k 5 60 $b 1099511630849 30 0 6 37 | tail -1
  timeout -k 5 60 $b 288230376151736833 33 32 16 37 | tail -1
  timeout -k 5 120 $b 68719484929 129 32 10 1152 512 20
  timeout -k 5 120 $b 1099511630849 90 0 6 128 256 20
done
