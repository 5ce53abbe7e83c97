#!/bin/bash
# Round 4: stall breakdown of the configs[4] commit kernels (rocprofv3 --pmc, one pass per group)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/pmc_line.sh samp_pmc \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES" \
  -- --no-ntt --extra j16 > gpurun_out/samp_pmc.txt 2>&1 || { echo PMC FAILED; tail -20 gpurun_out/samp_pmc.txt; exit 1; }
tail -3 gpurun_out/samp_pmc.txt
