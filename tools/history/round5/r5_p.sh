#!/bin/bash
# Round 5: stall counters of the configs[4] commit kernels (prep256 first), product library
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/pmc_line.sh r5p_j16 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" -- --no-ntt --extra j16 --steps 2 --warmup 1 > gpurun_out/r5p_j16_summary.txt 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/r5p_j16_summary.txt; exit 1; }
grep -A20 "prep256" gpurun_out/r5p_j16_summary.txt | head -22
