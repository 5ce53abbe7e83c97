#!/bin/bash
# PMC counter passes over the NTT bench (run on the GPU box via gpurun).  Each counter group
# is its own rocprofv3 run with --kernel-trace only (no sys/runtime tracing; see task rules).
set -e
OUT=${1:-$GRAFT_REPO_ROOT/gpurun_out/pmc}
ARGS=${2:---steps 2 --warmup 1 --no-cpu --no-extra}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > /dev/null 2>$OUT/p$i.err || echo "pass $i failed"
done
