#!/bin/bash
# Rehearsal of bench.py's N > 1 path on a one-GPU box (run via gpurun): two ranks share cuda:0 and
# talk over gloo (RINGO_BENCH_REHEARSAL=1), so the commit-key broadcast, the Evaluate all-reduce,
# the barriers / max-over-ranks timing and the self-checks all run as on an 8-GPU node (where
# the same code uses RCCL).  The values are not measurements: two ranks share one card.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
RINGO_BENCH_REHEARSAL=1 timeout -k 10 600 python -u bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu \
  > gpurun_out/rehearsal_n2.out 2> gpurun_out/rehearsal_n2.err || { echo "rehearsal failed"; tail -20 gpurun_out/rehearsal_n2.err; exit 1; }
tail -1 gpurun_out/rehearsal_n2.out  # gloo prints its connection lines on stdout before the JSON line
