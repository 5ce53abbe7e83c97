#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/r4_b.sh > gpurun_out/r4_b.out 2>&1; rb=$?
tail -40 gpurun_out/r4_b.out
[ $rb -eq 0 ] || exit $rb
bash tools/r4_c.sh
