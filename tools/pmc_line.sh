#!/bin/bash
# rocprofv3 PMC passes (one run per counter group, --kernel-trace only) of one bench line
# usage: tools/pmc_line.sh <outname> "<group1>" "<group2>" ... -- <bench args>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
shift
groups=()
while [ "$1" != "--" ]; do groups+=("$1"); shift; done
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "${groups[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --no-cpu --no-prewarm "$@" > $OUT/bench$i.json 2>$OUT/p$i.err || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.err; exit 1; }
  echo "pass $i ok"
done
python3 $R/tools/pmc_summary.py $OUT
