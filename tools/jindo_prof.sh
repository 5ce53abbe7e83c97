#!/bin/bash
# rocprofv3 kernel trace + stats of selected bench lines (run on the GPU box via gpurun):
#   tools/jindo_prof.sh <outdir-name> [bench args]   e.g.  tools/jindo_prof.sh j16 --extra j16
set -o pipefail
cd $GRAFT_REPO_ROOT
NAME=${1:-jprof}
shift || true
ARGS=${@:---no-cpu --steps 4 --warmup 1}
OUT=gpurun_out/$NAME
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/bench.json 2> $OUT/err.txt || { tail $OUT/err.txt; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv
python3 - $OUT <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1] + '/kernel_stats.csv')))
for r in rows[:25]:
    print(f"{float(r['Percentage']):6.2f}% {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f}us  {r['Name'][:110]}")
PY
