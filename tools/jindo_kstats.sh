#!/bin/bash
# Kernel stats (rocprofv3 --kernel-trace --stats) of one Jindo bench line under env variants:
#   tools/jindo_kstats.sh VAR "val1 val2 ..." [line, default j16]
# prints the top kernels (avg us, calls) per variant
set -o pipefail
R=$GRAFT_REPO_ROOT
LINE=${3:-j16}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in $2; do
  OUT=$R/gpurun_out/ks_$v
  export $1=$v
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py --no-ntt --extra $LINE --no-cpu --steps 4 --warmup 1 > $OUT.json 2> $OUT.err || { echo "trace $v failed"; tail -5 $OUT.err; exit 1; }
  f=$(find $OUT -name "*kernel_stats.csv" | head -1)
  echo "== $1=$v"
  python3 - "$f" <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f'{float(r["AverageNs"])/1e3:10.1f} us x{int(r["Calls"]):4d}  {r["Name"][:90]}')
EOF
done
