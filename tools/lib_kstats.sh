#!/bin/bash
# Kernel stats of one Jindo bench line for libringo variants in ringo-snark_amd/vlib:
#   tools/lib_kstats.sh "base v2 v4" [line]     (base = the in-tree lib/libringo.so)
set -o pipefail
R=$GRAFT_REPO_ROOT
LINE=${2:-j16}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in $1; do
  OUT=$R/gpurun_out/lk_$v
  if [ $v = base ]; then unset RINGO_LIB; else export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py --no-ntt --extra $LINE --no-cpu --steps 4 --warmup 1 > $OUT.json 2> $OUT.err || { echo "trace $v failed"; tail -5 $OUT.err; exit 1; }
  f=$(find $OUT -name "*kernel_stats.csv" | head -1)
  echo "== $v"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:9]:
    print(f'{float(r["AverageNs"])/1e3:10.1f} us x{int(r["Calls"]):4d}  {r["Name"][:70]}')
PY
done
