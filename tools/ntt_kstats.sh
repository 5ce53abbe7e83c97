#!/bin/bash
# Per-pass kernel times of the headline NTT line for libringo variants in ringo-snark_amd/vlib:
#   tools/ntt_kstats.sh "base r4 wlrow"     (base = the in-tree lib/libringo.so)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in $1; do
  OUT=$R/gpurun_out/nk_$v
  if [ $v = base ]; then unset RINGO_LIB; else export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py --no-extra --no-cpu --steps 50 --warmup 5 > $OUT.json 2> $OUT.err || { echo "trace $v failed"; tail -5 $OUT.err; exit 1; }
  f=$(find $OUT -name "*kernel_stats.csv" | head -1)
  echo "== $v"
  python3 - "$f" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "ntt16_pass" in r["Name"] and int(r["Calls"]) > 40]
rows.sort(key=lambda r: r["Name"])
tot = 0
for r in rows:
    tot += float(r["AverageNs"]) / 1e3
    print(f'{float(r["AverageNs"])/1e3:8.1f} us x{int(r["Calls"]):4d}  {r["Name"][:95]}')
print(f'{tot:8.1f} us per step (sum of pass averages)')
PY
done
