set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/jprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/jprof/trace -o run -- python3 bench.py --no-cpu --steps 4 --warmup 1 > gpurun_out/jprof/bench.json 2> gpurun_out/jprof/err.txt || { tail gpurun_out/jprof/err.txt; exit 1; }
f=$(find gpurun_out/jprof/trace -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/jprof/kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/jprof/kernel_stats.csv')))
for r in rows[:25]:
    print(f"{float(r['Percentage']):6.2f}% {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f}us  {r['Name'][:120]}")
PY
