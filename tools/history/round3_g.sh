#!/bin/bash
# cdt2 centre loop (one sign per digit, scalar deltaInv loads): sampler + Jindo parity, j16 kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_samplers.py tests/test_gpu_jindo.py > gpurun_out/g_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/g_tests.log; exit 1; }
tail -2 gpurun_out/g_tests.log
cd /tmp && export TMPDIR=/tmp RINGO_JINDO_SPLIT=0
OUT=$R/gpurun_out/g_j16
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py --no-ntt --extra j16 --no-cpu --steps 6 --warmup 1 > $OUT.json 2> $OUT.err || { echo "trace failed"; tail -5 $OUT.err; exit 1; }
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:9]:
    print(f'{float(r["AverageNs"])/1e3:10.1f} us x{int(r["Calls"]):4d}  {r["Name"][:70]}')
PY
python3 -c "import json; d=json.load(open('$OUT.json')); j=d['jindo_commit_2e16']; print('commits/s', j['value'], 'ms/batch', j['ms_per_batch'])"
