#!/bin/bash
# prep256 change check: Jindo parity (commit/sampled/2^16) then kernel stats of the j16 and j14 lines.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_jindo.py tests/test_gpu_jindo_2e16.py tests/test_gpu_samplers.py} > gpurun_out/e_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/e_tests.log; exit 1; }
tail -2 gpurun_out/e_tests.log
cd /tmp && export TMPDIR=/tmp RINGO_JINDO_SPLIT=0
for line in j16 j14; do
  OUT=$R/gpurun_out/e_$line
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py --no-ntt --extra $line --no-cpu --steps 6 --warmup 1 > $OUT.json 2> $OUT.err || { echo "trace $line failed"; tail -5 $OUT.err; exit 1; }
  f=$(find $OUT -name "*kernel_stats.csv" | head -1)
  echo "== $line"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:9]:
    print(f'{float(r["AverageNs"])/1e3:10.1f} us x{int(r["Calls"]):4d}  {r["Name"][:70]}')
PY
  python3 -c "import json; d=json.load(open('$OUT.json')); j=d.get('jindo_commit_2e16') or d.get('jindo_commit'); print('commits/s', j['value'], 'ms/batch', j['ms_per_batch'])"
done
