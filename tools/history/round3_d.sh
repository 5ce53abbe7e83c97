#!/bin/bash
# Counter-mode caching A/B (cdt2): sampler parity incl. the IV-boundary seeds, then kernel stats of
# the j16 line (single stream) with the current library and with lib/nopre (RG_CTR_PREFIX=0).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_samplers.py > gpurun_out/pre_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/pre_tests.log; exit 1; }
tail -2 gpurun_out/pre_tests.log
cd /tmp && export TMPDIR=/tmp RINGO_JINDO_SPLIT=0
for v in pre nopre; do
  OUT=$R/gpurun_out/ab_$v
  if [ $v = nopre ]; then export RINGO_LIB=$R/ringo-snark_amd/lib/nopre/libringo.so; else unset RINGO_LIB; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py --no-ntt --extra j16 --no-cpu --steps 6 --warmup 1 > $OUT.json 2> $OUT.err || { echo "trace $v failed"; tail -5 $OUT.err; exit 1; }
  f=$(find $OUT -name "*kernel_stats.csv" | head -1)
  echo "== $v"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:9]:
    print(f'{float(r["AverageNs"])/1e3:10.1f} us x{int(r["Calls"]):4d}  {r["Name"][:70]}')
PY
  python3 -c "import json; d=json.load(open('$OUT.json')); j=d['jindo_commit_2e16']; print('commits/s', j['value'], 'ms/batch', j['ms_per_batch'])"
done
