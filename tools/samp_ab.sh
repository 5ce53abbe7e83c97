#!/bin/bash
# Sampler A/B on the box: parity tests of the sampler/Jindo paths, then kernel stats of the j16
# (configs[4]) line with the current kernels and with RINGO_CDT=legacy RINGO_COSAC=legacy.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread ${TESTS:-tests/test_gpu_samplers.py tests/test_gpu_jindo.py} > gpurun_out/samp_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/samp_tests.log; exit 1; }
tail -2 gpurun_out/samp_tests.log
cd /tmp && export TMPDIR=/tmp
for v in new legacy; do
  OUT=$R/gpurun_out/samp_$v
  if [ $v = legacy ]; then export RINGO_CDT=legacy RINGO_COSAC=legacy; else unset RINGO_CDT RINGO_COSAC; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py --no-ntt --extra ${LINE:-j16} --no-cpu --steps 4 --warmup 1 > $OUT.json 2> $OUT.err || { echo "trace $v failed"; tail -5 $OUT.err; exit 1; }
  f=$(find $OUT -name "*kernel_stats.csv" | head -1)
  echo "== $v"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["AverageNs"])/1e3:10.1f} us x{int(r["Calls"]):4d}  {r["Name"][:90]}')
PY
  python3 -c "import json,sys; d=json.load(open('$OUT.json')); j=d.get('jindo_commit_2e16') or d.get('jindo_commit'); print('commits/s', j['value'], 'ms/batch', j['ms_per_batch'])"
done
