#!/bin/bash
# Sampler iteration loop: parity tests of the samplers, then single-stream kernel stats of j16.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_samplers.py ${EXTRA_TESTS:-} > gpurun_out/sq_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/sq_tests.log; exit 1; }
tail -2 gpurun_out/sq_tests.log
cd /tmp && export TMPDIR=/tmp RINGO_JINDO_SPLIT=0 RINGO_LIB=$R/ringo-snark_amd/lib/libringo_exp.so  # the switch lives in the experiments build
OUT=$R/gpurun_out/sq_new
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py --no-ntt --extra j16 --no-cpu --steps 4 --warmup 1 > $OUT.json 2> $OUT.err || { echo "trace failed"; tail -5 $OUT.err; exit 1; }
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:10]:
    print(f'{float(r["AverageNs"])/1e3:10.1f} us x{int(r["Calls"]):4d}  {r["Name"][:90]}')
PY
python3 -c "import json; d=json.load(open('$OUT.json')); j=d['jindo_commit_2e16']; print('single-stream commits/s', j['value'], 'ms/batch', j['ms_per_batch'])"
unset RINGO_JINDO_SPLIT RINGO_LIB
cd $R && timeout -k 10 240 python3 bench.py --no-ntt --extra j16 --no-cpu --steps 6 --warmup 1 > gpurun_out/sq_split.json 2> gpurun_out/sq_split.err && python3 -c "import json; d=json.load(open('gpurun_out/sq_split.json')); j=d['jindo_commit_2e16']; print('split commits/s', j['value'], 'ms/batch', j['ms_per_batch'])"
if [ -x tools/nttlab/mem_lab ]; then timeout -k 10 120 tools/nttlab/mem_lab 1024 > gpurun_out/mem_lab.txt 2>&1; cat gpurun_out/mem_lab.txt; fi
