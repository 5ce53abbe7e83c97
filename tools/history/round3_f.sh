#!/bin/bash
# NTT (COL M-round scalar twiddles) + prep256 borrow-select: NTT + Jindo parity, the NTT bench line
# (with its compute floor), then kernel stats of the j16 line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ntt.py tests/test_gpu_jindo.py tests/test_gpu_jindo_2e16.py > gpurun_out/f_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/f_tests.log; exit 1; }
tail -2 gpurun_out/f_tests.log
timeout -k 10 300 python -u bench.py --no-extra --no-cpu --steps 20 --warmup 3 > gpurun_out/f_ntt.json 2> gpurun_out/f_ntt.err || { echo "ntt bench failed"; tail -5 gpurun_out/f_ntt.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/f_ntt.json')); print('ntt', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['valu'].get('compute_floor_ms_per_step'))"
timeout -k 10 300 python -u bench.py --no-extra --no-cpu --steps 20 --warmup 3 > gpurun_out/f_ntt2.json 2> gpurun_out/f_ntt2.err || { echo "ntt bench failed"; tail -5 gpurun_out/f_ntt2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/f_ntt2.json')); print('ntt', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['valu'].get('compute_floor_ms_per_step'))"
cd /tmp && export TMPDIR=/tmp RINGO_JINDO_SPLIT=0
OUT=$R/gpurun_out/f_j16
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
