#!/bin/bash
# Round-3 call: NTT pass lab (L2 prefetch variant), full -m gpu suite, default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 240 tools/nttlab/pass_lab 1024 > gpurun_out/pass_lab.txt 2>&1; echo "pass_lab rc=$?"; cat gpurun_out/pass_lab.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r03b.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/gpu_tests_r03b.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r03b.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r03b.json 2> gpurun_out/bench_r03b.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_r03b.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_r03b.json'))
print('NTT', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('valu',{}).get('compute_floor_ms_per_step'))
for k in ('jindo_commit','jindo_commit_2e16'): print(k, d[k]['value'], d[k]['ms_per_batch'])
print('l4', d['l4_ntt']['value'])
"
