#!/bin/bash
# Round 5: full -m gpu suite and the default bench line on the current product library
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
T=${1:-aa}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5${T}_gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5${T}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/r5${T}_gpu_tests.txt
timeout -k 10 400 python -u bench.py > gpurun_out/r5${T}_bench.json 2> gpurun_out/r5${T}_bench.err || { echo "bench failed"; tail -5 gpurun_out/r5${T}_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5${T}_bench.json'))
print('headline', round(d['value']), d['roofline']['frac'], 'floor', d.get('compute_floor_ms_per_step'), 'ms', d['ms_per_step'])
for k in ('l4_ntt','wide_ntt_zp440','wide_ntt_zp880','jindo_commit','jindo_commit_2e16','jindo_evaluate_2e16'): print(k, round(d[k]['value']))"
