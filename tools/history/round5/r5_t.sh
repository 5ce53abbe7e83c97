#!/bin/bash
# Round 5: full -m gpu suite on the cleaned product library, smoke(), and one default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5t_gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5t_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/r5t_gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5t_smoke.txt 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r5t_smoke.txt; exit 1; }
tail -1 gpurun_out/r5t_smoke.txt
timeout -k 10 400 python -u bench.py > gpurun_out/r5t_bench.json 2> gpurun_out/r5t_bench.err || { echo "bench failed"; tail -5 gpurun_out/r5t_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5t_bench.json'))
print('headline', round(d['value']), round(d['ms_per_step'],4), d['roofline']['frac'])
for k in ('l4_ntt','wide_ntt_zp440','wide_ntt_zp880','jindo_commit','jindo_commit_2e16','jindo_evaluate_2e16'): print(k, round(d[k]['value']))"
