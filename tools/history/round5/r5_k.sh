#!/bin/bash
# Round 5: full -m gpu suite on the DAG product library, the default bench line, and the
# configs[4] commit timeline (kernel trace)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5k_gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5k_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/r5k_gpu_tests.txt
timeout -k 10 400 python -u bench.py > gpurun_out/r5k_bench.json 2> gpurun_out/r5k_bench.err || { echo "bench failed"; tail -5 gpurun_out/r5k_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5k_bench.json'))
print('headline', round(d['value']), d['roofline']['frac'])
for k in ('l4_ntt','wide_ntt_zp440','wide_ntt_zp880','jindo_commit','jindo_commit_2e16','jindo_evaluate_2e16'): print(k, round(d[k]['value']))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r5k_tr16 -o run -- python3 $R/bench.py --no-ntt --extra j16 --no-cpu --steps 4 --warmup 1 > $R/gpurun_out/r5k_tr16.json 2> $R/gpurun_out/r5k_tr16.err || { echo "trace failed"; exit 1; }
