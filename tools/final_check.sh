#!/bin/bash
# Round-end evidence on the GPU box for THIS libringo.so: profiles (kernel stats + per-line PMC ->
# kernel_counters.json), the whole -m gpu suite, smoke(), and the default bench line (which reads
# the fresh kernel_counters.json).  usage: tools/final_check.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-final}
cd $R && mkdir -p gpurun_out
bash tools/profile_bench.sh $R/gpurun_out/prof_$T > gpurun_out/prof_$T.log 2>&1 || { echo "profile failed"; tail -5 gpurun_out/prof_$T.log; exit 1; }
cp gpurun_out/prof_$T/kernel_counters.json profiles/kernel_counters.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1 || { echo "gpu tests failed"; tail -20 gpurun_out/gpu_tests_$T.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$T.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { echo "bench failed"; tail -5 gpurun_out/bench_$T.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$T.json'));print(d['value'],d['roofline']['frac'],d['jindo_commit']['value'],d['jindo_commit_2e16']['value'])"
