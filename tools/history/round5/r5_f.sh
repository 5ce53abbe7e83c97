#!/bin/bash
# Round 5: configs[2] commit vs batch per step (product), and one-stream (RINGO_JINDO_SPLIT=0,
# experiments build) kernel trace at 256 commits: standalone kernel times at the full launch
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for b in 256 512 1024; do
  timeout -k 10 300 python3 bench.py --no-ntt --extra j14 --no-cpu --j14-batch $b > gpurun_out/r5f_b$b.json 2> gpurun_out/r5f_b$b.err || { echo "bench $b failed"; tail -3 gpurun_out/r5f_b$b.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5f_b$b.json'))['jindo_commit']; print('batch $b', round(d['value']), round(d['ms_per_batch'],3))"
done
export RINGO_LIB=$R/ringo-snark_amd/lib/libringo_exp.so RINGO_JINDO_SPLIT=0
timeout -k 10 300 python3 bench.py --no-ntt --extra j14 --no-cpu > gpurun_out/r5f_nosplit.json 2> gpurun_out/r5f_nosplit.err || { echo "bench nosplit failed"; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5f_nosplit.json'))['jindo_commit']; print('nosplit 256', round(d['value']), round(d['ms_per_batch'],3))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5f_tr -o run -- python3 $R/bench.py --no-ntt --extra j14 --no-cpu --steps 4 --warmup 1 > $R/gpurun_out/r5f_tr.json 2> $R/gpurun_out/r5f_tr.err || { echo "trace failed"; exit 1; }
python3 $R/tools/trace_batch.py $R/gpurun_out/r5f_tr/run_kernel_trace.csv | tail -16
