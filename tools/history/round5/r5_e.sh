#!/bin/bash
# Round 5: full -m gpu suite on the product library, then the configs[2] / configs[4] Jindo
# lines' kernel traces (timeline + stats) for the commit work
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5e_gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r5e_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r5e_gpu_tests.txt
cd /tmp && export TMPDIR=/tmp
for line in j14 j16; do
  OUT=$R/gpurun_out/r5e_$line
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py --no-ntt --extra $line --no-cpu --steps 4 --warmup 1 > $OUT.json 2> $OUT.err || { echo "trace $line failed"; tail -5 $OUT.err; exit 1; }
done
for line in j14 j16; do
  timeout -k 10 300 python3 $R/bench.py --no-ntt --extra $line --no-cpu > $R/gpurun_out/r5e_bench_$line.json 2> $R/gpurun_out/r5e_bench_$line.err || { echo "bench $line failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$R/gpurun_out/r5e_bench_$line.json')); k=[x for x in d if x.startswith('jindo_commit')][0]; print('$line', k, round(d[k]['value']), round(d[k]['ms_per_batch'],3))"
done
