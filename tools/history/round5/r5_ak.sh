#!/bin/bash
# Round 5: NTT batch chunking after the reverse-order / default-store change: chunks over two
# streams (vlib d128 / d256 / d512) and single-stream chunks (experiments build, RINGO_NTT_CHUNK_MB)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_d128.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ntt.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5ak_tests.txt 2>&1 || { echo "tests failed"; tail -20 gpurun_out/r5ak_tests.txt; exit 1; }
tail -1 gpurun_out/r5ak_tests.txt
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python3 bench.py --no-extra --no-cpu --steps 50 --warmup 5 > gpurun_out/ak_$n.json 2> gpurun_out/ak_$n.err || { echo "bench $n failed"; tail -5 gpurun_out/ak_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ak_$n.json').read().strip().splitlines()[-1]); print('$n', round(d['value']), round(d['ms_per_step'],4))"
}
for rep in 1 2 3; do
  run base RINGO_DUMMY=1
  for c in d128 d256 d512; do run $c RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$c.so; done
  run s64 RINGO_LIB=$R/ringo-snark_amd/lib/libringo_exp.so RINGO_NTT_CHUNK_MB=64
  run s128 RINGO_LIB=$R/ringo-snark_amd/lib/libringo_exp.so RINGO_NTT_CHUNK_MB=128
done
