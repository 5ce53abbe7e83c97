#!/bin/bash
# NTT two-tiles-per-workgroup A/B: NTT parity with RINGO_NTT_TILES=2, then the NTT bench line
# alternately with 1 and 2 tiles per workgroup (same box).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
RINGO_NTT_TILES=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ntt.py > gpurun_out/j_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/j_tests.log; exit 1; }
tail -1 gpurun_out/j_tests.log
for k in 1 2 3; do
  for nt in 1 2; do
    RINGO_NTT_TILES=$nt timeout -k 10 200 python -u bench.py --no-extra --no-cpu --steps 30 --warmup 3 > gpurun_out/j_ntt_$nt.json 2> gpurun_out/j_ntt_$nt.err || { echo "bench failed"; tail -5 gpurun_out/j_ntt_$nt.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/j_ntt_$nt.json')); print('tiles $nt', round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
  done
done
