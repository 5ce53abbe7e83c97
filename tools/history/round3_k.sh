#!/bin/bash
# NTT L-round twiddles in LDS: NTT parity, then the NTT bench line alternately with the current
# library and vlib/noltw (RG_NTT_LTW=0, per-lane global twiddle loads), same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ntt.py > gpurun_out/k_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/k_tests.log; exit 1; }
tail -1 gpurun_out/k_tests.log
for k in 1 2 3; do
  for v in ltw noltw; do
    if [ $v = noltw ]; then export RINGO_LIB=$R/ringo-snark_amd/vlib/noltw/libringo.so; else unset RINGO_LIB; fi
    timeout -k 10 200 python -u bench.py --no-extra --no-cpu --steps 30 --warmup 3 > gpurun_out/k_ntt_$v.json 2> gpurun_out/k_ntt_$v.err || { echo "bench failed"; tail -5 gpurun_out/k_ntt_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/k_ntt_$v.json')); print('$v', round(d['ms_per_step'],4), round(d['roofline']['frac'],4), round(d['roofline']['valu']['compute_floor_ms_per_step'],4))"
  done
done
