#!/bin/bash
# Round 5: L = 4 NTT (ntt256_pass) with wave-private exchanges (l4wl) vs barriers (l4base):
# L = 4 NTT parity on l4wl, A/B x3 of the l4 line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_l4wl.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_ntt.py tests/test_gpu_buckler.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5m_tests.txt 2>&1 || { echo "l4wl tests failed"; tail -30 gpurun_out/r5m_tests.txt; exit 1; }
tail -1 gpurun_out/r5m_tests.txt
: > gpurun_out/r5m_ab.txt
for rep in 1 2 3; do
for v in l4base l4wl; do
  export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so
  timeout -k 10 300 python3 bench.py --no-ntt --extra l4 --no-cpu > gpurun_out/r5m_$v.json 2> gpurun_out/r5m_$v.err || { echo "bench $v failed"; tail -3 gpurun_out/r5m_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5m_$v.json'))['l4_ntt']; print('$v', round(d['value']), round(d.get('ms_per_step',0),4), d.get('compute_floor_ms_per_step'))" | tee -a gpurun_out/r5m_ab.txt
done
done
