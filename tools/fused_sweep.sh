#!/bin/bash
# fused NTT kernel: parity with the spin-bound check on, then bench variants (run via gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fs
RINGO_NTT_FUSED_CHECK=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_ntt.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fs/tests.log 2>&1 || { tail -30 gpurun_out/fs/tests.log; exit 1; }
tail -2 gpurun_out/fs/tests.log
for v in "${@:-0:4:6 1:4:6 2:4:6}"; do
  IFS=: read m w d <<< "$v"
  RINGO_NTT_FUSED=$m RINGO_NTT_FUSED_WPC=$w RINGO_NTT_FUSED_D=$d timeout -k 10 120 python bench.py --no-extra --no-cpu --steps 20 --warmup 3 > gpurun_out/fs/b_${m}_${w}_${d}.json 2>/dev/null || exit 1
  python3 -c "import json,sys;d=json.load(open('gpurun_out/fs/b_${m}_${w}_${d}.json'));print('$v', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['frac'],4), d['selfcheck_fwd_inv_identity'])"
done
