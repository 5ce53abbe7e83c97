#!/bin/bash
# Round 5: headline NTT at 4 waves/SIMD (occ4: 40 KiB of LDS padding, 2 workgroups per CU) vs 8:
# step time and the compute floor (the same launches without HBM data, experiments build)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
: > gpurun_out/r5o_occ.txt
for rep in 1 2; do
for v in base occ4; do
  if [ $v = base ]; then unset RINGO_LIB RINGO_EXP_LIB; else export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so RINGO_EXP_LIB=$R/ringo-snark_amd/vlib/libringo_exp_$v.so; fi
  timeout -k 10 300 python3 bench.py --no-extra --no-cpu --steps 50 --warmup 5 > gpurun_out/r5o_$v.json 2> gpurun_out/r5o_$v.err || { echo "bench $v failed"; tail -3 gpurun_out/r5o_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5o_$v.json')); print('$v', round(d['value']), round(d['ms_per_step'],4), 'floor', d['valu'].get('compute_floor_ms_per_step'))" | tee -a gpurun_out/r5o_occ.txt
done
done
