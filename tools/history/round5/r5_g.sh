#!/bin/bash
# Round 5: COSAC instance group size A/B (16 = product, 8, 4) at configs[2] and configs[4],
# plus kernel stats of cosac2 per variant at configs[2]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
: > gpurun_out/r5g_ab.txt
for rep in 1 2; do
for v in base cos8 cos4; do
  if [ $v = base ]; then unset RINGO_LIB; else export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so; fi
  timeout -k 10 300 python3 bench.py --no-ntt --extra j14,j16 --no-cpu > gpurun_out/r5g_$v.json 2> gpurun_out/r5g_$v.err || { echo "bench $v failed"; tail -3 gpurun_out/r5g_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5g_$v.json')); print('$v', round(d['jindo_commit']['value']), round(d['jindo_commit_2e16']['value']))" | tee -a gpurun_out/r5g_ab.txt
done
done
bash tools/lib_kstats.sh "base cos8 cos4" j14 2>&1 | grep -e "==" -e cosac2 | tee -a gpurun_out/r5g_ab.txt
