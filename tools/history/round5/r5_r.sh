#!/bin/bash
# Round 5: prep256 with its L-round twiddles lane-ordered in LDS (laneord): Jindo parity, A/B x2
# at configs[2] / configs[4], and its LDS bank-conflict counters at configs[4]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_laneord.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_jindo.py tests/test_gpu_jindo_2e16.py tests/test_gpu_samplers.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5r_tests.txt 2>&1 || { echo "laneord tests failed"; tail -30 gpurun_out/r5r_tests.txt; exit 1; }
tail -1 gpurun_out/r5r_tests.txt
: > gpurun_out/r5r_ab.txt
for rep in 1 2; do
for v in base laneord; do
  if [ $v = base ]; then unset RINGO_LIB; else export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so; fi
  timeout -k 10 300 python3 bench.py --no-ntt --extra j14,j16 --no-cpu > gpurun_out/r5r_$v.json 2> gpurun_out/r5r_$v.err || { echo "bench $v failed"; tail -3 gpurun_out/r5r_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5r_$v.json')); print('$v', round(d['jindo_commit']['value']), round(d['jindo_commit_2e16']['value']))" | tee -a gpurun_out/r5r_ab.txt
done
done
export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_laneord.so
bash tools/pmc_line.sh r5r_j16 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" -- --no-ntt --extra j16 --steps 2 --warmup 1 > gpurun_out/r5r_j16_summary.txt 2>&1 || { echo "pmc failed"; exit 1; }
grep -A18 "prep256" gpurun_out/r5r_j16_summary.txt | grep -e prep -e duration -e BANK -e INSTS_LDS -e WAIT_ANY
