#!/bin/bash
# Round 4: wide-field (zp440 / zp880) NTT parity on the GPU, then the wide bench line with the
# LDS-tiled pass kernel (product) and the per-stage kernels (experiments build, RINGO_NTT_KERNEL=stage).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ntt.py tests/test_gpu_buckler.py > gpurun_out/wide_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/wide_tests.log; exit 1; }
tail -2 gpurun_out/wide_tests.log
timeout -k 10 200 python3 bench.py --no-ntt --extra wide --no-cpu --steps 8 > gpurun_out/wide_bench.json 2> gpurun_out/wide_bench.err || { echo BENCH FAILED; tail -5 gpurun_out/wide_bench.err; exit 1; }
cat gpurun_out/wide_bench.json
RINGO_LIB=$R/ringo-snark_amd/lib/libringo_exp.so RINGO_NTT_KERNEL=stage timeout -k 10 300 python3 bench.py --no-ntt --extra wide --no-cpu --steps 8 > gpurun_out/wide_bench_stage.json 2> gpurun_out/wide_bench_stage.err || { echo STAGE BENCH FAILED; tail -5 gpurun_out/wide_bench_stage.err; exit 1; }
cat gpurun_out/wide_bench_stage.json
