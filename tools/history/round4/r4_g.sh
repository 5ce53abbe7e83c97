#!/bin/bash
# Round 4: the full GPU suite after the digits fromMont (REDC-only) and wide-inverse (per-stage
# halving) changes, then the wide bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/g_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/g_tests.log; exit 1; }
tail -2 gpurun_out/g_tests.log
timeout -k 10 200 python3 bench.py --no-ntt --extra wide --no-cpu --steps 8 > gpurun_out/g_wide_bench.json 2> gpurun_out/g_wide_bench.err || { echo BENCH FAILED; tail -5 gpurun_out/g_wide_bench.err; exit 1; }
cat gpurun_out/g_wide_bench.json
