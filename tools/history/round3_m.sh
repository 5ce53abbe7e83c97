#!/bin/bash
# MFMA MAC round: default bench line, A/B bench with mac3h (RINGO_JINDO_MAC=h), then the -m gpu suite.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/m_bench.json 2> gpurun_out/m_bench.err || { echo BENCH FAILED; tail -20 gpurun_out/m_bench.err; exit 1; }
python3 - <<'PY'
import json
d=json.load(open("gpurun_out/m_bench.json"))
print("ntt", d["value"], d["ms_per_step"])
for k in ("jindo_commit","jindo_commit_2e16"):
    x=d[k]; print(k, round(x["value"]), round(x["ms_per_batch"],3), "injected", round(x["injected"]["value"]))
PY
RINGO_JINDO_MAC=h timeout -k 10 400 python -u bench.py > gpurun_out/m_bench_h.json 2> gpurun_out/m_bench_h.err || { echo BENCH_H FAILED; tail -20 gpurun_out/m_bench_h.err; exit 1; }
python3 - <<'PY'
import json
d=json.load(open("gpurun_out/m_bench_h.json"))
for k in ("jindo_commit","jindo_commit_2e16"):
    x=d[k]; print("mac3h", k, round(x["value"]), round(x["ms_per_batch"],3), "injected", round(x["injected"]["value"]))
PY
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/m_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/m_gpu_tests.log; exit 1; }
tail -2 gpurun_out/m_gpu_tests.log
