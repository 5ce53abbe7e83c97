#!/bin/bash
# Round-3 combined GPU call: sampler parity + A/B kernel stats, NTT line with its compute floor,
# VALU op costs (tools/ubench/ops3), the box's counter list.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 60 tools/ubench/ops3 > gpurun_out/ops3.txt 2>&1 && cat gpurun_out/ops3.txt || echo "ops3 failed"
timeout -k 10 400 bash tools/samp_ab.sh || exit 1
cd $R
timeout -k 10 300 python -u bench.py --no-extra --no-cpu --steps 20 --warmup 3 > gpurun_out/ntt_probe.json 2> gpurun_out/ntt_probe.err || { echo NTT BENCH FAILED; tail -20 gpurun_out/ntt_probe.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ntt_probe.json')); print('NTT', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('valu'))"
cd /tmp && export TMPDIR=/tmp && timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || echo "counter list failed"
grep -c "" $R/gpurun_out/counters_list.txt
