#!/bin/bash
# Round 5: three default bench.py runs back to back on one box (the spread of every line)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py > gpurun_out/r5am_bench_$i.json 2> gpurun_out/r5am_bench_$i.err || { echo "bench $i failed"; tail -5 gpurun_out/r5am_bench_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r5am_bench_$i.json'))
print('run $i', 'headline', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['frac'],4), 'floor', round(d['roofline']['valu']['compute_floor_ms_per_step'],4),
      ' '.join(f\"{k}={round(d[k]['value'])}\" for k in ('l4_ntt','wide_ntt_zp440','wide_ntt_zp880','jindo_commit','jindo_commit_2e16','jindo_evaluate_2e16')))"
done
