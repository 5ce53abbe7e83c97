#!/bin/bash
# Round 4: the default bench line three times on one box (final library): run-to-run spread
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
: > gpurun_out/bench_repeats.txt
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py > gpurun_out/bench_rep$i.json 2> gpurun_out/bench_rep$i.err || { echo "bench $i failed"; tail -5 gpurun_out/bench_rep$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/bench_rep$i.json'))
x=[('headline', d['value'], d['roofline']['frac'])] + [(k, d[k]['value'], None) for k in ('l4_ntt','wide_ntt_zp440','wide_ntt_zp880','jindo_commit','jindo_commit_2e16','jindo_evaluate_2e16')]
print('run $i', ' | '.join('%s %.1f%s' % (k, v, (' (%.4f)' % f) if f else '') for k, v, f in x))" | tee -a gpurun_out/bench_repeats.txt
done
