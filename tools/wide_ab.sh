#!/bin/bash
# A/B of wide-field NTT variants (tools/wide_ab_build.sh) on one box: the wide bench line per
# library, two rounds in alternating order.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
out=gpurun_out/wide_ab.txt
: > $out
for rep in 1 2; do
  for v in "$@"; do
    RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so timeout -k 10 200 python3 bench.py --no-ntt --extra wide --no-cpu --steps 8 > gpurun_out/wab_$v.json 2> gpurun_out/wab_$v.err || { echo "$v FAILED"; tail -5 gpurun_out/wab_$v.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/wab_$v.json'))
print('$v', ' '.join('%s %.1f NTT/s %.3f ms ok=%s' % (k, d[k]['value'], d[k]['ms_per_step'], d[k]['selfcheck_fwd_inv_identity']) for k in ('wide_ntt_zp440','wide_ntt_zp880')))" | tee -a $out
  done
done
