#!/bin/bash
# One-box A/B of library variants (tools/var_build.sh) on bench lines:
#   tools/lib_ab.sh <lines, e.g. j14,j16> <name> ...   (two rounds, alternating order)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
lines=$1; shift
out=gpurun_out/lib_ab.txt
: > $out
for rep in 1 2; do
  for v in "$@"; do
    RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so timeout -k 10 300 python3 bench.py --no-ntt --extra $lines --no-cpu > gpurun_out/lab_$v.json 2> gpurun_out/lab_$v.err || { echo "$v FAILED"; tail -5 gpurun_out/lab_$v.err; exit 1; }
    python3 - "$v" <<'PY' | tee -a $out
import json, sys
v = sys.argv[1]
d = json.load(open(f"gpurun_out/lab_{v}.json"))
parts = []
for k, x in d.items():
    if isinstance(x, dict) and "value" in x:
        ms = x.get("ms_per_batch", x.get("ms_per_step"))
        parts.append(f"{k} {x['value']:.1f} ms {ms:.3f}" if ms is not None else f"{k} {x['value']:.1f}")
print(v, " | ".join(parts))
PY
  done
done
