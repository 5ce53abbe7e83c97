#!/bin/bash
# A/B of one bench line between the in-tree libringo.so (base) and variants in ringo-snark_amd/vlib:
#   tools/ab_line.sh "base np4 base np4" l4
set -o pipefail
R=$GRAFT_REPO_ROOT
LINE=${2:-l4}
mkdir -p $R/gpurun_out
for v in $1; do
  if [ $v = base ]; then unset RINGO_LIB; else export RINGO_LIB=$R/ringo-snark_amd/vlib/libringo_$v.so; fi
  OUT=$R/gpurun_out/ab_${v}_$LINE
  timeout -k 10 240 python3 $R/bench.py --no-ntt --extra $LINE --no-cpu --steps 20 --warmup 3 > $OUT.json 2> $OUT.err || { echo "bench $v failed"; tail -5 $OUT.err; exit 1; }
  python3 - $OUT.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k, v in d.items():
    if isinstance(v, dict) and "value" in v:
        print(sys.argv[2], k, round(v["value"], 1), v.get("unit"), v.get("ms_per_step"))
PY
done
