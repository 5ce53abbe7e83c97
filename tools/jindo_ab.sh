#!/bin/bash
# A/B of the Jindo bench lines under environment variants (run on the box via gpurun):
#   tools/jindo_ab.sh VAR "val1 val2 ..." [extra lines, default j14,j16]
# prints commits/s and ms per batch (sampled and injected) for each value of $VAR
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VAR=$1
VALS=$2
LINES=${3:-j14,j16}
for v in $VALS; do
  env $VAR=$v timeout -k 10 240 python bench.py --no-ntt --extra $LINES --no-cpu > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/ab_$v.err; exit 1; }
  python3 - "$v" <<'EOF'
import json, sys
v = sys.argv[1]
d = json.load(open(f"gpurun_out/ab_{v}.json"))
for k in ("jindo_commit", "jindo_commit_2e16"):
    if k in d:
        print(v, k, round(d[k]["value"]), "ms", round(d[k]["ms_per_batch"], 3), "injected ms", round(d[k]["injected"]["ms_per_batch"], 3))
EOF
done
