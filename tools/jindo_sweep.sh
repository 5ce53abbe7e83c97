#!/bin/bash
# Jindo commit: parity tests, then bench lines under env variants "VAR=val,VAR2=val" (run via gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/js
timeout -k 10 300 python -u -m pytest tests/test_gpu_jindo.py -x -q --timeout 200 --timeout-method thread > gpurun_out/js/tests.log 2>&1 || { tail -30 gpurun_out/js/tests.log; exit 1; }
tail -1 gpurun_out/js/tests.log
i=0
for v in "$@"; do
  i=$((i+1))
  env $(echo $v | tr ',' ' ') timeout -k 10 200 python bench.py --no-cpu --steps 6 --warmup 1 --batch 16 --extra j14,j16 > gpurun_out/js/b$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/js/b$i.json'));print('$v', round(d['jindo_commit']['value']), round(d['jindo_commit']['ms_per_batch'],3), round(d['jindo_commit_2e16']['value']), round(d['jindo_commit_2e16']['ms_per_batch'],3))"
done
