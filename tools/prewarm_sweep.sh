set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "0.3 20" "0.3 200" "2 20" "2 200" "0.3 20"; do
  set -- $cfg
  RINGO_PREWARM_S=$1 timeout -k 10 120 python3 bench.py --no-extra --no-cpu --steps $2 --warmup 3 > gpurun_out/pw_$1_$2.json 2>gpurun_out/pw.err || { tail -3 gpurun_out/pw.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/pw_$1_$2.json').read().strip().splitlines()[-1]);print('$1 $2', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
done
