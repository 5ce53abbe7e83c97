#!/bin/bash
# Single-stream (RINGO_JINDO_SPLIT=0) kernel stats of the j16 line, current vs legacy samplers,
# then PMC passes over the current sampler kernels.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp RINGO_JINDO_SPLIT=0
for v in new legacy; do
  OUT=$R/gpurun_out/iso_$v
  if [ $v = legacy ]; then export RINGO_CDT=legacy RINGO_COSAC=legacy; else unset RINGO_CDT RINGO_COSAC; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/bench.py --no-ntt --extra j16 --no-cpu --steps 4 --warmup 1 > $OUT.json 2> $OUT.err || { echo "trace $v failed"; tail -5 $OUT.err; exit 1; }
  f=$(find $OUT -name "*kernel_stats.csv" | head -1)
  echo "== $v"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f'{float(r["AverageNs"])/1e3:10.1f} us x{int(r["Calls"]):4d}  {r["Name"][:90]}')
PY
  python3 -c "import json; d=json.load(open('$OUT.json')); j=d['jindo_commit_2e16']; print('commits/s', j['value'], 'ms/batch', j['ms_per_batch'])"
done
unset RINGO_CDT RINGO_COSAC
mkdir -p $R/gpurun_out/sampmc
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $R/gpurun_out/sampmc/p$i -o run -- python3 $R/bench.py --no-ntt --extra j16 --no-cpu --no-prewarm --steps 2 --warmup 0 > /dev/null 2>$R/gpurun_out/sampmc/p$i.err || { echo "pmc pass $i failed"; tail -3 $R/gpurun_out/sampmc/p$i.err; exit 1; }
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/sampmc | grep -A14 -E "cdt2|cosac2|mlwe_noise|uniform_elems|prep256|mac3h|digits" | head -120
