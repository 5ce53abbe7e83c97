"""Timeline of one timed batch in a rocprofv3 kernel trace of a Jindo bench line (tuning aid).
usage: python tools/trace_batch.py run_kernel_trace.csv [first-kernel-substring]
Finds the last occurrence of the batch's first kernel (default cdt2_noise) that starts a batch,
prints each kernel of that batch with its stream, start offset and duration (us)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else "uniform_whole"
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
# a batch begins where the first kernel appears after a gap from the previous batch's kernels
b0 = starts[-4] if len(starts) >= 4 else starts[0]
b1 = starts[-2] if len(starts) >= 4 else len(rows)
t0 = rows[b0]["s"]
busy = {}
for r in rows[b0:b1]:
    n = r["Kernel_Name"].replace("void ", "").replace("rg::", "")[:60]
    d = (r["e"] - r["s"]) / 1e3
    print(f'q{r["Queue_Id"]:>2} +{(r["s"]-t0)/1e3:8.1f} {d:8.1f} us  {n}')
    busy[n] = busy.get(n, 0) + d
print(f"span {(max(r['e'] for r in rows[b0:b1]) - t0)/1e3:.1f} us")
for n, d in sorted(busy.items(), key=lambda x: -x[1]):
    print(f"{d:9.1f} us  {n}")
