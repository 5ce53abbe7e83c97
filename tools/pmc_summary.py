"""Summarise rocprofv3 --pmc CSVs: per kernel name, mean counter value per dispatch."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/**/*kernel_trace.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for name, cs in acc.items():
    if "rg::" not in name:
        continue
    print(name[:110])
    d = sum(dur[name]) / max(len(dur[name]), 1)
    print(f"   mean duration (profiled) {d/1e3:.1f} us over {len(dur[name])} dispatches")
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v)/len(v):16.4g}")
