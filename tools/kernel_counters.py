"""Collect rocprofv3 PMC passes of single bench lines into profiles/kernel_counters.json.

usage: python tools/kernel_counters.py <profile-dir> <out.json> <libringo.so>
<profile-dir>/<line>/p<i>/run_counter_collection.csv (one counter group per pass) and
<profile-dir>/<line>/bench.json (the bench line of that run, which reports steps_executed)
are read; for every libringo kernel of the line the counter values are SUMMED over its
dispatches (bench.py divides by the steps that run executed, then by the units per step).
FETCH_SIZE / WRITE_SIZE are in KiB as rocprofv3 reports them (bench.py applies the gfx950
x2 correction to FETCH_SIZE, MI355X_MICROARCH.md "HBM")."""
import csv
import glob
import hashlib
import json
import os
import sys
from collections import defaultdict

root, out, lib = sys.argv[1], sys.argv[2], sys.argv[3]
res = {"lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
       "source": f"rocprofv3 --pmc passes of single bench lines ({os.path.basename(root.rstrip('/'))})", "lines": {}}
for ldir in sorted(glob.glob(os.path.join(root, "*"))):
    line = os.path.basename(ldir)
    bj = os.path.join(ldir, "bench.json")
    if not os.path.exists(bj):
        continue
    b = json.loads([l for l in open(bj) if l.startswith("{")][-1])
    steps = b["steps_executed"].get(line)
    if not steps:
        continue
    acc = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(int)
    for f in sorted(glob.glob(os.path.join(ldir, "p*", "**", "*counter_collection.csv"), recursive=True)):
        seen = set()
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "rg::" not in name:
                continue
            acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), name)
            if key not in seen:
                seen.add(key)
                calls[(f, name)] += 1
    kern = {}
    for name, cs in acc.items():
        kern[name] = dict(cs)
        kern[name]["dispatches_per_pass"] = max(v for (f, n), v in calls.items() if n == name)
    res["lines"][line] = {"steps": steps, "steps_executed": b["steps_executed"], "kernels": kern}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: {"steps": v["steps"], "kernels": len(v["kernels"])} for k, v in res["lines"].items()}))
