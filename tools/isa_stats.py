"""Instruction mix of the kernels in a hipcc --save-temps gfx950 .s file (tuning aid).
usage: python tools/isa_stats.py file.s [name-substring]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
sub = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"^(_Z\S+):\s*;.*?$(.*?)^\.Lfunc_end", s, re.M | re.S):
    name, body = m.group(1), m.group(2)
    if sub not in name:
        continue
    ins = [l.split()[0] for l in body.split("\n") if l.startswith("\t") and not l.strip().startswith((".", ";"))]
    c = collections.Counter(ins)
    meta = re.search(r"\.name:\s+" + re.escape(name) + r"\n(?:.*\n){0,30}?\s+\.vgpr_count:\s+(\d+)", s)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    print(f"{name[:100]}  total={len(ins)} valu={valu} vgpr={meta.group(1) if meta else '?'}")
    print("   ", ", ".join(f"{k}:{v}" for k, v in sorted(c.items(), key=lambda x: -x[1])[:45]))
