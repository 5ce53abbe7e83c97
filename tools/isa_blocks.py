"""Basic blocks of one kernel in a gfx950 assembly listing: label, #VALU/#SALU/#LDS/#VMEM,
and the branch at its end (to read which blocks form a hot loop).
usage: python tools/isa_blocks.py <file.s> <substring of kernel name>"""
import re
import sys

s = open(sys.argv[1]).read().split('\n')
pat = sys.argv[2]
start = next(i for i, l in enumerate(s) if pat in l and l.split(';')[0].rstrip().endswith(':') and not l.startswith(('\t', '.')))
end = next(i for i in range(start, len(s)) if s[i].startswith('.Lfunc_end'))
blk, cnt, last = 'entry', [0, 0, 0, 0, 0], ''
def flush():
    print(f"{blk:14s} valu {cnt[0]:4d} salu {cnt[1]:4d} lds {cnt[2]:3d} vmem {cnt[3]:3d} other {cnt[4]:3d}  {last}")
for l in s[start + 1:end]:
    t = l.strip()
    if re.match(r'^\.LBB\S+:', t):
        flush()
        blk, cnt, last = t.split(':')[0], [0, 0, 0, 0, 0], ''
        continue
    if not l.startswith('\t') or t.startswith(('.', ';')) or not t:
        continue
    op = t.split()[0]
    if op.startswith('v_'):
        cnt[0] += 1
    elif op.startswith('s_') and not op.startswith(('s_waitcnt', 's_nop', 's_cbranch', 's_branch', 's_endpgm')):
        cnt[1] += 1
    elif op.startswith('ds_'):
        cnt[2] += 1
    elif op.startswith(('global_', 'buffer_', 'flat_', 'scratch_')):
        cnt[3] += 1
    else:
        cnt[4] += 1
    if op.startswith(('s_cbranch', 's_branch')):
        last = t
flush()
