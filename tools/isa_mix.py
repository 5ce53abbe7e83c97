"""Static instruction mix of kernels in a gfx950 assembly listing.
usage: python tools/isa_mix.py <file.s> <substring of mangled kernel name>..."""
import sys
from collections import Counter

s = open(sys.argv[1]).read()
for pat in sys.argv[2:]:
    key = None
    for line in s.split('\n'):
        if pat in line and not line.startswith(('.', '\t', ';')) and line.split(';')[0].rstrip().endswith(':'):
            key = line.split(':')[0]
            break
    if key is None:
        print(pat, 'not found')
        continue
    i = s.index('\n' + key + ':') + 1
    j = s.index('.Lfunc_end', i)
    body = s[i:j].split('\n')
    ins = [l.strip().split()[0] for l in body if l.startswith('\t') and not l.strip().startswith(('.', ';'))]
    c = Counter(ins)
    print(key, len(ins), 'instructions')
    print('  ', c.most_common(30))
