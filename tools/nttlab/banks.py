# half-wave model: ds_*_b64, 32 lanes per cycle, 64 banks x 4 B; u64 index p occupies banks 2p, 2p+1 (mod 64)
import itertools
def xH(t, y): return t + 32 * y
def xM(t, y): return ((t >> 2) << 5) | (y << 2) | (t & 3)
def xL(t, r): return 8 * t + r
PATS = {'H': xH, 'M': xM, 'L': xL}
def lanes(col, sw):
    out = []
    for tid in range(64):
        if col: s, t = tid % sw, tid // sw
        else: s, t = tid // 32, tid % 32
        out.append((s, t))
    return out
def conflict_free(pos, pat, col, sw):
    L = lanes(col, sw)
    for v in range(8):
        for half in (L[:32], L[32:]):
            banks = set()
            for (s, t) in half:
                p = pos(s, PATS[pat](t, v))
                for b in (2 * p % 64, (2 * p + 1) % 64):
                    if b in banks: return False
                    banks.add(b)
    return True
sw = 4
for col in (True, False):
    print("COL" if col else "ROW")
    for ex in [('H', 'M'), ('M', 'L'), ('L', 'H')]:
        found = []
        for padn in range(256, 256 + 64):
            for name, f in [('0', lambda x: 0), ('x>>5', lambda x: x >> 5), ('4(x>>5)', lambda x: 4 * (x >> 5)),
                            ('x>>3', lambda x: x >> 3), ('(x>>3)&7', lambda x: (x >> 3) & 7), ('2(x>>5)', lambda x: 2 * (x >> 5)),
                            ('x>>4', lambda x: x >> 4), ('8(x>>5)', lambda x: 8 * (x >> 5)), ('(x>>5)+(x>>3)', lambda x: (x>>5)+(x>>3))]:
                pos = lambda s, x, padn=padn, f=f: s * padn + x + f(x)
                if all(conflict_free(pos, p, col, sw) for p in ex):
                    found.append((padn, name))
        print(" ", ex, found[:6])
