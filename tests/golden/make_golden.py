"""Generate the committed parity fixtures under tests/golden/ from the oracle restatements
(oracle/pyref.py, oracle/liboracle.so).  Run in the build container:  python tests/golden/make_golden.py

Fixtures (data only):
  jindo_params.json  Jindo shapes for the BASELINE configs + jindo_test sizes, from the
                     restatement of jindo.NewParameters (params.go:126-320) and Lattigo's
                     NTT-friendly prime generator (third-party: Go float/Lattigo parity unpinned).
  ntt_golden.json    SHA-256 digests of oracle NTT outputs on SplitMix64 inputs for every field
                     and several ranks (regression pins for the restatement itself).
  jindo_commit_golden.json  digests of one oracle commit at targetN 2^10 (jindo_test size) with
                     seeded injected randomness + the CK digest for crs "Jindo!".
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)

import coracle as co  # noqa: E402
import pyref  # noqa: E402
from tests.jindo_util import make_randomness, make_v  # noqa: E402

Q255 = 0x430D45996B62AFC2D65643D9E6FB65558E9630DC8C3732810000000000000001
Q128 = 0x82BD02ADD980D88E6706E10000000001

CONFIGS = {
    "t10_b1": (Q255, 1 << 10, 1),
    "t10_b8": (Q255, 1 << 10, 8),
    "t14_b1": (Q255, 1 << 14, 1),        # configs[2]
    "t16_b1": (Q255, 1 << 16, 1),
    "t16_b4096": (Q255, 1 << 16, 4096),  # configs[4]
    "mult_t8193_b12": (Q128, 8193, 12),  # configs[0] (examples/mult at rank 2^12)
}
# the other fields of the zp package as Jindo fields (buckler/compile.go:178 commits Buckler
# witnesses with jindo.NewParameters[E] of the Buckler field): every encode exponent 4 .. 64, field
# limbs 1, 2, 4, 7, 14, one- and two-prime rings, both sides of prep256's lazy-butterfly bound
_FIELDS = json.load(open(os.path.join(HERE, "fields.json")))
for _name, _f, _tn, _b in (("p63_t10_b2", "p63", 1 << 10, 2), ("zp110_t10_b1", "zp110", 1 << 10, 1),
                           ("zp220_t10_b1", "zp220", 1 << 10, 1), ("zp440_t10_b2", "zp440", 1 << 10, 2),
                           ("zp880_t10_b1", "zp880", 1 << 10, 1), ("zp440_t14_b1", "zp440", 1 << 14, 1),
                           ("zp880_t14_b1", "zp880", 1 << 14, 1)):
    CONFIGS[_name] = (int(_FIELDS[_f]["q_hex"], 16), _tn, _b)


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    params = {}
    for name, (q, tn, b) in CONFIGS.items():
        P = pyref.JindoParams(q, tn, b).as_dict()
        P["field_q_hex"] = hex(q)
        P["target_n"] = tn
        params[name] = P
    json.dump(params, open(os.path.join(HERE, "jindo_params.json"), "w"), indent=1)

    fields = json.load(open(os.path.join(HERE, "fields.json")))
    ntt = {}
    for name, f in sorted(fields.items()):
        q = int(f["q_hex"], 16)
        cf = co.CField(q)
        L = cf.L
        for logn in [3, 8, 12]:
            N = 1 << logn
            if (q - 1) % (2 * N):
                continue
            for cyc in [False, True]:
                tw, twi, ninv = cf.tables(N, cyclic=cyc)
                rng = np.random.default_rng(logn * 1000 + L)
                vals = [int.from_bytes(rng.bytes(8 * L), "little") % q for _ in range(N)]
                a = co.to_limbs(vals, L)[None]
                y = cf.ntt_fwd(a, tw)
                z = cf.ntt_inv(a, twi, ninv)
                ntt[f"{name}/{logn}/{'cyclic' if cyc else 'nega'}"] = {
                    "seed": logn * 1000 + L, "tw": digest(tw), "twinv": digest(twi), "fwd": digest(y),
                    "inv": digest(z), "fwd_head": [str(int(x)) for x in y.reshape(-1)[:4]]}
    json.dump(ntt, open(os.path.join(HERE, "ntt_golden.json"), "w"), indent=1, sort_keys=True)

    # one commit at the jindo_test size with seeded randomness
    P = params["t10_b1"]
    F = pyref.Field(Q255)
    ck = pyref.commit_key(pyref.JindoParams(Q255, 1 << 10, 1), b"Jindo!")
    ck_np = [np.array(x, dtype=np.uint64) for x in ck]
    cj = co.CJindo(P, Q255)
    out = {"ck": [digest(x) for x in ck_np], "cases": {}}
    for nv in [1024, 300, 1]:
        v = make_v(Q255, nv, seed=nv)
        rnd = make_randomness(P, Q255, seed=nv + 1)
        o = cj.commit(ck_np[0], ck_np[1], ck_np[2], v, rnd["last_row"], rnd["mask"], rnd["enc_noise"],
                      rnd["mlwe_noise"])
        out["cases"][str(nv)] = {k: digest(val) for k, val in o.items()}
    json.dump(out, open(os.path.join(HERE, "jindo_commit_golden.json"), "w"), indent=1, sort_keys=True)
    print("fixtures written")


if __name__ == "__main__":
    main()
