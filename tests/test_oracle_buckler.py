"""CPU: the C oracle's Buckler prover restatements (oracle.c of_buckler_encode /
of_buckler_eval_circuit, restating buckler/encoder.go:32-54 and buckler/prover.go:355-379)
pinned by what they compute, independently of the loops:
  * Encode: the output is a polynomial of degree < embRank whose reduction mod X^rank - 1 has
    cyclic NTT (the oracle's transform, pinned in test_oracle.py) equal to v; coefficients
    rank+1.. are zero, and RandEncode's reduction equals Encode's (r (X^rank - 1) vanishes on the
    evaluation points) with coefficient rank = r;
  * evalCircuit: pointwise sum_c bc * sum_t coeff * pw * prod w in Python integers on the
    Montgomery representatives (a.b.R^-1 per product)."""
import numpy as np
import pytest

import coracle as co


def _rand(cf, n, rng):
    v = [int.from_bytes(rng.bytes(8 * cf.L + 8), "little") % cf.q for _ in range(n)]
    return co.to_limbs(v, cf.L)


@pytest.mark.parametrize("key", ["p63", "mult_zp", "jindo_zp"])
@pytest.mark.parametrize("rank,emb", [(16, 32), (64, 65), (256, 1024)])
def test_encode_pinned(fields, key, rank, emb):
    q = fields[key]
    cf = co.CField(q)
    rng = np.random.default_rng(rank * 7 + emb)
    v = _rand(cf, rank, rng)
    out = cf.buckler_encode(v, emb)
    assert (out[rank:] == 0).all()
    tw, _, _ = cf.tables(rank, cyclic=True)
    assert (cf.ntt_fwd(out[None, :rank], tw)[0] == v).all()
    r = _rand(cf, 1, rng)[0]
    outr = cf.buckler_encode(v, emb, rnd=r)
    assert (outr[rank] == r).all() and (outr[rank + 1:] == 0).all() and (outr[1:rank] == out[1:rank]).all()
    folded = outr[:rank].copy()
    folded[0] = co.to_limbs([(co.from_limbs(outr[:1])[0] + co.from_limbs(outr[rank:rank + 1])[0]) % q], cf.L)[0]
    assert (folded == out[:rank]).all()


@pytest.mark.parametrize("key", ["p63", "mult_zp", "jindo_zp"])
def test_eval_circuit_pinned(fields, key):
    q = fields[key]
    cf = co.CField(q)
    L = cf.L
    Rinv = pow(1 << (64 * L), -1, q)
    rng = np.random.default_rng(11)
    rank, nw, npw = 32, 4, 2
    w = _rand(cf, nw * rank, rng).reshape(nw, rank, L)
    pw = _rand(cf, npw * rank, rng).reshape(npw, rank, L)
    co_ = lambda: _rand(cf, 1, rng)[0]  # noqa: E731
    cons = [
        [(co_(), None, [0, 1]), (co_(), 1, [2]), (co_(), None, [3])],  # a*b + pw1*c + d
        [],                                                            # empty constraint
        [(co_(), 0, []), (co_(), None, []), (co_(), None, [2, 2, 2])],  # pw0, constant, c^3
    ]
    bc = co_()
    got = cf.buckler_eval_circuit(cons, bc, w, pw)
    W = [[co.from_limbs(w[i, j:j + 1])[0] for j in range(rank)] for i in range(nw)]
    P = [[co.from_limbs(pw[i, j:j + 1])[0] for j in range(rank)] for i in range(npw)]
    B = co.from_limbs(bc[None])[0]
    mm = lambda a, b: a * b * Rinv % q  # noqa: E731
    for j in range(rank):
        acc = 0
        for c in cons:
            ev = 0
            for coeff, p, ws in c:
                t = co.from_limbs(np.asarray(coeff)[None])[0]
                if p is not None:
                    t = mm(t, P[p][j])
                for k in ws:
                    t = mm(t, W[k][j])
                ev = (ev + t) % q
            acc = (acc + mm(ev, B)) % q
        assert co.from_limbs(got[j:j + 1])[0] == acc
