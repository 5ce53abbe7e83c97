"""CPU: the C oracle's remaining bigpoly operators (oracle.c of_quorem_vanishing / of_aut /
of_poly_evaluate, restating math/bigpoly/cyclic.go:18-37, cyclotomic.go:29-86, poly.go:64-76)
pinned by the mathematics they implement, independently of the loops:
  * p = quo (X^N - 1) + rem with deg rem < N;
  * NTT(Aut_idx(p)) = Aut_idx(NTT(p)) between the coefficient and NTT-domain paths, through the
    oracle's negacyclic transform (itself pinned in test_oracle.py), and Aut is the ring map
    X -> X^idx of Z_q[X]/(X^N + 1) (checked on monomials);
  * Evaluate = sum p_i x^i in Python integers (Montgomery representatives in and out);
  * ModSwitch (pyref.mod_switch, cyclotomic.go:98-124) = ceil(p q / qBig - 1/2) mod q in exact
    rationals: the reference's remainder rule is round-half-down, for either sign of p."""
import numpy as np
import pytest

import coracle as co


def _rand(cf, n, rng):
    v = [int.from_bytes(rng.bytes(8 * cf.L + 8), "little") % cf.q for _ in range(n)]
    return co.to_limbs(v, cf.L)


@pytest.mark.parametrize("key", ["p63", "jindo_zp"])
@pytest.mark.parametrize("rank,N", [(64, 16), (64, 24), (64, 64), (64, 100), (32, 1), (32, 0)])
def test_quorem_identity(fields, key, rank, N):
    q = fields[key]
    cf = co.CField(q)
    rng = np.random.default_rng(rank + N)
    p = _rand(cf, rank, rng)
    quo, rem = cf.quorem_vanishing(p, N)
    if N == 0:  # X^0 - 1 = 0: the reference's loop moves every coefficient to the quotient
        assert (quo == p).all() and (rem == 0).all()
        return
    P, Q, R = co.from_limbs(p), co.from_limbs(quo), co.from_limbs(rem)
    prod = [0] * (rank + max(N, 0))  # quo * (X^N - 1), quo has degree < rank - N
    for i, c in enumerate(Q):
        prod[i + N] += c
        prod[i] -= c
    want = [(prod[i] + R[i]) % q for i in range(rank)]
    assert want == [x % q for x in P]
    assert all(x == 0 for x in prod[rank:]) or all(c == 0 for c in Q[max(rank - N, 0):])
    if N > 0:
        assert all(r == 0 for r in R[N:])


@pytest.mark.parametrize("key", ["p63", "jindo_zp"])
@pytest.mark.parametrize("idx", [1, 3, 5, 127, -1, -3, 2 * 64 + 5])
def test_aut_is_ring_map_and_commutes_with_ntt(fields, key, idx):
    q = fields[key]
    cf = co.CField(q)
    N = 64
    rng = np.random.default_rng(idx % 1000)
    p = _rand(cf, N, rng)
    a = cf.aut(p, idx, False)
    tw, _, _ = cf.tables(N)
    assert (cf.ntt_fwd(a[None], tw)[0] == cf.aut(cf.ntt_fwd(p[None], tw)[0], idx, True)).all()
    for i in (0, 1, 7, N - 1):  # monomial X^i -> +-X^(i idx mod N)
        m = np.zeros_like(p)
        m[i] = p[i]
        got = co.from_limbs(cf.aut(m, idx, False))
        j = (i * idx) % (2 * N)
        want = [0] * N
        v = co.from_limbs(p[i:i + 1])[0]
        want[j % N] = v if j < N else (q - v) % q
        assert got == want


@pytest.mark.parametrize("key", ["p63", "jindo_zp"])
@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 300])
def test_evaluate_is_sum_of_powers(fields, key, n):
    q = fields[key]
    cf = co.CField(q)
    rng = np.random.default_rng(n)
    p = _rand(cf, max(n, 1), rng)[:n]
    x = _rand(cf, 1, rng)
    R = 1 << (64 * cf.L)
    rinv = pow(R, -1, q)
    xv = co.from_limbs(x)[0] * rinv % q
    want = sum(c * rinv % q * pow(xv, i, q) for i, c in enumerate(co.from_limbs(p) if n else [])) % q
    got = co.from_limbs(cf.evaluate(p if n else np.zeros((0, cf.L), np.uint64), x)[None])[0] * rinv % q
    assert got == want


@pytest.mark.parametrize("key", ["p63", "bfv_zp", "jindo_zp"])
@pytest.mark.parametrize("qbig", [2, 3, 2**61 - 1, 2**64, 3 * 2**100 + 7, 2**300 - 2**17, 2**511 - 1])
def test_mod_switch_is_round_half_down(fields, key, qbig):
    from fractions import Fraction
    import math

    import pyref
    q = fields[key]
    rng = np.random.default_rng(qbig % 1000)
    ps = [0, 1, -1, qbig - 1, -(qbig - 1), qbig >> 1, -(qbig >> 1), (qbig + 1) >> 1, -((qbig + 1) >> 1)]
    ps += [int.from_bytes(rng.bytes(72), "little") % qbig - (qbig >> 1) for _ in range(40)]
    if qbig % 2 == 0:  # exact ties p q = (k + 1/2) qBig, when q is odd
        ps += [(qbig // 2) * pow(q, -1, qbig) % qbig] if math.gcd(q, qbig) == 1 else []
    got = pyref.mod_switch(ps, qbig, q)
    want = [math.ceil(Fraction(p * q, qbig) - Fraction(1, 2)) % q for p in ps]
    assert got == want
