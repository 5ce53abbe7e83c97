"""CPU: pin the oracle.

  * field constants derived by both restatements == the reference's generated constants
    (tests/golden/fields.json <- jindo/internal/zp/element.go:47-72,781-789 and siblings);
  * Montgomery CIOS word-level restatement == value-level product on the reference's static
    edge values (element_test.go:315-358) and random values, every field;
  * C oracle == big-int restatement for field ops, tables, transforms (all fields);
  * negacyclic NTT satisfies the evaluation identity NTT(a)[i] = a(psi^(2 brv(i) + 1)) and the
    cyclic one NTT(a)[i] = a(w^brv(i)) -- independent of the butterfly loop structure;
  * NTT products == negacyclic / cyclic convolutions;
  * regression digests (tests/golden/ntt_golden.json);
  * Jindo: C oracle commit == big-int commit (2- and 3-prime rings), DecodeTo(Encode) == v.
"""
import hashlib
import json
import os
import random

import numpy as np
import pytest

import coracle as co
import pyref

HERE = os.path.dirname(os.path.abspath(__file__))
FIELDS = json.load(open(os.path.join(HERE, "golden", "fields.json")))


def _q(name):
    return int(FIELDS[name]["q_hex"], 16)


def static_values(F):
    """element_test.go:315-358 staticTestValues, as Montgomery-limb values < q."""
    q, L = F.q, F.L
    ql = F.limbs(q)
    vals = [0, F.to_mont(1), F.rSquare, F.to_mont(q - 1), F.to_mont(2)]
    a = list(ql)
    a[0] -= 1
    vals.append(F.from_limbs(a))
    vals += [0, 0, 1, 1 << 64 if L > 1 else 1, 2, 2 << 64 if L > 1 else 2]
    a = list(ql)
    a[L - 1] -= 1
    vals.append(F.from_limbs(a))
    a[0] += 1
    vals.append(F.from_limbs(a))
    a = list(ql)
    a[L - 1] = 0
    vals.append(F.from_limbs(a))
    return [v for v in vals if v < q]


@pytest.mark.parametrize("name", sorted(FIELDS))
def test_field_constants_match_reference(name):
    f = FIELDS[name]
    q = int(f["q_hex"], 16)
    F = pyref.Field(q)
    assert F.L == f["limbs"]
    assert F.qInvNeg == int(f["qInvNeg"])
    assert F.limbs(F.rSquare) == [int(x) for x in f["rSquare_le"]]
    cf = co.CField(q)
    qinv, r2, one = cf.consts()
    assert qinv == int(f["qInvNeg"]) and r2 == F.rSquare and one == F.R % q


@pytest.mark.parametrize("name", sorted(FIELDS))
def test_field_ops_c_vs_bigint(name):
    q = _q(name)
    F = pyref.Field(q)
    cf = co.CField(q)
    rng = random.Random(99)
    vals = static_values(F) + [rng.randrange(q) for _ in range(64)]
    for x in vals:
        assert cf.neg(x) == F.neg(x)
        for y in vals[::3]:
            m = F.mul(x, y)
            assert F.mont_cios(x, y) == m
            assert cf.mul(x, y) == m
            assert cf.add(x, y) == F.add(x, y)
            assert cf.sub(x, y) == F.sub(x, y)


@pytest.mark.parametrize("name", sorted(FIELDS))
@pytest.mark.parametrize("cyclic", [False, True])
def test_transforms_c_vs_bigint_and_identity(name, cyclic):
    q = _q(name)
    F = pyref.Field(q)
    cf = co.CField(q)
    rng = random.Random(5)
    for logn in [3, 5, 7]:
        N = 1 << logn
        if (q - 1) % (2 * N):
            continue
        tables = pyref.cyclic_tables if cyclic else pyref.cyclotomic_tables
        tw, twi, ninv, root = tables(F, N)
        ctw, ctwi, cninv = cf.tables(N, cyclic=cyclic)
        assert co.from_limbs(ctw) == tw and co.from_limbs(ctwi) == twi
        a = [rng.randrange(q) for _ in range(N)]
        y = pyref.ntt_fwd(F, a, tw)
        assert co.from_limbs(cf.ntt_fwd(co.to_limbs(a, F.L)[None], ctw)[0]) == y
        assert pyref.ntt_inv(F, y, twi, ninv) == a
        # evaluation identity on plain values
        plain = [F.from_mont(x) for x in a]
        for i in range(N):
            e = (2 * pyref.bit_reverse(i, logn) + 1) if not cyclic else pyref.bit_reverse(i, logn)
            pt = pow(root, e, q)
            want = sum(c * pow(pt, k, q) for k, c in enumerate(plain)) % q
            assert F.from_mont(y[i]) == want


@pytest.mark.parametrize("cyclic", [False, True])
def test_ntt_product_is_convolution(cyclic):
    q = _q("zp110")
    F = pyref.Field(q)
    N = 16
    tw, twi, ninv, _ = (pyref.cyclic_tables if cyclic else pyref.cyclotomic_tables)(F, N)
    rng = random.Random(1)
    a = [rng.randrange(q) for _ in range(N)]
    b = [rng.randrange(q) for _ in range(N)]
    prod = pyref.ntt_inv(F, pyref.vec_mul(F, pyref.ntt_fwd(F, a, tw), pyref.ntt_fwd(F, b, tw)), twi, ninv)
    pa, pb = [F.from_mont(x) for x in a], [F.from_mont(x) for x in b]
    conv = [0] * N
    for i in range(N):
        for j in range(N):
            k = i + j
            s = 1
            if k >= N:
                k -= N
                s = 1 if cyclic else -1
            conv[k] = (conv[k] + s * pa[i] * pb[j]) % q
    assert [F.from_mont(x) for x in prod] == conv


def test_ntt_regression_digests():
    G = json.load(open(os.path.join(HERE, "golden", "ntt_golden.json")))
    for key, g in G.items():
        name, logn, kind = key.split("/")
        q = _q(name)
        cf = co.CField(q)
        N = 1 << int(logn)
        tw, twi, ninv = cf.tables(N, cyclic=(kind == "cyclic"))
        rng = np.random.default_rng(g["seed"])
        vals = [int.from_bytes(rng.bytes(8 * cf.L), "little") % q for _ in range(N)]
        a = co.to_limbs(vals, cf.L)[None]
        d = lambda x: hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()
        assert d(tw) == g["tw"] and d(twi) == g["twinv"], key
        assert d(cf.ntt_fwd(a, tw)) == g["fwd"] and d(cf.ntt_inv(a, twi, ninv)) == g["inv"], key


def test_unsupported_rank_rejected():
    cf = co.CField(97)  # 97 - 1 = 2^5 * 3 (ntt.go:35-37,162-164 require 2N | q-1)
    with pytest.raises(ValueError, match="NTT not supported"):
        cf.tables(32)
    with pytest.raises(ValueError, match="NTT not supported"):
        cf.tables(64, cyclic=True)
    with pytest.raises(ValueError, match="power of two"):
        cf.tables(12)
