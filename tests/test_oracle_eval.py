"""CPU: the C oracle's Prover.Evaluate core (oracle.c of_jindo_eval_*, restating
jindo/prover.go:228-314) pinned against a direct big-int evaluation of the reference's loops:
every product is MulCoeffsMontgomeryThenAdd, acc += a * b * 2^-64 mod q.  Shapes: the
jindo_test (targetN 2^10) parameter sets, batch 1 and batch 8."""
import json
import os

import numpy as np
import pytest

import coracle as co

HERE = os.path.dirname(os.path.abspath(__file__))
PARAMS = json.load(open(os.path.join(HERE, "golden", "jindo_params.json")))


def _rand_res(rng, primes, shape):
    """uniform residues per RNS limb: shape (..., nl, d)"""
    out = np.zeros(shape, np.uint64)
    for l, q in enumerate(primes):
        out[..., l, :] = rng.integers(0, q, size=out[..., l, :].shape, dtype=np.uint64)
    return out


def _mont_dot(a_terms, b_terms, primes):
    """sum_t a_t * b_t * 2^-64 mod q per limb, Python ints; a_terms/b_terms: lists of [nl][d]"""
    nl, d = a_terms[0].shape
    out = np.zeros((nl, d), np.uint64)
    for l, q in enumerate(primes):
        rinv = pow(2 ** 64, -1, q)
        for k in range(d):
            s = sum(int(a[l, k]) * int(b[l, k]) for a, b in zip(a_terms, b_terms))
            out[l, k] = s * rinv % q
    return out


@pytest.mark.parametrize("name", ["t10_b1", "t10_b8"])
def test_eval_core_matches_bigint(name):
    P = PARAMS[name]
    fq = int(P["field_q_hex"], 16)
    cj = co.CJindo(P, fq)
    sh = cj.eval_shapes()
    B = P["batch"]
    rng = np.random.default_rng(5)
    q, qo = P["q"], P["qo"]
    incom = _rand_res(rng, qo, (B,) + sh["ob_incom"])
    enc = _rand_res(rng, q, (B,) + sh["ob_enc"])
    mlwe = _rand_res(rng, q, (B,) + sh["ob_mlwe"])
    bq = _rand_res(rng, q, (B, len(q), P["d"]))
    bo = _rand_res(rng, qo, (B, len(qo), P["d"]))
    ob = cj.eval_batch(incom, enc, mlwe, bq, bo)
    if B == 1:
        assert (ob["ob_enc"] == enc[0]).all() and (ob["ob_incom"] == incom[0]).all()
    else:  # spot-check polynomials of every part (full big-int check is slow in Python)
        for j in (0, sh["ob_incom"][0] - 1):
            assert (ob["ob_incom"][j] == _mont_dot([incom[i, j] for i in range(B)], list(bo), qo)).all()
        for (c, r) in ((0, 0), (P["cols"], P["rows"] - 1)):
            assert (ob["ob_enc"][c, r] == _mont_dot([enc[i, c, r] for i in range(B)], list(bq), q)).all()
        assert (ob["ob_mlwe"][1, 2] == _mont_dot([mlwe[i, 1, 2] for i in range(B)], list(bq), q)).all()
    left = _rand_res(rng, q, (P["rows"], len(q), P["d"]))
    part = cj.eval_partial(ob["ob_enc"], left)
    for i in (0, P["cols"]):  # Partial[0] and PartialMask
        assert (part[i] == _mont_dot(list(left), list(ob["ob_enc"][i]), q)).all()
    chals = _rand_res(rng, q, (P["cols"], len(q), P["d"]))
    pe, pm = cj.eval_respond(ob["ob_enc"], ob["ob_mlwe"], chals)
    for i in (0, P["rows"] - 1):
        dot = _mont_dot(list(chals), [ob["ob_enc"][j, i] for j in range(P["cols"])], q)
        want = np.array([[(int(dot[l, k]) + int(ob["ob_enc"][P["cols"], i, l, k])) % q[l] for k in range(P["d"])]
                         for l in range(len(q))], dtype=np.uint64)
        assert (pe[i] == want).all()
    i = sh["pf_mlwe"][0] - 1
    dot = _mont_dot(list(chals), [ob["ob_mlwe"][j, i] for j in range(P["cols"])], q)
    want = np.array([[(int(dot[l, k]) + int(ob["ob_mlwe"][P["cols"], i, l, k])) % q[l] for k in range(P["d"])]
                     for l in range(len(q))], dtype=np.uint64)
    assert (pm[i] == want).all()
