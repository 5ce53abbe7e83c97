"""The Jindo protocol around Commit / Evaluate / Verify for tests (jindo_test.go:26-52): an
honest proof built by the C oracle (test infrastructure), with the Fiat-Shamir challenges drawn
as random 16-byte strings and encoded by encodeChallengeTo (utils.go:20-46), x random, the
prover's left encodes / rightVec / evaluations (utils.go:63-82, poly.go:64-76) computed on the
host, and the randomness drawn by the oracle's restatement of the device samplers at the
reference's widths."""
import numpy as np

import coracle as co
import pyref
from tests.jindo_util import make_v

SD_KEYS = ("ecd_sd", "ecd_blind_sd", "mask_sd", "mask_blind_sd", "mlwe_sd", "mask_mlwe_sd")


def random_ck(P, seed):
    """A commit key of uniform residues (completeness does not depend on how it was derived)."""
    rng = np.random.default_rng(seed)
    q, qo, d = P["q"], P["qo"], P["d"]

    def res(primes, shape):
        out = np.zeros(shape + (len(primes), d), np.uint64)
        for l, p in enumerate(primes):
            out[..., l, :] = rng.integers(0, p, size=out[..., l, :].shape, dtype=np.uint64)
        return out

    return (res(q, (P["in_msis"], P["rows"])), res(q, (P["in_msis"], P["mlwe"])),
            res(qo, (P["out_msis"], P["in_com_dcmp_len"])))


def mont(F, x):
    """Montgomery form of the integer x (x R mod q) via CField: x * R^2 * R^-1."""
    _, r2, _ = F.consts()
    return F.mul(x % F.q, r2)


def left_right(P, F, x):
    """leftVec / rightVec (utils.go:63-82) of the Montgomery element x, as Montgomery ints."""
    one = mont(F, 1)
    cs = P["cols"] * P["slots"]
    skip = one
    for _ in range(cs):
        skip = F.mul(skip, x)
    left = [one]
    for _ in range(1, P["rows"]):
        left.append(F.mul(left[-1], skip))
    left[-1] = x
    right = [one]
    for _ in range(1, cs):
        right.append(F.mul(right[-1], x))
    return left, right


def honest_proof(P, fq, ck, seed, nv=None, B=None):
    """Commit B = params.batch vectors, Evaluate at a random x, return every Verify input
    (include/ringo.h rg_jindo_verify_dev layouts) plus the openings."""
    cj = co.CJindo(P, fq)
    F = co.CField(fq)
    L = F.L
    B = B or P["batch"]
    nv = nv or P["rank"]
    rng = np.random.default_rng(seed)
    v = np.stack([make_v(fq, nv, seed=seed * 100 + b) for b in range(B)])
    seeds = rng.bytes(192)
    rnd = cj.sample([P[k] for k in SD_KEYS], pyref.delta_inv(P["base"], P["exp"]), seeds, 0, v)
    opens = [cj.commit(ck[0], ck[1], ck[2], v[b], rnd["last_row"][b], rnd["mask"][b], rnd["enc_noise"][b],
                       rnd["mlwe_noise"][b]) for b in range(B)]
    com = np.stack([o["com"] for o in opens])
    incom = np.stack([o["incom"] for o in opens])
    enc = np.stack([o["enc"] for o in opens])
    mlwe = np.stack([o["mlwe"] for o in opens])
    x = mont(F, int.from_bytes(rng.bytes(40), "little"))
    bbytes = [rng.bytes(16) for _ in range(B)]
    if B > 1:
        bq = np.stack([cj.encode_challenge(0, b) for b in bbytes])
        bo = np.stack([cj.encode_challenge(1, b) for b in bbytes])
    else:
        bq = bo = None
    ob = cj.eval_batch(incom, enc, mlwe, bq if bq is not None else np.zeros((1, len(P["q"]), P["d"]), np.uint64),
                       bo if bo is not None else np.zeros((1, len(P["qo"]), P["d"]), np.uint64))
    left_e, right_e = left_right(P, F, x)
    left = np.stack([cj.encode(co.to_limbs([e], L)) for e in left_e])
    partial = cj.eval_partial(ob["ob_enc"], left)
    chals = np.stack([cj.encode_challenge(0, rng.bytes(16)) for _ in range(P["cols"])])
    pe, pm = cj.eval_respond(ob["ob_enc"], ob["ob_mlwe"], chals)
    xl = co.to_limbs([x], L)[0]
    y = np.stack([F.evaluate(v[b], xl) for b in range(B)])
    return dict(batch=B, com=com, bq=bq, bo=bo, chals=chals, left=left, right=co.to_limbs(right_e, L), y=y,
                pf_incom=ob["ob_incom"], pf_partial=partial, pf_enc=pe, pf_mlwe=pm,
                opens=dict(incom=incom, enc=enc, mlwe=mlwe), v=v, x=x)


VERIFY_KEYS = ("com", "bq", "bo", "chals", "left", "right", "y", "pf_incom", "pf_partial", "pf_enc", "pf_mlwe")


def oracle_verify(P, fq, ck, pr):
    cj = co.CJindo(P, fq)
    return cj.verify(ck, pr["batch"], *[pr[k] for k in VERIFY_KEYS], P["in_com_dcmp_two_nm"], P["res_two_nm"])
