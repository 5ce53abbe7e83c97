"""GPU: Verifier.Verify (rg_jindo_verify_dev, jindo/verifier.go:50-282) against the C oracle
(oracle.c of_jindo_verify) on the same proofs -- both norms' exact sums of squares, the four
checks and both sides of the evaluation check -- for honest and tampered proofs; then the
reference's TestJindo flow (jindo_test.go:26-52) entirely on the GPU: Commit (device samplers),
Evaluate's device work, Verify == true, and false once a proof word changes."""
import json
import os

import numpy as np
import pytest

import coracle as co
from ringo import jindo
from tests.jindo_proto import VERIFY_KEYS, honest_proof, left_right, mont, oracle_verify

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
PARAMS = json.load(open(os.path.join(HERE, "golden", "jindo_params.json")))


def _t(a):
    import torch
    return None if a is None else torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to("cuda")


def _h(t):
    return t.cpu().numpy().view(np.uint64)


_CACHE = {}


def _setup(name):
    if name not in _CACHE:
        P = PARAMS[name]
        fq = int(P["field_q_hex"], 16)
        params = jindo.Parameters.from_dict(P, fq)
        vrf = jindo.Verifier(params, crs=b"Jindo!")
        ck = vrf._p.commit_key()
        _CACHE[name] = (P, fq, params, vrf, ck, honest_proof(P, fq, ck, seed=23))
    return _CACHE[name]


def _gpu_verify(vrf, pr):
    return vrf.verify_dev(pr["batch"], *[_t(pr[k]) for k in VERIFY_KEYS])


def _same(r, want):
    assert r.outer_norm_sq == want["outer_sq"]
    assert r.inner_norm_sq == want["inner_sq"]
    assert [r.outer_ok, r.inner_ok, r.consistency_ok, r.eval_ok] == want["flags"]
    assert (r.eval_lhs == want["eval_lhs"]).all() and (r.eval_rhs == want["eval_rhs"]).all()
    assert r.ok == want["ok"]


# the zp package's other fields as Jindo fields (test_gpu_jindo_fields.py)
FIELDS = ["p63_t10_b2", "zp110_t10_b1", "zp220_t10_b1", "zp440_t10_b2", "zp880_t10_b1"]


@pytest.mark.parametrize("name", ["t10_b1", "t10_b8", "t14_b1", "mult_t8193_b12"] + FIELDS)
def test_verify_matches_oracle(name):
    P, fq, params, vrf, ck, pr = _setup(name)
    want = oracle_verify(P, fq, ck, pr)
    assert want["ok"], want["flags"]  # the honest proof verifies (TestJindo)
    _same(_gpu_verify(vrf, pr), want)


@pytest.mark.parametrize("name", ["t10_b1", "t10_b8", "mult_t8193_b12", "p63_t10_b2", "zp880_t10_b1"])
@pytest.mark.parametrize("what", ["pf_enc", "pf_incom", "y", "pf_partial", "pf_mlwe", "com"])
def test_tampered_verify_matches_oracle(name, what):
    P, fq, params, vrf, ck, pr = _setup(name)
    bad = dict(pr)
    bad[what] = pr[what].copy()
    flat = bad[what].reshape(-1)
    i = min(5, flat.size - 1)
    flat[i] = (int(flat[i]) + 12345) % (1 << 40)
    want = oracle_verify(P, fq, ck, bad)
    assert not want["ok"], (name, what)
    _same(_gpu_verify(vrf, bad), want)


@pytest.mark.parametrize("name", ["t10_b1", "t10_b8", "t14_b1", "mult_t8193_b12"] + FIELDS)
def test_jindo_flow_on_gpu(name):
    """TestJindo (jindo_test.go:26-52) on the device: Commit with the device samplers, Evaluate's
    MACs on the device (challenges from encodeChallengeTo of random bytes; leftVec / rightVec /
    Poly.Evaluate by the caller), Verify on the device."""
    import torch
    P, fq, params, vrf, ck, _ = _setup(name)
    prv = jindo.Prover(params, ck=ck)
    cj = co.CJindo(P, fq)
    F = co.CField(fq)
    B, nv, L = P["batch"], P["rank"], params.L
    rng = np.random.default_rng(41)
    from tests.jindo_util import make_v
    v = np.stack([make_v(fq, nv, seed=500 + b) for b in range(B)])
    sh = params.shapes(B)
    o = {k: torch.zeros(sh[k], dtype=torch.int64, device="cuda") for k in ("incom", "enc", "mlwe_out", "com")}
    prv.commit_sampled_dev(B, _t(v), nv, jindo.Seeds.derive(b"flow-" + name.encode()), 0, o["incom"], o["enc"],
                           o["mlwe_out"], o["com"])
    x = mont(F, int.from_bytes(rng.bytes(40), "little"))
    es = prv.eval_shapes()
    e = {k: torch.zeros(es[k], dtype=torch.int64, device="cuda") for k in es}
    if B > 1:
        bb = [rng.bytes(16) for _ in range(B)]
        bq = np.stack([cj.encode_challenge(0, b) for b in bb])
        bo = np.stack([cj.encode_challenge(1, b) for b in bb])
    else:
        bq = bo = None
    prv.eval_batch_dev(B, o["incom"], o["enc"], o["mlwe_out"], _t(bq), _t(bo), e["ob_incom"], e["ob_enc"], e["ob_mlwe"])
    left_e, right_e = left_right(P, F, x)
    left = np.stack([cj.encode(co.to_limbs([a], L)) for a in left_e])
    prv.eval_partial_dev(e["ob_enc"], _t(left), e["partial"])
    chals = np.stack([cj.encode_challenge(0, rng.bytes(16)) for _ in range(P["cols"])])
    prv.eval_respond_dev(e["ob_enc"], e["ob_mlwe"], _t(chals), e["pf_enc"], e["pf_mlwe"])
    xl = co.to_limbs([x], L)[0]
    y = np.stack([F.evaluate(v[b], xl) for b in range(B)])
    torch.cuda.synchronize()
    args = dict(com=o["com"], bq=_t(bq), bo=_t(bo), chals=_t(chals), left=_t(left), right=_t(co.to_limbs(right_e, L)),
                y=_t(y), pf_incom=e["ob_incom"], pf_partial=e["partial"], pf_enc=e["pf_enc"], pf_mlwe=e["pf_mlwe"])
    r = vrf.verify_dev(B, *[args[k] for k in VERIFY_KEYS])
    assert r.ok and r.outer_ok and r.inner_ok and r.consistency_ok and r.eval_ok
    # the same proof, checked by the oracle, is accepted with the same norms
    host = {k: (None if a is None else _h(a)) for k, a in args.items()}
    want = co.CJindo(P, fq).verify(ck, B, *[host[k] for k in VERIFY_KEYS], P["in_com_dcmp_two_nm"], P["res_two_nm"])
    assert want["ok"] and want["outer_sq"] == r.outer_norm_sq and want["inner_sq"] == r.inner_norm_sq
    # a changed response word is rejected
    args["pf_enc"] = e["pf_enc"].clone()
    args["pf_enc"].view(-1)[7] += 1
    assert not vrf.verify_dev(B, *[args[k] for k in VERIFY_KEYS]).ok
