"""GPU parity of the Jindo commit over the zp package's other fields (the Buckler fields that
buckler/compile.go:178 hands to jindo.NewParameters[E]): p63 (exp 4, 1 limb, 64 slots), zp110
(exp 8, 2 limbs), zp220 (exp 16, 4 limbs), zp440 (exp 32, 7 limbs, one 59.x-bit ring prime, above
prep256's lazy-butterfly bound 2^64/36) and zp880 (exp 64, 14 limbs, 4 slots, one 58-bit ring
prime, below it), at targetN 2^10 and, for zp440 / zp880, 2^14.  Shapes:
tests/golden/jindo_params.json (restated NewParameters;
test_oracle_jindo.py pins the C oracle against the big-int restatement on the same shapes).

Per shape: the CRS commit key; Commit with injected randomness, full and ragged v, every output of
prover.go:45-202 bit for bit; the device samplers' draws against the C oracle's
(rg_jindo_sample_dev, uniform.go / gaussian_twin_cdt.go / the COSAC and rounded samplers); the
sampled commit == the injected commit on those draws == the oracle's commit; Evaluate's device
loops (prover.go:228-314) on those openings."""
import json
import os

import numpy as np
import pytest

import coracle as co
import pyref
from ringo import jindo
from tests.jindo_util import make_randomness, make_v

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
PARAMS = json.load(open(os.path.join(HERE, "golden", "jindo_params.json")))
SD_KEYS = jindo.STDDEV_KEYS
# targetN 2^14 adds larger grids: zp880's 60-bit ring prime (the generic MAC, prime >= 2^60) and
# zp440's two 31-bit primes
NAMES = ["p63_t10_b2", "zp110_t10_b1", "zp220_t10_b1", "zp440_t10_b2", "zp880_t10_b1", "zp440_t14_b1", "zp880_t14_b1"]


def _setup(name):
    P = PARAMS[name]
    q = int(P["field_q_hex"], 16)
    return P, q, jindo.Parameters.from_dict(P, q)


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to("cuda")


def _h(t):
    return t.cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("name", NAMES)
def test_commit_key_and_injected_commit(name):
    P, q, params = _setup(name)
    prv = jindo.NewProver(params, b"Jindo!")
    ck = prv.commit_key()
    want_ck = pyref.commit_key(pyref.JindoParams(q, P["target_n"], P["batch"]), b"Jindo!")
    for g, w in zip(ck, want_ck):
        assert (g == np.array(w, dtype=np.uint64)).all()
    cj = co.CJindo(P, q)
    for nv in (P["rank"], 333, 1):
        v = make_v(q, nv, seed=nv + 5)
        rnd = make_randomness(P, q, seed=nv + 11)
        com, op = prv.Commit(v, jindo.Randomness(**rnd))
        want = cj.commit(ck[0], ck[1], ck[2], v, rnd["last_row"], rnd["mask"], rnd["enc_noise"], rnd["mlwe_noise"])
        assert (op.Encode == want["enc"]).all(), (name, nv, "Encode")
        assert (op.MLWE == want["mlwe"]).all(), (name, nv, "MLWE")
        assert (op.InCommit == want["incom"]).all(), (name, nv, "InCommit")
        assert (com.Value == want["com"]).all(), (name, nv, "Commitment")


@pytest.mark.parametrize("name", NAMES)
def test_sampled_commit_and_evaluate(name):
    import torch
    P, q, params = _setup(name)
    prv = jindo.NewProver(params, b"Jindo!")
    ck = prv.commit_key()
    B, first = 3, 17
    nv = P["rank"] - 7
    v = np.stack([make_v(q, nv, seed=61 + b) for b in range(B)])
    seeds = jindo.Seeds.derive(b"fields-" + name.encode())
    sh = params.shapes(B)
    z = lambda k: torch.zeros(sh[k], dtype=torch.int64, device="cuda")
    r = {k: z(k) for k in ("last_row", "mask", "enc_noise", "mlwe_noise")}
    prv.sample_dev(B, _t(v), nv, seeds, first, r["last_row"], r["mask"], r["enc_noise"], r["mlwe_noise"])
    a = {k: z(k) for k in ("incom", "enc", "mlwe_out", "com")}
    prv.commit_sampled_dev(B, _t(v), nv, seeds, first, a["incom"], a["enc"], a["mlwe_out"], a["com"])
    b_ = {k: z(k) for k in ("incom", "enc", "mlwe_out", "com")}
    prv.commit_dev(B, _t(v), nv, r["last_row"], r["mask"], r["enc_noise"], r["mlwe_noise"], b_["incom"], b_["enc"],
                   b_["mlwe_out"], b_["com"])
    torch.cuda.synchronize()
    cj = co.CJindo(P, q)
    want = cj.sample([P[k] for k in SD_KEYS], pyref.delta_inv(P["base"], P["exp"]), seeds.raw(), first, v)
    assert (_h(r["last_row"]) == want["last_row"]).all()
    assert (_h(r["mask"]) == want["mask"]).all()
    assert (r["mlwe_noise"].cpu().numpy() == want["mlwe_noise"]).all()
    assert (r["enc_noise"].cpu().numpy() == want["enc_noise"]).all()
    for k in a:
        assert torch.equal(a[k], b_[k]), k
    for b in range(B):
        w = cj.commit(ck[0], ck[1], ck[2], v[b], want["last_row"][b], want["mask"][b], want["enc_noise"][b],
                      want["mlwe_noise"][b])
        assert (_h(a["com"][b]) == w["com"]).all(), b
        assert (_h(a["enc"][b]) == w["enc"]).all(), b
        assert (_h(a["mlwe_out"][b]) == w["mlwe"]).all(), b
        assert (_h(a["incom"][b]) == w["incom"]).all(), b
    # Evaluate's device loops on these openings, injected challenges
    rng = np.random.default_rng(5)

    def res(primes, shape):
        out = np.zeros(shape, np.uint64)
        for l, qq in enumerate(primes):
            out[..., l, :] = rng.integers(0, qq, size=out[..., l, :].shape, dtype=np.uint64)
        return out

    # (params.batch openings; with batch 1 the openBatch is open[0], no challenge: prover.go:267-269)
    E = P["batch"]
    op = {k: a[k][:E].contiguous() for k in ("incom", "enc", "mlwe_out")}
    es = prv.eval_shapes()
    bq, bo = res(P["q"], (E, len(P["q"]), P["d"])), res(P["qo"], (E, len(P["qo"]), P["d"]))
    left = res(P["q"], (P["rows"], len(P["q"]), P["d"]))
    chals = res(P["q"], (P["cols"], len(P["q"]), P["d"]))
    out = {k: torch.zeros(es[k], dtype=torch.int64, device="cuda") for k in es}
    single = E == 1
    prv.eval_batch_dev(E, op["incom"], op["enc"], op["mlwe_out"], None if single else _t(bq),
                       None if single else _t(bo), out["ob_incom"], out["ob_enc"], out["ob_mlwe"])
    prv.eval_partial_dev(out["ob_enc"], _t(left), out["partial"])
    prv.eval_respond_dev(out["ob_enc"], out["ob_mlwe"], _t(chals), out["pf_enc"], out["pf_mlwe"])
    torch.cuda.synchronize()
    ob = cj.eval_batch(_h(op["incom"]), _h(op["enc"]), _h(op["mlwe_out"]), bq, bo)
    for k in ("ob_incom", "ob_enc", "ob_mlwe"):
        assert (_h(out[k]) == ob[k]).all(), k
    assert (_h(out["partial"]) == cj.eval_partial(ob["ob_enc"], left)).all()
    pe, pm = cj.eval_respond(ob["ob_enc"], ob["ob_mlwe"], chals)
    assert (_h(out["pf_enc"]) == pe).all()
    assert (_h(out["pf_mlwe"]) == pm).all()
