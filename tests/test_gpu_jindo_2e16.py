"""GPU parity at the configs[4] shape (NewParameters(2^16, 4096): 2 x 58-bit ringQ primes, 2 x
54-bit ringQOut primes, rows 513, cols 8, inMSIS 16, J = 16, logOutCut 74) -- the shape the
bench's jindo_commit_2e16 / jindo_evaluate_2e16 lines run -- plus the Ajtai-core entry point
(rg_jindo_commit_core, prover.go:144-202), the MAC's extreme inputs, per-stream scratch and the
device-resident commit key.  Oracle: oracle/oracle.c (CJindo), bit-exact."""
import json
import os

import numpy as np
import pytest

import coracle as co
from ringo import jindo
from tests.jindo_util import make_randomness, make_v

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
PARAMS = json.load(open(os.path.join(HERE, "golden", "jindo_params.json")))
_CACHE = {}


def _prover(name):
    if name not in _CACHE:
        P = PARAMS[name]
        q = int(P["field_q_hex"], 16)
        params = jindo.Parameters.from_dict(P, q)
        prv = jindo.NewProver(params, b"Jindo!")
        _CACHE[name] = (P, q, params, prv, prv.commit_key())
    return _CACHE[name]


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to("cuda")


def _h(t):
    return t.cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("nv", [65536, 40000, 1])
def test_commit_2e16_matches_oracle(nv):
    P, q, params, prv, ck = _prover("t16_b4096")
    v = make_v(q, nv, seed=nv + 1)
    rnd = make_randomness(P, q, seed=nv + 2, param_sd=True)
    com, op = prv.Commit(v, jindo.Randomness(**rnd))
    want = co.CJindo(P, q).commit(ck[0], ck[1], ck[2], v, rnd["last_row"], rnd["mask"], rnd["enc_noise"],
                                  rnd["mlwe_noise"])
    assert (op.Encode == want["enc"]).all()
    assert (op.MLWE == want["mlwe"]).all()
    assert (op.InCommit == want["incom"]).all()
    assert (com.Value == want["com"]).all()


def test_commit_dev_batch_2e16_matches_oracle():
    """Three commits of one batched rg_jindo_commit_dev call (the bench's path) at configs[4]."""
    import torch
    P, q, params, prv, ck = _prover("t16_b4096")
    B, nv = 3, 65536
    sh = params.shapes(B)
    vs = np.stack([make_v(q, nv, seed=300 + b) for b in range(B)])
    rnd = make_randomness(P, q, seed=31, batch=B, param_sd=True)
    outs = {k: torch.zeros(sh[k], dtype=torch.int64, device="cuda") for k in ["incom", "enc", "mlwe_out", "com"]}
    prv.commit_dev(B, _t(vs), nv, _t(rnd["last_row"]), _t(rnd["mask"]), _t(rnd["enc_noise"]), _t(rnd["mlwe_noise"]),
                   outs["incom"], outs["enc"], outs["mlwe_out"], outs["com"])
    torch.cuda.synchronize()
    cj = co.CJindo(P, q)
    for b in range(B):
        w = cj.commit(ck[0], ck[1], ck[2], vs[b], rnd["last_row"][b], rnd["mask"][b], rnd["enc_noise"][b],
                      rnd["mlwe_noise"][b])
        assert (_h(outs["enc"][b]) == w["enc"]).all(), b
        assert (_h(outs["mlwe_out"][b]) == w["mlwe"]).all(), b
        assert (_h(outs["incom"][b]) == w["incom"]).all(), b
        assert (_h(outs["com"][b]) == w["com"]).all(), b


def _residues(primes, shape, rng, fill=None):
    out = np.zeros(shape, np.uint64)
    for l, qq in enumerate(primes):
        if fill == "max":
            out[..., l, :] = qq - 1
        else:
            out[..., l, :] = rng.integers(0, qq, size=out[..., l, :].shape, dtype=np.uint64)
    return out


@pytest.mark.parametrize("name", ["t10_b1", "t14_b1", "mult_t8193_b12", "t16_b4096"])
def test_commit_core_matches_oracle(name):
    """rg_jindo_commit_core on uniform NTT-domain openings vs of_jindo_commit_core."""
    P, q, params, prv, ck = _prover(name)
    rng = np.random.default_rng(5)
    sh = params.shapes()
    enc = _residues(P["q"], sh["enc"], rng)
    mlwe = _residues(P["q"], sh["mlwe_out"], rng)
    com, incom = prv.commit_core(enc, mlwe)
    w = co.CJindo(P, q).commit_core(ck[0], ck[1], ck[2], enc, mlwe)
    assert (incom == w["incom"]).all()
    assert (com == w["com"]).all()


@pytest.mark.parametrize("name", ["t16_b4096", "t10_b8"])
def test_mac_extreme_inputs(name):
    """Every commit-key and opening word q - 1: the MFMA MAC's digit diagonals and signed 128-bit
    fold reach their largest magnitudes (configs[4]: 545 terms x 2^58 x 2^58 = 2^125.1, the bound
    mac_mfma_nb admits) and the exact sums their maximum; the InCommit words fed to the outer MAC
    are whatever rounding gives.  A second prover holds an all-(q-1) key."""
    P, q, params, _, _ = _prover(name)
    sh, cks = params.shapes(), params.ck_shapes()
    rng = np.random.default_rng(0)
    ck = (_residues(P["q"], cks["ck_in"], rng, "max"), _residues(P["q"], cks["ck_mlwe"], rng, "max"),
          _residues(P["qo"], cks["ck_out"], rng, "max"))
    prv = jindo.Prover(params, ck=ck)
    enc = _residues(P["q"], sh["enc"], rng, "max")
    mlwe = _residues(P["q"], sh["mlwe_out"], rng, "max")
    com, incom = prv.commit_core(enc, mlwe)
    w = co.CJindo(P, q).commit_core(ck[0], ck[1], ck[2], enc, mlwe)
    assert (incom == w["incom"]).all()
    assert (com == w["com"]).all()


def test_commit_core_dev_batch_equals_commit():
    """commit_core_dev over the Openings of commit_dev reproduces InCommit and the Commitment."""
    import torch
    P, q, params, prv, ck = _prover("t10_b8")
    B, nv = 3, 700
    sh = params.shapes(B)
    vs = np.stack([make_v(q, nv, seed=40 + b) for b in range(B)])
    rnd = make_randomness(P, q, seed=41, batch=B)
    o = {k: torch.zeros(sh[k], dtype=torch.int64, device="cuda") for k in ["incom", "enc", "mlwe_out", "com"]}
    prv.commit_dev(B, _t(vs), nv, _t(rnd["last_row"]), _t(rnd["mask"]), _t(rnd["enc_noise"]), _t(rnd["mlwe_noise"]),
                   o["incom"], o["enc"], o["mlwe_out"], o["com"])
    inc2, com2 = torch.zeros_like(o["incom"]), torch.zeros_like(o["com"])
    prv.commit_core_dev(B, o["enc"], o["mlwe_out"], inc2, com2)
    torch.cuda.synchronize()
    assert torch.equal(inc2, o["incom"]) and torch.equal(com2, o["com"])


def test_two_streams_one_handle():
    """One handle, two streams, both queued before either finishes: per-stream scratch keeps the
    commits apart (the handle's scratch used to be shared)."""
    import torch
    P, q, params, prv, ck = _prover("t14_b1")
    B, nv = 4, 16384
    sh = params.shapes(B)
    ins, outs = [], []
    for s in range(2):
        vs = np.stack([make_v(q, nv, seed=500 + 10 * s + b) for b in range(B)])
        rnd = make_randomness(P, q, seed=60 + s, batch=B)
        ins.append((vs, rnd))
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    dev_in = [(_t(vs), _t(r["last_row"]), _t(r["mask"]), _t(r["enc_noise"]), _t(r["mlwe_noise"])) for vs, r in ins]
    torch.cuda.synchronize()
    for s in range(2):
        o = {k: torch.zeros(sh[k], dtype=torch.int64, device="cuda") for k in ["incom", "enc", "mlwe_out", "com"]}
        for _ in range(3):  # keep both streams busy at once
            prv.commit_dev(B, *dev_in[s][:1], nv, *dev_in[s][1:], o["incom"], o["enc"], o["mlwe_out"], o["com"],
                           streams[s])
        outs.append(o)
    torch.cuda.synchronize()
    cj = co.CJindo(P, q)
    for s in range(2):
        vs, r = ins[s]
        for b in (0, B - 1):
            w = cj.commit(ck[0], ck[1], ck[2], vs[b], r["last_row"][b], r["mask"][b], r["enc_noise"][b],
                          r["mlwe_noise"][b])
            assert (_h(outs[s]["com"][b]) == w["com"]).all(), (s, b)
            assert (_h(outs[s]["incom"][b]) == w["incom"]).all(), (s, b)


def test_prover_from_device_key():
    """rg_jindo_create_dev (the key an RCCL broadcast leaves in device memory) == the CRS prover."""
    import torch
    P, q, params, prv, ck = _prover("t10_b8")
    dk = [_t(x) for x in ck]
    prv2 = jindo.Prover(params, ck_dev=dk)
    for a, b in zip(prv2.commit_key(), ck):
        assert (a == b).all()
    v = make_v(q, 900, seed=9)
    rnd = make_randomness(P, q, seed=10)
    c1, o1 = prv.Commit(v, jindo.Randomness(**rnd))
    c2, o2 = prv2.Commit(v, jindo.Randomness(**rnd))
    assert (c1.Value == c2.Value).all() and (o1.InCommit == o2.InCommit).all()
    with pytest.raises(Exception):
        jindo.Prover(params, ck_dev=[dk[0][:10], dk[1], dk[2]])  # too short: refused before any copy


def test_evaluate_2e16_matches_oracle():
    """Prover.Evaluate device work (prover.go:228-314) at configs[4] over a 3-opening shard."""
    import torch
    P, q, params, prv, ck = _prover("t16_b4096")
    B, nv = 3, 65536
    sh = params.shapes(B)
    vs = np.stack([make_v(q, nv, seed=700 + b) for b in range(B)])
    rnd = make_randomness(P, q, seed=71, batch=B, param_sd=True)
    op = {k: torch.zeros(sh[k], dtype=torch.int64, device="cuda") for k in ["incom", "enc", "mlwe_out", "com"]}
    prv.commit_dev(B, _t(vs), nv, _t(rnd["last_row"]), _t(rnd["mask"]), _t(rnd["enc_noise"]), _t(rnd["mlwe_noise"]),
                   op["incom"], op["enc"], op["mlwe_out"], op["com"])
    rng = np.random.default_rng(72)
    es = prv.eval_shapes()
    bq, bo = _residues(P["q"], (B, len(P["q"]), P["d"]), rng), _residues(P["qo"], (B, len(P["qo"]), P["d"]), rng)
    left = _residues(P["q"], (P["rows"], len(P["q"]), P["d"]), rng)
    chals = _residues(P["q"], (P["cols"], len(P["q"]), P["d"]), rng)
    out = {k: torch.zeros(es[k], dtype=torch.int64, device="cuda") for k in es}
    prv.eval_batch_dev(B, op["incom"], op["enc"], op["mlwe_out"], _t(bq), _t(bo), out["ob_incom"], out["ob_enc"],
                       out["ob_mlwe"])
    prv.eval_partial_dev(out["ob_enc"], _t(left), out["partial"])
    prv.eval_respond_dev(out["ob_enc"], out["ob_mlwe"], _t(chals), out["pf_enc"], out["pf_mlwe"])
    torch.cuda.synchronize()
    cj = co.CJindo(P, q)
    ob = cj.eval_batch(_h(op["incom"]), _h(op["enc"]), _h(op["mlwe_out"]), bq, bo)
    for k in ("ob_incom", "ob_enc", "ob_mlwe"):
        assert (_h(out[k]) == ob[k]).all(), k
    assert (_h(out["partial"]) == cj.eval_partial(ob["ob_enc"], left)).all()
    pe, pm = cj.eval_respond(ob["ob_enc"], ob["ob_mlwe"], chals)
    assert (_h(out["pf_enc"]) == pe).all() and (_h(out["pf_mlwe"]) == pm).all()
