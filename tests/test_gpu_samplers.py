"""GPU parity of the device samplers (csrc/csprng.hpp, jindo.hip section 6) against the C
restatement (oracle/oracle.c of_jindo_sample / of_uniform_words over OpenSSL AES), bit for bit:
the AES-256-CTR UniformSampler stream, deltaInv, and every draw of Prover.Commit's randomness
(lastRow, mask, encode noise with its deltaInv centres, MLWE noise) over several parameter sets,
batches and first_commit offsets; then the end-to-end device Commit on that randomness."""
import hashlib
import json
import os

import numpy as np
import pytest

import coracle as co
import pyref
from ringo import jindo
from tests.jindo_util import make_v

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
PARAMS = json.load(open(os.path.join(HERE, "golden", "jindo_params.json")))
SD_KEYS = jindo.STDDEV_KEYS


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to("cuda")


def _h(t):
    return t.cpu().numpy()


@pytest.mark.parametrize("inst,first,n", [(0, 0, 3000), (5, 1000, 100), (1 << 30, 2040, 20)])
def test_uniform_words_match_oracle(inst, first, n):
    import torch
    seed = b"Jindo!"
    out = torch.zeros(n, dtype=torch.int64, device="cuda")
    jindo.uniform_words_dev(seed, inst, first, n, out)
    torch.cuda.synchronize()
    assert (_h(out).view(np.uint64) == co.uniform_words(seed, inst, first, n)).all()


@pytest.mark.parametrize("name", ["t10_b1", "mult_t8193_b12"])
def test_delta_inv_matches_bigfloat(name):
    P = PARAMS[name]
    q = int(P["field_q_hex"], 16)
    prv = jindo.NewProver(jindo.Parameters.from_dict(P, q), b"Jindo!")
    assert prv.delta_inv() == pyref.delta_inv(P["base"], P["exp"])


def _seeds(tag):
    return jindo.Seeds.derive(tag)


@pytest.mark.parametrize("name,B,nv,first", [("t10_b1", 2, None, 3), ("t10_b1", 1, 300, 0), ("t10_b8", 3, 700, 11),
                                             ("mult_t8193_b12", 1, None, 0), ("t14_b1", 1, None, 5),
                                             ("t16_b4096", 1, 40000, 511)])
def test_sample_matches_oracle(name, B, nv, first):
    import torch
    P = PARAMS[name]
    q = int(P["field_q_hex"], 16)
    params = jindo.Parameters.from_dict(P, q)
    prv = jindo.NewProver(params, b"Jindo!")
    nv = nv or P["rank"]
    v = np.stack([make_v(q, nv, seed=21 + b) for b in range(B)])
    seeds = _seeds(b"sample-" + name.encode())
    sh = params.shapes(B)
    o = {k: torch.zeros(sh[k], dtype=torch.int64, device="cuda") for k in ("last_row", "mask", "enc_noise", "mlwe_noise")}
    prv.sample_dev(B, _t(v), nv, seeds, first, o["last_row"], o["mask"], o["enc_noise"], o["mlwe_noise"])
    torch.cuda.synchronize()
    want = co.CJindo(P, q).sample([P[k] for k in SD_KEYS], pyref.delta_inv(P["base"], P["exp"]), seeds.raw(), first, v)
    assert (_h(o["last_row"]).view(np.uint64) == want["last_row"]).all()
    assert (_h(o["mask"]).view(np.uint64) == want["mask"]).all()
    assert (_h(o["mlwe_noise"]) == want["mlwe_noise"]).all()
    assert (_h(o["enc_noise"]) == want["enc_noise"]).all()


def test_commit_sampled_end_to_end():
    """rg_jindo_commit_sampled_dev == rg_jindo_commit_dev on rg_jindo_sample_dev's draws == the
    C oracle's commit on the C oracle's draws."""
    import torch
    name = "t10_b8"
    P = PARAMS[name]
    q = int(P["field_q_hex"], 16)
    params = jindo.Parameters.from_dict(P, q)
    prv = jindo.NewProver(params, b"Jindo!")
    ck = prv.commit_key()
    B, nv, first = 2, 1024, 7
    v = np.stack([make_v(q, nv, seed=31 + b) for b in range(B)])
    seeds = _seeds(b"e2e")
    sh = params.shapes(B)
    z = lambda k: torch.zeros(sh[k], dtype=torch.int64, device="cuda")
    a = {k: z(k) for k in ("incom", "enc", "mlwe_out", "com")}
    prv.commit_sampled_dev(B, _t(v), nv, seeds, first, a["incom"], a["enc"], a["mlwe_out"], a["com"])
    r = {k: z(k) for k in ("last_row", "mask", "enc_noise", "mlwe_noise")}
    prv.sample_dev(B, _t(v), nv, seeds, first, r["last_row"], r["mask"], r["enc_noise"], r["mlwe_noise"])
    b_ = {k: z(k) for k in ("incom", "enc", "mlwe_out", "com")}
    prv.commit_dev(B, _t(v), nv, r["last_row"], r["mask"], r["enc_noise"], r["mlwe_noise"], b_["incom"], b_["enc"],
                   b_["mlwe_out"], b_["com"])
    torch.cuda.synchronize()
    for k in a:
        assert torch.equal(a[k], b_[k]), k
    cj = co.CJindo(P, q)
    rnd = cj.sample([P[k] for k in SD_KEYS], pyref.delta_inv(P["base"], P["exp"]), seeds.raw(), first, v)
    for b in range(B):
        w = cj.commit(ck[0], ck[1], ck[2], v[b], rnd["last_row"][b], rnd["mask"][b], rnd["enc_noise"][b],
                      rnd["mlwe_noise"][b])
        assert (_h(a["com"][b]).view(np.uint64) == w["com"]).all(), b
        assert (_h(a["enc"][b]).view(np.uint64) == w["enc"]).all(), b


def test_sample_moments_2e16():
    """configs[4]: device draws have the reference's widths (distribution check on one commit)."""
    import torch
    P = PARAMS["t16_b4096"]
    q = int(P["field_q_hex"], 16)
    params = jindo.Parameters.from_dict(P, q)
    prv = jindo.NewProver(params, b"Jindo!")
    v = make_v(q, P["rank"], seed=3)[None]
    sh = params.shapes(1)
    o = {k: torch.zeros(sh[k], dtype=torch.int64, device="cuda") for k in ("last_row", "mask", "enc_noise", "mlwe_noise")}
    prv.sample_dev(1, _t(v), P["rank"], _seeds(b"moments"), 0, o["last_row"], o["mask"], o["enc_noise"],
                   o["mlwe_noise"])
    torch.cuda.synchronize()
    en, mn, cols = _h(o["enc_noise"])[0].astype(np.float64), _h(o["mlwe_noise"])[0].astype(np.float64), P["cols"]
    assert abs(en[:cols, 1:].std() / P["ecd_sd"] - 1) < 0.01
    assert abs(en[cols, 1:].std() / P["mask_sd"] - 1) < 0.01
    assert abs(mn[:cols].std() / P["mlwe_sd"] - 1) < 0.02
    assert abs(mn[cols].std() / P["mask_mlwe_sd"] - 1) < 0.05


def test_commit_sampled_two_stream_split():
    """A sampled batch of >= 64 commits runs as two halves on two streams (the caller's and the
    handle's auxiliary one, joined by events): equal, bit for bit, to the single-stream runs of
    the same commits (rg_jindo_sample_dev + rg_jindo_commit_dev of the whole batch, and two
    sub-batches of < 64 with their first_commit offsets), on a caller stream that is not the null
    stream."""
    import torch
    name = "t10_b1"
    P = PARAMS[name]
    q = int(P["field_q_hex"], 16)
    params = jindo.Parameters.from_dict(P, q)
    prv = jindo.NewProver(params, b"Jindo!")
    B, nv, first = 70, 1000, 5
    v = np.stack([make_v(q, nv, seed=400 + b) for b in range(B)])
    seeds = _seeds(b"split")
    sh = params.shapes(B)
    z = lambda k: torch.zeros(sh[k], dtype=torch.int64, device="cuda")
    keys = ("incom", "enc", "mlwe_out", "com")
    st = torch.cuda.Stream()
    a = {k: z(k) for k in keys}
    dv = _t(v)
    torch.cuda.synchronize()
    prv.commit_sampled_dev(B, dv, nv, seeds, first, a["incom"], a["enc"], a["mlwe_out"], a["com"], st)
    st.synchronize()
    b_ = {k: z(k) for k in keys}
    for lo, hi in ((0, 30), (30, B)):
        prv.commit_sampled_dev(hi - lo, dv[lo:hi], nv, seeds, first + lo, b_["incom"][lo:hi], b_["enc"][lo:hi],
                               b_["mlwe_out"][lo:hi], b_["com"][lo:hi])
    r = {k: z(k) for k in ("last_row", "mask", "enc_noise", "mlwe_noise")}
    prv.sample_dev(B, dv, nv, seeds, first, r["last_row"], r["mask"], r["enc_noise"], r["mlwe_noise"])
    c = {k: z(k) for k in keys}
    prv.commit_dev(B, dv, nv, r["last_row"], r["mask"], r["enc_noise"], r["mlwe_noise"], c["incom"], c["enc"],
                   c["mlwe_out"], c["com"])
    torch.cuda.synchronize()
    for k in keys:
        assert torch.equal(a[k], b_[k]), k
        assert torch.equal(a[k], c[k]), k
