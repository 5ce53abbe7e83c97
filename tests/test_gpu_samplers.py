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


@pytest.mark.parametrize("inst,first,n", [(0, 0, 3000), (5, 1000, 100), (1 << 30, 2040, 20), ((1 << 40) + 3, 0, 1100),
                                           (1 << 41, 1020, 40), ((1 << 64) - 1, 0, 70)])
def test_uniform_words_match_oracle(inst, first, n):
    import torch
    seed = b"Jindo!"
    out = torch.zeros(n, dtype=torch.int64, device="cuda")
    jindo.uniform_words_dev(seed, inst, first, n, out)
    torch.cuda.synchronize()
    assert (_h(out).view(np.uint64) == co.uniform_words(seed, inst, first, n)).all()


@pytest.mark.parametrize("tries", [0, 1])
def test_uniform_long_draws_fixup(tmp_path, tries):
    """MustSetRandom's whole-word draws that uniform_whole_kernel leaves (all-ones, flagged) are
    completed by uniform_fix_kernel with the same words: on the experiments build with
    RINGO_JINDO_UNI_TRIES=0 (every draw goes to the fix-up) or 1 (the ~47% rejected on their first
    try at q255 do), lastRow and mask still equal the oracle's draws (tests/exp_child.py)."""
    import subprocess
    import sys
    name, B, first = "t10_b1", 2, 3
    out = tmp_path / f"uni_{tries}.npz"
    r = subprocess.run([sys.executable, os.path.join(HERE, "exp_child.py"), "uni", str(tries), str(out), name, str(B),
                        str(first)], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    got = np.load(out)
    P = PARAMS[name]
    q = int(P["field_q_hex"], 16)
    v = np.stack([make_v(q, P["rank"], seed=21 + b) for b in range(B)])
    want = co.CJindo(P, q).sample([P[k] for k in SD_KEYS], pyref.delta_inv(P["base"], P["exp"]),
                                  _seeds(b"uni-" + name.encode()).raw(), first, v)
    assert (got["last_row"].view(np.uint64) == want["last_row"]).all()
    assert (got["mask"].view(np.uint64) == want["mask"]).all()


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
                                             ("t16_b4096", 1, 40000, 511),
                                             # COSAC instances past 2^40 (the window start carries into
                                             # the counter's high word) ...
                                             ("t16_b4096", 1, 40000, 940000),
                                             # ... and the last commit whose instances fit in a u64
                                             ("t16_b4096", 1, 40000, (1 << 64) // (9 * 513 * 256) - 1)])
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


def _iv_low16(seed):
    """low 16 bits of a UniformSampler's IV = SHA-384(seed)[32:48] (big-endian counter)"""
    return int.from_bytes(hashlib.sha384(seed).digest()[46:48], "big")


def _seed_with_iv_low(lo, hi, tag):
    for i in range(1 << 22):
        s = hashlib.sha256(tag + i.to_bytes(4, "little")).digest()
        if lo <= _iv_low16(s) <= hi:
            return s
    raise AssertionError("no seed found")


@pytest.mark.parametrize("lo,hi", [(0xFF81, 0xFFFF), (0xFF70, 0xFF80), (0, 0x7F)])
def test_cdt_counter_prefix_boundary(lo, hi):
    """cdt2_noise_kernel's counter-mode caching (csprng.hpp aes_prefix) serves a polynomial's 128
    blocks when its window start's low 16 counter bits leave room for them without a carry, and
    the plain AES otherwise.  The window start's low 24 bits are the IV's, so the seed decides:
    an IV straddling the boundary (>= 0xFF81: plain path), one that just fits (<= 0xFF80) and a
    small one, each bit-exact against the oracle."""
    import dataclasses

    import torch
    name, B, nv, first = "t10_b8", 3, 700, 11
    P = PARAMS[name]
    q = int(P["field_q_hex"], 16)
    params = jindo.Parameters.from_dict(P, q)
    prv = jindo.NewProver(params, b"Jindo!")
    v = np.stack([make_v(q, nv, seed=41 + b) for b in range(B)])
    seeds = dataclasses.replace(_seeds(b"prefix"), enc_cdt=_seed_with_iv_low(lo, hi, b"iv-%d" % lo))
    sh = params.shapes(B)
    o = {k: torch.zeros(sh[k], dtype=torch.int64, device="cuda") for k in ("last_row", "mask", "enc_noise", "mlwe_noise")}
    prv.sample_dev(B, _t(v), nv, seeds, first, o["last_row"], o["mask"], o["enc_noise"], o["mlwe_noise"])
    torch.cuda.synchronize()
    want = co.CJindo(P, q).sample([P[k] for k in SD_KEYS], pyref.delta_inv(P["base"], P["exp"]), seeds.raw(), first, v)
    assert (_h(o["enc_noise"]) == want["enc_noise"]).all()
    assert (_h(o["mlwe_noise"]) == want["mlwe_noise"]).all()


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
    """A sampled batch runs as one DAG over the caller's stream and two helper streams of it
    (samplers and the MLWE prep beside the TwinCDT / encode chain, joined by events): equal, bit
    for bit, to other schedules of the same commits (rg_jindo_sample_dev + rg_jindo_commit_dev of
    the whole batch on one stream, and two sub-batches with their first_commit offsets), on a
    caller stream that is not the null stream."""
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


def test_first_commit_range_rejected():
    """The sampled entry points refuse a first_commit whose instance numbers would pass 2^64 - 1
    (include/ringo.h rg_jindo_seeds); the last one that fits is accepted."""
    import torch
    from ringo._lib import RingoError
    P = PARAMS["t10_b1"]
    q = int(P["field_q_hex"], 16)
    params = jindo.Parameters.from_dict(P, q)
    prv = jindo.NewProver(params, b"Jindo!")
    per = max((P["cols"] + 1) * P["rows"] * P["d"], (P["cols"] + 1) * (P["in_msis"] + P["mlwe"]) * P["d"],
              (P["cols"] + P["rows"]) * P["slots"])  # the largest per-commit instance count of a domain
    v = make_v(q, 64, seed=5)[None]
    sh = params.shapes(1)
    o = {k: torch.zeros(sh[k], dtype=torch.int64, device="cuda") for k in ("last_row", "mask", "enc_noise", "mlwe_noise")}
    last_ok = (1 << 64) // per - 1
    prv.sample_dev(1, _t(v), 64, _seeds(b"range"), last_ok, o["last_row"], o["mask"], o["enc_noise"], o["mlwe_noise"])
    torch.cuda.synchronize()
    for first in (last_ok + 1, (1 << 64) - 1):
        with pytest.raises(RingoError):
            prv.sample_dev(1, _t(v), 64, _seeds(b"range"), first, o["last_row"], o["mask"], o["enc_noise"],
                           o["mlwe_noise"])
    sc = params.shapes(1)
    z = {k: torch.zeros(sc[k], dtype=torch.int64, device="cuda") for k in ("incom", "enc", "mlwe_out", "com")}
    with pytest.raises(RingoError):
        prv.commit_sampled_dev(1, _t(v), 64, _seeds(b"range"), last_ok + 1, z["incom"], z["enc"], z["mlwe_out"],
                               z["com"])


def test_commit_sampled_concurrent_streams():
    """Two host threads issue sampled batches of different sizes (64 and 160: both split over an
    auxiliary stream) on their own streams at once; each result equals the same batch run alone on
    the default stream, bit for bit (the auxiliary stream and its scratch belong to the caller
    stream).  Then each stream's scratch is released and the handle still works."""
    import threading
    import torch
    P = PARAMS["t10_b1"]
    q = int(P["field_q_hex"], 16)
    params = jindo.Parameters.from_dict(P, q)
    prv = jindo.NewProver(params, b"Jindo!")
    nv = 500
    keys = ("incom", "enc", "mlwe_out", "com")
    jobs = []
    for i, B in enumerate((64, 160)):
        v = _t(np.stack([make_v(q, nv, seed=700 + 17 * i + b) for b in range(B)]))
        sh = params.shapes(B)
        jobs.append(dict(B=B, v=v, first=1000 * i, st=torch.cuda.Stream(), sh=sh,
                         out={k: torch.zeros(sh[k], dtype=torch.int64, device="cuda") for k in keys}))
    torch.cuda.synchronize()
    errs = []
    dev = torch.cuda.current_device()

    def work(j):
        try:
            torch.cuda.set_device(dev)
            for _ in range(3):  # repeated, so the two callers' launches interleave
                prv.commit_sampled_dev(j["B"], j["v"], nv, _seeds(b"conc"), j["first"], *[j["out"][k] for k in keys],
                                       stream=j["st"])
            j["st"].synchronize()
        except Exception as e:  # noqa: BLE001 -- re-raised on the main thread
            errs.append(e)

    th = [threading.Thread(target=work, args=(j,)) for j in jobs]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for j in jobs:
        ref = {k: torch.zeros(j["sh"][k], dtype=torch.int64, device="cuda") for k in keys}
        prv.commit_sampled_dev(j["B"], j["v"], nv, _seeds(b"conc"), j["first"], *[ref[k] for k in keys])
        torch.cuda.synchronize()
        for k in keys:
            assert torch.equal(j["out"][k], ref[k]), (j["B"], k)
    for j in jobs:
        prv.release_stream(j["st"])
    again = {k: torch.zeros(jobs[0]["sh"][k], dtype=torch.int64, device="cuda") for k in keys}
    prv.commit_sampled_dev(64, jobs[0]["v"], nv, _seeds(b"conc"), 0, *[again[k] for k in keys], stream=jobs[0]["st"])
    jobs[0]["st"].synchronize()
    for k in keys:
        assert torch.equal(again[k], jobs[0]["out"][k]), k


def test_unsupported_sampling_shape_refused():
    """Device sampling covers d = 256, slots % 4 == 0 and encode TwinCDT tables of <= 96 entries
    (every NewParameters shape of a field with exp <= 64).  Outside that the sampled entry points
    return RG_ERR_UNSUPPORTED with the reason, before any launch: here an encode stddev far above
    NewParameters' ecdStdDev (a 2,000-entry table)."""
    import torch
    from ringo._lib import RingoError
    P = PARAMS["t10_b1"]
    q = int(P["field_q_hex"], 16)
    params = jindo.Parameters.from_dict(P, q)
    sd = list(params.stddevs)
    sd[0] = 400.0
    params.stddevs = tuple(sd)
    prv = jindo.NewProver(params, b"Jindo!")
    v = make_v(q, 64, seed=5)[None]
    sh = params.shapes(1)
    o = {k: torch.zeros(sh[k], dtype=torch.int64, device="cuda") for k in ("last_row", "mask", "enc_noise", "mlwe_noise")}
    with pytest.raises(RingoError, match="TwinCDT table"):
        prv.sample_dev(1, _t(v), 64, _seeds(b"big"), 0, o["last_row"], o["mask"], o["enc_noise"], o["mlwe_noise"])
