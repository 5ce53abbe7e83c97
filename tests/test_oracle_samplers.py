"""CPU: the sampler restatements (math/csprng, jindo/encoder.go:50-67,149-183, prover.go:65-139)
used as the oracle of the device samplers -- pinned where the reference pins anything:
  * the AES-256-CTR UniformSampler stream of oracle.c (OpenSSL AES_encrypt on counter blocks)
    equals pyref's (OpenSSL EVP CTR), including the XOR-accumulating buffer past word 1024, and
    sampler instance n equals the sampler whose IV is IV + n 2^24;
  * deltaInv (exact big.Float emulation) against -b^i / p;
  * the Gaussian samples' first two moments against the reference's standard deviations
    (the samplers' float paths use libm's exp/log: parity with Go's math package is unpinned,
    so these are distribution tests)."""
import hashlib
import json
import os

import numpy as np
import pytest

import coracle as co
import pyref
from tests.jindo_util import make_v

HERE = os.path.dirname(os.path.abspath(__file__))
PARAMS = json.load(open(os.path.join(HERE, "golden", "jindo_params.json")))
SD_KEYS = ("ecd_sd", "ecd_blind_sd", "mask_sd", "mask_blind_sd", "mlwe_sd", "mask_mlwe_sd")


def test_oracle_stream_matches_pyref():
    for seed in (b"Jindo!", bytes(range(32))):
        w = co.uniform_words(seed, 0, 0, 2100)
        u = pyref.UniformSampler(seed)
        assert [int(x) for x in w] == [u.sample() for _ in range(2100)]
        w2 = co.uniform_words(seed, 0, 1500, 10)  # random access into chunk 1
        assert (w2 == w[1500:1510]).all()


@pytest.mark.parametrize("inst", [1, 7, 1 << 40])
def test_instance_is_the_sampler_at_shifted_iv(inst):
    seed = b"instance-test-seed-0123456789abc"
    r = hashlib.sha384(seed).digest()
    iv = (int.from_bytes(r[32:48], "big") + (inst << 24)) % (1 << 128)
    u = pyref.UniformSampler(key=r[:32], iv=iv.to_bytes(16, "big"))
    assert [int(x) for x in co.uniform_words(seed, inst, 0, 1030)] == [u.sample() for _ in range(1030)]


@pytest.mark.parametrize("base,exp", [(60272, 16), (60256, 8), (47104, 4)])
def test_delta_inv(base, exp):
    from fractions import Fraction
    d = pyref.delta_inv(base, exp)
    p = base ** exp + 1
    thr = 2.0 ** -50 / (base * exp)
    for i, x in enumerate(d):
        exact = -Fraction(base ** i, p)
        if abs(float(exact)) < thr * 0.999:
            assert x == 0.0
        else:
            assert abs(Fraction(x) - exact) <= abs(exact) * Fraction(1, 2 ** 52), i


def _sample(name, B=1, nv=None, first=0, seed=b"s"):
    P = PARAMS[name]
    q = int(P["field_q_hex"], 16)
    nv = nv or P["rank"]
    v = np.stack([make_v(q, nv, seed=11 + b) for b in range(B)])
    seeds = b"".join(hashlib.sha256(seed + bytes([i])).digest() for i in range(6))
    cj = co.CJindo(P, q)
    sd = [P[k] for k in SD_KEYS]
    out = cj.sample(sd, pyref.delta_inv(P["base"], P["exp"]), seeds, first, v)
    return P, q, out


def test_oracle_sample_moments():
    """t14: TwinCDT (ecd, mlwe), COSAC (mask columns) and rounded (MLWE mask) widths."""
    P, q, o = _sample("t14_b1")
    en, mn, cols = o["enc_noise"][0], o["mlwe_noise"][0], P["cols"]
    data = en[:cols, 1:].astype(np.float64)  # TwinCDT rows (centres are O(1))
    assert abs(data.std() / P["ecd_sd"] - 1) < 0.02
    assert abs(data.mean()) < 0.5
    mask = en[cols, 1:].astype(np.float64)  # COSAC, maskStdDev
    assert abs(mask.std() / P["mask_sd"] - 1) < 0.03
    assert abs(en[:cols, 0].astype(np.float64).std() / P["ecd_blind_sd"] - 1) < 0.1  # COSAC, 2k samples
    ml = mn[:cols].astype(np.float64)
    assert abs(ml.std() / P["mlwe_sd"] - 1) < 0.02 and abs(ml.mean()) < 0.1
    assert abs(mn[cols].astype(np.float64).std() / P["mask_mlwe_sd"] - 1) < 0.05


def test_oracle_uniform_elements():
    P, q, o = _sample("t10_b1", B=2)
    L = (q.bit_length() + 63) // 64
    for b in range(2):
        vals = [sum(int(x) << (64 * l) for l, x in enumerate(e)) for e in o["mask"][b].reshape(-1, L)]
        assert all(x < q for x in vals) and len(set(vals)) == len(vals)
        assert (o["last_row"][b, -1] == 0).all()
    # same seeds, shifted first_commit: commit 1 of (first 0, batch 2) == commit 0 of (first 1)
    _, _, o1 = _sample("t10_b1", B=1, first=1)
    P2, q2, o2 = _sample("t10_b1", B=2)
    assert (o1["mask"][0] == o2["mask"][1]).all() and (o1["last_row"][0] == o2["last_row"][1]).all()
