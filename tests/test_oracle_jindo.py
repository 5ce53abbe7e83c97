"""CPU: Jindo restatements agree with each other and with the scheme's algebra.

  * C oracle commit == big-int commit (prover.go:45-202), 2-prime and 3-prime rings, full and
    partial v (the reference's row-skipping branches, prover.go:103-105,121-123);
  * DecodeTo(Encode) == v: decoding the opening's encodes (encoder.go:204-219) recovers the
    committed rows -- exercises the Lattigo-convention NTT/MForm chain end to end;
  * parameter shapes == the SURVEY.md §8 table (restated NewParameters, params.go:126-320);
  * CK stream: first words of the AES-CTR keystream for crs "Jindo!" are stable (fixture).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import coracle as co
import pyref
from tests.jindo_util import make_randomness, make_v

HERE = os.path.dirname(os.path.abspath(__file__))
PARAMS = json.load(open(os.path.join(HERE, "golden", "jindo_params.json")))


def test_params_match_survey_table():
    want = {  # rows, cols, inMSIS, mlwe, dcmp, outMSIS, logIn, logOut, |q|, |qo|
        "t10_b1": (33, 2, 10, 32, 30, 6, 41, 29, 2, 1),
        "t10_b8": (65, 1, 15, 32, 30, 13, 41, 66, 2, 2),
        "t14_b1": (129, 8, 10, 32, 90, 6, 42, 31, 2, 1),
        "t16_b1": (257, 16, 10, 32, 170, 6, 43, 31, 2, 1),
        "t16_b4096": (513, 8, 16, 32, 144, 15, 43, 74, 2, 2),
        "mult_t8193_b12": (130, 2, 21, 32, 63, 21, 41, 109, 3, 3),
    }
    for k, w in want.items():
        P = PARAMS[k]
        got = (P["rows"], P["cols"], P["in_msis"], P["mlwe"], P["in_com_dcmp_len"], P["out_msis"],
               P["log_in_cut"], P["log_out_cut"], len(P["q"]), len(P["qo"]))
        assert got == w, k
        for q in P["q"] + P["qo"]:
            assert pyref.is_prime(q) and (q - 1) % (2 * P["d"]) == 0


@pytest.mark.parametrize("name,nv", [("t10_b1", 1024), ("t10_b1", 300), ("t10_b8", 700), ("mult_t8193_b12", 1500),
                                     # the zp package's other fields as Jindo fields (exp 4 .. 64,
                                     # limbs 1 .. 14; buckler/compile.go:178)
                                     ("p63_t10_b2", 1019), ("zp110_t10_b1", 1019), ("zp220_t10_b1", 1019),
                                     ("zp440_t10_b2", 1019), ("zp880_t10_b1", 1019)])
def test_c_commit_equals_bigint_commit(name, nv):
    P = PARAMS[name]
    q = int(P["field_q_hex"], 16)
    F = pyref.Field(q)
    Pp = pyref.JindoParams(q, P["target_n"], P["batch"])
    ck = pyref.commit_key(Pp, b"Jindo!")
    v = make_v(q, nv, seed=nv)
    rnd = make_randomness(P, q, seed=3)
    vals = co.from_limbs(v)
    prnd = dict(last_row=co.from_limbs(rnd["last_row"]),
                mask=[co.from_limbs(rnd["mask"][j]) for j in range(P["rows"])],
                enc_noise=rnd["enc_noise"].tolist(), mlwe_noise=rnd["mlwe_noise"].tolist())
    com, op = pyref.commit(Pp, F, ck, vals, prnd)
    o = co.CJindo(P, q).commit(*[np.array(x, np.uint64) for x in ck], v, rnd["last_row"], rnd["mask"],
                               rnd["enc_noise"], rnd["mlwe_noise"])
    assert (o["com"] == np.array(com, np.uint64)).all()
    assert (o["incom"] == np.array(op["InCommit"], np.uint64)).all()
    assert (o["enc"] == np.array(op["Encode"], np.uint64)).all()
    assert (o["mlwe"] == np.array(op["MLWE"], np.uint64)).all()


def test_decode_of_encode_recovers_rows():
    """encoder.go:204-219 DecodeTo applied to Opening.Encode returns the committed values:
    Encode = NTT(MForm(digits + s (X^slots - b))) and X^slots = b kills the noise term."""
    name = "t10_b1"
    P = PARAMS[name]
    q = int(P["field_q_hex"], 16)
    F = pyref.Field(q)
    Pp = pyref.JindoParams(q, P["target_n"], P["batch"])
    ck = [np.array(x, np.uint64) for x in pyref.commit_key(Pp, b"Jindo!")]
    nv = 1024
    v = make_v(q, nv, seed=11)
    rnd = make_randomness(P, q, seed=12)
    o = co.CJindo(P, q).commit(*ck, v, rnd["last_row"], rnd["mask"], rnd["enc_noise"], rnd["mlwe_noise"])
    ring = pyref.Ring(P["d"], P["q"])
    vals = co.from_limbs(v)
    cs = P["cols"] * P["slots"]
    for i in range(P["cols"]):
        for j in range(1, P["rows"] - 1):
            s0 = j * cs + i * P["slots"]
            if s0 >= nv:
                break
            limbs = o["enc"][i, j]
            coeffs = [sr.imform(sr.intt(list(map(int, limbs[l])))) for l, sr in enumerate(ring.sub)]
            cvals = [pyref.reconstruct(P["q"], [coeffs[l][k] for l in range(len(P["q"]))]) for k in range(P["d"])]
            for s in range(P["slots"]):
                acc = 0
                for jj in range(P["exp"] - 1, -1, -1):
                    acc = (acc * P["base"] + cvals[jj * P["slots"] + s]) % q
                want = F.from_mont(vals[s0 + s]) if s0 + s < nv else 0
                assert acc == want, (i, j, s)


def test_ck_stream_stable():
    u = pyref.UniformSampler(b"Jindo!")
    words = [u.sample() for _ in range(4)]
    h = hashlib.sha256(b"".join(w.to_bytes(8, "little") for w in words)).hexdigest()
    G = json.load(open(os.path.join(HERE, "golden", "jindo_commit_golden.json")))
    P = PARAMS["t10_b1"]
    q = int(P["field_q_hex"], 16)
    ck = pyref.commit_key(pyref.JindoParams(q, P["target_n"], P["batch"]), b"Jindo!")
    assert [hashlib.sha256(np.ascontiguousarray(np.array(x, np.uint64)).tobytes()).hexdigest() for x in ck] == G["ck"]
    assert len(h) == 64


def test_uniform_sampler_refill_xors_into_buffer():
    """uniform.go:64-70: every 8192-byte refill is `XORKeyStream(buf, buf)`, so Sample() word
    w of chunk c = 1024 w-words is KS_0[w] ^ ... ^ KS_c[w] (KS_i = i-th 8192-byte keystream chunk),
    not plain keystream; the CK derivation (entities.go:21-73) reads ~10^6 words through it."""
    u = pyref.UniformSampler(b"Jindo!")
    words = [u.sample() for _ in range(3 * 1024 + 5)]
    r = hashlib.sha384(b"Jindo!").digest()
    ks = pyref.aes256_ctr_keystream(r[:32], r[32:48], 4 * 8192)
    kw = [int.from_bytes(ks[8 * i:8 * i + 8], "little") for i in range(4 * 1024)]
    for w in (0, 1, 1023):
        assert words[w] == kw[w]
    for w in (1024, 1500, 2047):
        assert words[w] == kw[w] ^ kw[w - 1024]
    for w in (2048, 3 * 1024 + 4):
        c, o = divmod(w, 1024)
        x = 0
        for i in range(c + 1):
            x ^= kw[1024 * i + o]
        assert words[w] == x
