"""jindo mirror (jindo/) over libringo.

    params = Parameters(...)            # shapes as jindo.Parameters holds them (params.go:64-123)
    prv = NewProver(params, b"Jindo!")  # prover.go:28 (commit key derived from the CRS on the host)
    com, open_ = prv.Commit(v, rnd)     # prover.go:45, randomness injected (see Randomness)

The reference's Commit draws its randomness internally (crypto/rand, Gaussian samplers); this
mirror takes those draws as arguments so the result is bit-exact against Go given identical
draws.  The Go-side NewParameters float search is not re-derived here: shapes
are passed in (tests take them from committed fixtures).
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from ._lib import JindoParamsC, JindoSeedsC, JindoStddevsC, check, iptr, lib, ptr, vp
from .bigpoly import RingoPanic, _addr, _stream


STDDEV_KEYS = ("ecd_sd", "ecd_blind_sd", "mask_sd", "mask_blind_sd", "mlwe_sd", "mask_mlwe_sd")


@dataclass
class Seeds:
    """One 32-byte seed per sampler Commit draws from (include/ringo.h rg_jindo_seeds)."""
    enc_cdt: bytes
    enc_cosac: bytes
    enc_cosac_round: bytes
    mlwe_cdt: bytes
    mlwe_round: bytes
    uniform: bytes

    @classmethod
    def derive(cls, master):
        """Six seeds from one: SHA-256(master || name) (a convenience; Go draws each from crypto/rand)."""
        import hashlib
        return cls(**{k: hashlib.sha256(bytes(master) + k.encode()).digest() for k in cls.__dataclass_fields__})

    def raw(self):
        return b"".join(getattr(self, k) for k in self.__dataclass_fields__)

    def c_struct(self):
        s = JindoSeedsC()
        for k in self.__dataclass_fields__:
            v = getattr(self, k)
            if len(v) != 32:
                raise RingoPanic("seed must be 32 bytes")
            ctypes.memmove(getattr(s, k), v, 32)
        return s


@dataclass
class Parameters:
    rank: int
    rows: int
    cols: int
    slots: int
    exp: int
    d: int
    in_msis: int
    out_msis: int
    mlwe: int
    dcmp: int
    log_in_cut: int
    log_out_cut: int
    base: int
    q: list
    qo: list
    field_q: int
    stddevs: tuple = None  # ecd, ecd_blind, mask, mask_blind, mlwe, mask_mlwe (params.go:99-111)
    res_two_nm: float = None          # ResTwoNm() (params.go:432-435)
    in_com_dcmp_two_nm: float = None  # InComDcmpTwoNm() (params.go:437-440)

    @classmethod
    def from_dict(cls, P, field_q):
        return cls(rank=P["rank"], rows=P["rows"], cols=P["cols"], slots=P["slots"], exp=P["exp"], d=P["d"],
                   in_msis=P["in_msis"], out_msis=P["out_msis"], mlwe=P["mlwe"], dcmp=P["in_com_dcmp_len"],
                   log_in_cut=P["log_in_cut"], log_out_cut=P["log_out_cut"], base=P["base"], q=list(P["q"]),
                   qo=list(P["qo"]), field_q=int(field_q),
                   stddevs=tuple(P[k] for k in STDDEV_KEYS) if all(k in P for k in STDDEV_KEYS) else None,
                   res_two_nm=P.get("res_two_nm"), in_com_dcmp_two_nm=P.get("in_com_dcmp_two_nm"))

    @property
    def L(self):
        return (self.field_q.bit_length() + 63) // 64

    @property
    def nq(self):
        return len(self.q)

    @property
    def nqo(self):
        return len(self.qo)

    def c_struct(self):
        s = JindoParamsC()
        for k in ["rank", "rows", "cols", "slots", "exp", "d", "in_msis", "out_msis", "mlwe", "dcmp", "log_in_cut",
                  "log_out_cut"]:
            setattr(s, k, int(getattr(self, k)))
        s.base = self.base
        s.nq, s.nqo = self.nq, self.nqo
        for i, x in enumerate(self.q):
            s.q[i] = x
        for i, x in enumerate(self.qo):
            s.qo[i] = x
        s.field_limbs = self.L
        for i in range(self.L):
            s.field_q[i] = (self.field_q >> (64 * i)) & ((1 << 64) - 1)
        return s

    # array shapes (include/ringo.h rg_jindo_commit)
    def shapes(self, batch=None):
        nm = self.in_msis + self.mlwe
        sh = dict(last_row=(self.cols * self.slots, self.L), mask=(self.rows, self.slots, self.L),
                  enc_noise=(self.cols + 1, self.rows, self.d), mlwe_noise=(self.cols + 1, nm, self.d),
                  incom=(self.dcmp, self.nqo, self.d), enc=(self.cols + 1, self.rows, self.nq, self.d),
                  mlwe_out=(self.cols + 1, nm, self.nq, self.d), com=(self.out_msis, self.nq, self.d))
        if batch is not None:
            sh = {k: (batch,) + v for k, v in sh.items()}
        return sh

    def ck_shapes(self):
        return dict(ck_in=(self.in_msis, self.rows, self.nq, self.d),
                    ck_mlwe=(self.in_msis, self.mlwe, self.nq, self.d),
                    ck_out=(self.out_msis, self.dcmp, self.nqo, self.d))


@dataclass
class Randomness:
    """The draws Prover.Commit makes internally (prover.go:65-139), injected."""
    last_row: np.ndarray    # [cols*slots][L] Montgomery, last entry 0
    mask: np.ndarray        # [rows][slots][L]
    enc_noise: np.ndarray   # [cols+1][rows][d] int64
    mlwe_noise: np.ndarray  # [cols+1][inMSIS+mlwe][d] int64


@dataclass
class Opening:  # entities.go:103-107
    InCommit: np.ndarray
    Encode: np.ndarray
    MLWE: np.ndarray


@dataclass
class Commitment:  # entities.go:80-82
    Value: np.ndarray


def _words(shape):
    n = 1
    for x in shape:
        n *= int(x)
    return n


class Prover:
    def __init__(self, params, crs=None, ck=None, ck_dev=None, stream=None):
        """ck: host arrays (rg_jindo_create); ck_dev: device buffers on the current GPU, e.g. where
        an RCCL broadcast put the key (rg_jindo_create_dev: copied device-to-device); else the
        key is derived from `crs` (NewCommitKey, entities.go:21-73)."""
        self.params = params
        h = vp()
        ps = params.c_struct()
        if ck_dev is not None:
            sh = params.ck_shapes()
            a, b, c = (_addr(x, _words(sh[k])) for x, k in zip(ck_dev, ("ck_in", "ck_mlwe", "ck_out")))
            st = lib().rg_jindo_create_dev(ctypes.byref(ps), a, b, c, _stream(stream), ctypes.byref(h))
        elif ck is not None:
            a, b, c = (np.ascontiguousarray(x, np.uint64) for x in ck)
            st = lib().rg_jindo_create(ctypes.byref(ps), ptr(a), ptr(b), ptr(c), ctypes.byref(h))
        else:
            st = lib().rg_jindo_create_from_crs(ctypes.byref(ps), crs, len(crs), ctypes.byref(h))
        check(st)
        self.h = h
        self._L = lib()
        if params.stddevs is not None:
            sd = JindoStddevsC(*params.stddevs)
            check(lib().rg_jindo_set_stddevs(self.h, ctypes.byref(sd)))

    def __del__(self):
        if getattr(self, "h", None) and getattr(self, "_L", None):  # the CDLL bound at creation
            self._L.rg_jindo_destroy(self.h)  # (module globals may already be gone at interpreter exit)
            self.h = None

    def commit_key(self):
        sh = self.params.ck_shapes()
        out = {k: np.zeros(v, np.uint64) for k, v in sh.items()}
        check(lib().rg_jindo_commit_key(self.h, ptr(out["ck_in"]), ptr(out["ck_mlwe"]), ptr(out["ck_out"])))
        return out["ck_in"], out["ck_mlwe"], out["ck_out"]

    def Commit(self, v, rnd):
        """Commit(v) (prover.go:45-62) with injected randomness; v: [n][L] Montgomery."""
        P = self.params
        v = np.ascontiguousarray(v, np.uint64)
        if v.shape[0] > P.rank:
            raise RingoPanic("len(v) > params.rank")
        sh = P.shapes()
        o = {k: np.zeros(sh[k], np.uint64) for k in ["incom", "enc", "mlwe_out", "com"]}
        args = [np.ascontiguousarray(rnd.last_row, np.uint64), np.ascontiguousarray(rnd.mask, np.uint64)]
        en = np.ascontiguousarray(rnd.enc_noise, np.int64)
        mn = np.ascontiguousarray(rnd.mlwe_noise, np.int64)
        check(lib().rg_jindo_commit(self.h, ptr(v), v.shape[0], ptr(args[0]), ptr(args[1]), iptr(en), iptr(mn),
                                    ptr(o["incom"]), ptr(o["enc"]), ptr(o["mlwe_out"]), ptr(o["com"])))
        return Commitment(o["com"]), Opening(o["incom"], o["enc"], o["mlwe_out"])

    def commit_key_dev(self):
        """Device addresses of the handle's commit key (ck_in, ck_mlwe, ck_out)."""
        a, b, c = vp(), vp(), vp()
        check(lib().rg_jindo_commit_key_dev(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    def commit_dev(self, batch, v, nv, last_row, mask, enc_noise, mlwe_noise, incom, enc, mlwe, com, stream=None):
        """rg_jindo_commit_dev on device buffers (tensors or int addresses)."""
        sh = self.params.shapes(batch)
        w = {k: _words(x) for k, x in sh.items()}
        L = self.params.L
        check(lib().rg_jindo_commit_dev(self.h, batch, _addr(v, batch * nv * L), nv, _addr(last_row, w["last_row"]),
                                        _addr(mask, w["mask"]), _addr(enc_noise, w["enc_noise"]),
                                        _addr(mlwe_noise, w["mlwe_noise"]), _addr(incom, w["incom"]),
                                        _addr(enc, w["enc"]), _addr(mlwe, w["mlwe_out"]), _addr(com, w["com"]),
                                        _stream(stream)))

    def delta_inv(self):
        """Encoder.deltaInv (encoder.go:50-67) as the library computes it."""
        out = (ctypes.c_double * self.params.exp)()
        check(lib().rg_jindo_delta_inv(self.h, out))
        return list(out)

    def sample_dev(self, batch, v, nv, seeds, first_commit, last_row, mask, enc_noise, mlwe_noise, stream=None):
        """rg_jindo_sample_dev: the randomness Commit draws, on the device (layouts of commit_dev)."""
        sh = self.params.shapes(batch)
        sc = seeds.c_struct()
        check(lib().rg_jindo_sample_dev(self.h, batch, _addr(v, batch * nv * self.params.L), nv, ctypes.byref(sc),
                                        first_commit, _addr(last_row, _words(sh["last_row"])),
                                        _addr(mask, _words(sh["mask"])), _addr(enc_noise, _words(sh["enc_noise"])),
                                        _addr(mlwe_noise, _words(sh["mlwe_noise"])), _stream(stream)))

    def commit_sampled_dev(self, batch, v, nv, seeds, first_commit, incom, enc, mlwe, com, stream=None):
        """Prover.Commit end to end on the device: sampling + commit (rg_jindo_commit_sampled_dev)."""
        sh = self.params.shapes(batch)
        sc = seeds.c_struct()
        check(lib().rg_jindo_commit_sampled_dev(self.h, batch, _addr(v, batch * nv * self.params.L), nv,
                                                ctypes.byref(sc), first_commit, _addr(incom, _words(sh["incom"])),
                                                _addr(enc, _words(sh["enc"])), _addr(mlwe, _words(sh["mlwe_out"])),
                                                _addr(com, _words(sh["com"])), _stream(stream)))

    MAC_KINDS = {0: "generic", 1: "valu3", 2: "mfma"}  # include/ringo.h RG_MAC_*

    def mac_kinds(self):
        """(inner, outer): which kernel runs each Ajtai product of this handle."""
        a, b = ctypes.c_int(), ctypes.c_int()
        check(lib().rg_jindo_mac_kinds(self.h, ctypes.byref(a), ctypes.byref(b)))
        return self.MAC_KINDS[a.value], self.MAC_KINDS[b.value]

    def release_stream(self, stream=None):
        """Drop the scratch the handle caches for `stream` (rg_jindo_release_stream)."""
        check(lib().rg_jindo_release_stream(self.h, _stream(stream)))

    def commit_core(self, enc, mlwe):
        """The Ajtai core of Commit (prover.go:144-202) from NTT-domain Opening.Encode / MLWE:
        returns (Commitment.Value, Opening.InCommit)."""
        sh = self.params.shapes()
        enc = np.ascontiguousarray(enc, np.uint64)
        mlwe = np.ascontiguousarray(mlwe, np.uint64)
        if enc.shape != sh["enc"] or mlwe.shape != sh["mlwe_out"]:
            raise RingoPanic("inconsistent input(s)")
        incom, com = np.zeros(sh["incom"], np.uint64), np.zeros(sh["com"], np.uint64)
        check(lib().rg_jindo_commit_core(self.h, ptr(enc), ptr(mlwe), ptr(incom), ptr(com)))
        return com, incom

    def commit_core_dev(self, batch, enc, mlwe, incom, com, stream=None):
        sh = self.params.shapes(batch)
        check(lib().rg_jindo_commit_core_dev(self.h, batch, _addr(enc, _words(sh["enc"])),
                                             _addr(mlwe, _words(sh["mlwe_out"])), _addr(incom, _words(sh["incom"])),
                                             _addr(com, _words(sh["com"])), _stream(stream)))


    # ---- Prover.Evaluate (jindo/prover.go:205-324), device-resident, challenges injected ----
    # The Fiat-Shamir transcript, encodeChallengeTo, leftVec/encode and Poly.Evaluate stay with
    # the caller (Go in the reference); these are its MulCoeffsMontgomeryThenAdd loops.
    def eval_shapes(self):
        P = self.params
        nm = P.in_msis + P.mlwe
        return dict(ob_incom=(P.dcmp, P.nqo, P.d), ob_enc=(P.cols + 1, P.rows, P.nq, P.d),
                    ob_mlwe=(P.cols + 1, nm, P.nq, P.d), partial=(P.cols + 1, P.nq, P.d),
                    pf_enc=(P.rows, P.nq, P.d), pf_mlwe=(nm, P.nq, P.d))

    def eval_batch_dev(self, batch, incom, enc, mlwe, bq, bo, ob_incom, ob_enc, ob_mlwe, stream=None):
        """openBatch = sum_i open[i] * batch[i] (prover.go:228-269); Proof.InCommit = ob_incom.
        bq = bo = None (params.batch == 1): openBatch = open[0]."""
        P, sh, es = self.params, self.params.shapes(batch), self.eval_shapes()
        w = lambda k: _words(sh[k])
        check(lib().rg_jindo_eval_batch_dev(self.h, batch, _addr(incom, w("incom")), _addr(enc, w("enc")),
                                            _addr(mlwe, w("mlwe_out")), _addr(bq, batch * P.nq * P.d),
                                            _addr(bo, batch * P.nqo * P.d), _addr(ob_incom, _words(es["ob_incom"])),
                                            _addr(ob_enc, _words(es["ob_enc"])), _addr(ob_mlwe, _words(es["ob_mlwe"])),
                                            _stream(stream)))

    def eval_reduce_dev(self, ob_incom, ob_enc, ob_mlwe, stream=None):
        """Words mod q in place (after summing partial openBatches across GPUs)."""
        es = self.eval_shapes()
        check(lib().rg_jindo_eval_reduce_dev(self.h, _addr(ob_incom, _words(es["ob_incom"])),
                                             _addr(ob_enc, _words(es["ob_enc"])), _addr(ob_mlwe, _words(es["ob_mlwe"])),
                                             _stream(stream)))

    def eval_partial_dev(self, ob_enc, left, partial, stream=None):
        """Proof.Partial[0..cols) and PartialMask (= partial[cols]) (prover.go:274-282)."""
        P, es = self.params, self.eval_shapes()
        check(lib().rg_jindo_eval_partial_dev(self.h, _addr(ob_enc, _words(es["ob_enc"])),
                                              _addr(left, P.rows * P.nq * P.d), _addr(partial, _words(es["partial"])),
                                              _stream(stream)))

    def eval_respond_dev(self, ob_enc, ob_mlwe, chals, pf_enc, pf_mlwe, stream=None):
        """Proof.Encode and Proof.MLWE (prover.go:300-314)."""
        P, es = self.params, self.eval_shapes()
        check(lib().rg_jindo_eval_respond_dev(self.h, _addr(ob_enc, _words(es["ob_enc"])),
                                              _addr(ob_mlwe, _words(es["ob_mlwe"])), _addr(chals, P.cols * P.nq * P.d),
                                              _addr(pf_enc, _words(es["pf_enc"])), _addr(pf_mlwe, _words(es["pf_mlwe"])),
                                              _stream(stream)))


class VerifyResultC(ctypes.Structure):  # include/ringo.h rg_jindo_verify_result
    _fields_ = [("outer_norm_sq", ctypes.c_uint64 * 10), ("inner_norm_sq", ctypes.c_uint64 * 10),
                ("outer_ok", ctypes.c_int), ("inner_ok", ctypes.c_int), ("consistency_ok", ctypes.c_int),
                ("eval_ok", ctypes.c_int), ("eval_lhs", ctypes.c_uint64 * 16), ("eval_rhs", ctypes.c_uint64 * 16),
                ("ok", ctypes.c_int)]


@dataclass
class VerifyResult:
    ok: bool
    outer_ok: bool
    inner_ok: bool
    consistency_ok: bool
    eval_ok: bool
    outer_norm_sq: int
    inner_norm_sq: int
    eval_lhs: np.ndarray
    eval_rhs: np.ndarray


class Verifier:
    """NewVerifier (verifier.go:25-47): the commit key from the CRS and the rings' tables, on the
    device (the same deterministic state a Prover handle holds)."""

    def __init__(self, params, crs=None, ck=None):
        self.params = params
        self._p = Prover(params, crs=crs, ck=ck)
        self.h = self._p.h

    def verify_dev(self, batch, com, bq, bo, chals, left, right, y, pf_incom, pf_partial, pf_enc, pf_mlwe,
                   stream=None):
        """Verify(x, com, y, pf) (verifier.go:50-133) on device buffers, challenges injected
        (include/ringo.h rg_jindo_verify_dev); bq = bo = None when params.batch == 1."""
        P = self.params
        if P.res_two_nm is None or P.in_com_dcmp_two_nm is None:
            raise RingoPanic("Parameters lack the two-norm bounds")
        r = VerifyResultC()
        nm, pq = P.in_msis + P.mlwe, P.nq * P.d
        check(lib().rg_jindo_verify_dev(self.h, batch, _addr(com, batch * P.out_msis * pq), _addr(bq, batch * pq),
                                        _addr(bo, batch * P.nqo * P.d), _addr(chals, P.cols * pq),
                                        _addr(left, P.rows * pq), _addr(right, P.cols * P.slots * P.L),
                                        _addr(y, batch * P.L), _addr(pf_incom, P.dcmp * P.nqo * P.d),
                                        _addr(pf_partial, (P.cols + 1) * pq), _addr(pf_enc, P.rows * pq),
                                        _addr(pf_mlwe, nm * pq), float(P.in_com_dcmp_two_nm), float(P.res_two_nm),
                                        ctypes.byref(r), _stream(stream)))
        word = lambda w: sum(int(x) << (64 * i) for i, x in enumerate(w))
        L = P.L
        return VerifyResult(bool(r.ok), bool(r.outer_ok), bool(r.inner_ok), bool(r.consistency_ok), bool(r.eval_ok),
                            word(r.outer_norm_sq), word(r.inner_norm_sq), np.array(r.eval_lhs[:L], np.uint64),
                            np.array(r.eval_rhs[:L], np.uint64))

    def Verify(self, batch, com, bq, bo, chals, left, right, y, pf_incom, pf_partial, pf_enc, pf_mlwe):
        """Host arrays (numpy) in the verify_dev layouts: staged to the device, then verify_dev."""
        import torch
        if len(com) != batch or len(y) != batch:  # verifier.go:51-54
            raise RingoPanic("len(v) != params.batch")
        dev = torch.device("cuda", torch.cuda.current_device())
        t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)
        args = [t(a) for a in (com, bq, bo, chals, left, right, y, pf_incom, pf_partial, pf_enc, pf_mlwe)]
        return self.verify_dev(batch, *args)


def NewVerifier(params, crs):
    return Verifier(params, crs=crs)


def uniform_words_dev(seed, instance, first_word, n, out, stream=None):
    """UniformSampler.Sample() words [first_word, first_word + n) of instance `instance` of
    NewUniformSamplerWithSeed(seed) into the device buffer `out` (rg_uniform_words_dev)."""
    check(lib().rg_uniform_words_dev(bytes(seed), len(seed), instance, first_word, n, _addr(out, n), _stream(stream)))


def NewProver(params, crs):
    return Prover(params, crs=crs)
