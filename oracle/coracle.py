"""ctypes binding of oracle/liboracle.so (the C restatement).  TEST INFRASTRUCTURE ONLY:
imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the
product path (ringo-snark_amd/)."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

u64p = ctypes.POINTER(ctypes.c_uint64)
i64p = ctypes.POINTER(ctypes.c_int64)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liboracle.so not built (run `make -C oracle`)")
        _LIB = ctypes.CDLL(path)
        L = _LIB
        L.of_field_size.restype = ctypes.c_size_t
        L.of_primitive_root.restype = ctypes.c_uint64
        L.of_primitive_root.argtypes = [ctypes.c_uint64]
        L.of_lattigo_psi.restype = ctypes.c_uint64
        L.of_lattigo_psi.argtypes = [ctypes.c_uint64, ctypes.c_int]
        L.of_jindo_create.restype = ctypes.c_void_p
        L.of_jindo_create.argtypes = [ctypes.c_void_p]
        L.of_jindo_destroy.argtypes = [ctypes.c_void_p]
        L.of_ntt_fwd.argtypes = [ctypes.c_void_p, u64p, u64p, u64p, ctypes.c_int, ctypes.c_long]
        L.of_ntt_inv.argtypes = [ctypes.c_void_p, u64p, u64p, u64p, u64p, ctypes.c_int, ctypes.c_long]
        L.of_vec.argtypes = [ctypes.c_void_p, ctypes.c_int, u64p, u64p, u64p, ctypes.c_long]
        L.of_quorem_vanishing.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_long, u64p, u64p, u64p]
        L.of_aut.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_long, ctypes.c_int, u64p, u64p]
        L.of_poly_evaluate.argtypes = [ctypes.c_void_p, u64p, ctypes.c_long, u64p, u64p]
        L.of_buckler_encode.argtypes = [ctypes.c_void_p, u64p, u64p, ctypes.c_int, ctypes.c_long, u64p, u64p, u64p]
        lp = ctypes.POINTER(ctypes.c_long)
        L.of_buckler_eval_circuit.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_long, lp, u64p, lp, lp, lp,
                                              u64p, u64p, u64p, u64p]
        L.of_jindo_eval_batch.argtypes = [ctypes.c_void_p, ctypes.c_long] + [u64p] * 8
        L.of_jindo_eval_partial.argtypes = [ctypes.c_void_p, u64p, u64p, u64p]
        L.of_jindo_eval_respond.argtypes = [ctypes.c_void_p] + [u64p] * 5
        L.of_jindo_commit_core.argtypes = [ctypes.c_void_p] + [u64p] * 7
        L.of_jindo_sample.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                      ctypes.c_char_p, ctypes.c_uint64, ctypes.c_long, u64p, ctypes.c_long, u64p, u64p,
                                      i64p, i64p]
        L.of_uniform_words.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_long,
                                       u64p]
        L.of_sampler_draws.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_double, ctypes.c_double, ctypes.c_long,
                                       ctypes.c_long, ctypes.POINTER(ctypes.c_int64)]
        L.of_sampler_draws.restype = ctypes.c_int
        L.of_jindo_verify.restype = ctypes.c_int
        L.of_jindo_verify.argtypes = ([ctypes.c_void_p] + [u64p] * 3 + [ctypes.c_long] + [u64p] * 11 +
                                      [ctypes.c_double, ctypes.c_double, u64p, ctypes.POINTER(ctypes.c_int), u64p])
        L.of_jindo_encode_challenge.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, u64p]
        L.of_jindo_encode.argtypes = [ctypes.c_void_p, u64p, ctypes.c_int, u64p]
        L.of_norm_below.restype = ctypes.c_int
        L.of_norm_below.argtypes = [u64p, ctypes.c_double]
    return _LIB


def ptr(a, t=u64p):
    return a.ctypes.data_as(t) if a is not None else None


def to_limbs(values, L):
    """list of ints -> np.uint64 [n, L] little-endian limbs"""
    out = np.zeros((len(values), L), dtype=np.uint64)
    m = (1 << 64) - 1
    for i, v in enumerate(values):
        for j in range(L):
            out[i, j] = (v >> (64 * j)) & m
    return out


def from_limbs(arr):
    arr = np.asarray(arr, dtype=np.uint64).reshape(-1, arr.shape[-1])
    L = arr.shape[1]
    return [sum(int(arr[i, j]) << (64 * j) for j in range(L)) for i in range(arr.shape[0])]


class CField:
    def __init__(self, q, L=None):
        self.q = q
        self.L = L or (q.bit_length() + 63) // 64
        self.buf = ctypes.create_string_buffer(lib().of_field_size())
        ql = to_limbs([q], self.L)[0]
        rc = lib().of_field_init(self.buf, self.L, ptr(ql))
        if rc:
            raise ValueError("bad field")

    def consts(self):
        qinv = ctypes.c_uint64()
        r2 = np.zeros(self.L, np.uint64)
        one = np.zeros(self.L, np.uint64)
        lib().of_field_consts(self.buf, ctypes.byref(qinv), ptr(r2), ptr(one))
        return qinv.value, from_limbs(r2[None, :])[0], from_limbs(one[None, :])[0]

    def _bin(self, fn, x, y=None):
        z = np.zeros(self.L, np.uint64)
        xa = to_limbs([x], self.L)[0]
        if y is None:
            getattr(lib(), fn)(self.buf, ptr(z), ptr(xa))
        else:
            ya = to_limbs([y], self.L)[0]
            getattr(lib(), fn)(self.buf, ptr(z), ptr(xa), ptr(ya))
        return from_limbs(z[None, :])[0]

    def mul(self, x, y):
        return self._bin("of_f_mul", x, y)

    def add(self, x, y):
        return self._bin("of_f_add", x, y)

    def sub(self, x, y):
        return self._bin("of_f_sub", x, y)

    def neg(self, x):
        return self._bin("of_f_neg", x)

    # ---- bigpoly operators (cyclic.go:18-37, cyclotomic.go:29-86, poly.go:64-76) ----
    def quorem_vanishing(self, p, N):
        p = np.ascontiguousarray(p, np.uint64)
        quo, rem = np.zeros_like(p), np.zeros_like(p)
        lib().of_quorem_vanishing(self.buf, p.shape[0], N, ptr(quo), ptr(rem), ptr(p))
        return quo, rem

    def aut(self, p, idx, ntt):
        p = np.ascontiguousarray(p, np.uint64)
        out = np.zeros_like(p)
        lib().of_aut(self.buf, p.shape[0], idx, 1 if ntt else 0, ptr(out), ptr(p))
        return out

    def evaluate(self, p, x):
        p = np.ascontiguousarray(p, np.uint64)
        xx = np.ascontiguousarray(x, np.uint64).reshape(self.L)
        out = np.zeros(self.L, np.uint64)
        lib().of_poly_evaluate(self.buf, ptr(p), p.shape[0], ptr(xx), ptr(out))
        return out

    # ---- buckler prover (buckler/encoder.go:32-54, buckler/prover.go:355-379) ----
    def buckler_encode(self, v, emb, rnd=None):
        """Encoder.EncodeTo / RandEncodeTo of v [rank, L] into a new [emb, L] array."""
        v = np.ascontiguousarray(v, np.uint64)
        rank = v.shape[0]
        _, twi, ninv = self.tables(rank, cyclic=True)
        out = np.zeros((emb, self.L), np.uint64)
        r = None if rnd is None else np.ascontiguousarray(rnd, np.uint64).reshape(self.L)
        lib().of_buckler_encode(self.buf, ptr(twi), ptr(ninv), rank, emb, ptr(out), ptr(v), ptr(r))
        return out

    def buckler_eval_circuit(self, constraints, batch_const, w, pw):
        """constraints: list of constraints, each a list of terms (coeff [L] Montgomery words,
        public-witness index or None, [witness indices]); w, pw: [n, rank, L]."""
        lp = ctypes.POINTER(ctypes.c_long)
        term_off, coeffs, pw_idx, wit_off, wit_idx = [0], [], [], [0], []
        for c in constraints:
            for coeff, p, ws in c:
                coeffs.append(np.asarray(coeff, np.uint64).reshape(self.L))
                pw_idx.append(-1 if p is None else p)
                wit_idx.extend(ws)
                wit_off.append(len(wit_idx))
            term_off.append(len(pw_idx))
        arr = lambda x: np.ascontiguousarray(np.array(x, dtype=np.int64))  # noqa: E731
        to, pi, wo, wi = arr(term_off), arr(pw_idx), arr(wit_off), arr(wit_idx + [0])
        cf = np.ascontiguousarray(np.array(coeffs, np.uint64).reshape(-1, self.L)) if coeffs else \
            np.zeros((1, self.L), np.uint64)
        w = np.ascontiguousarray(w, np.uint64)
        rank = w.shape[-2]
        pwa = np.ascontiguousarray(pw if pw is not None and len(pw) else np.zeros((1, rank, self.L)), np.uint64)
        out = np.zeros((rank, self.L), np.uint64)
        bc = np.ascontiguousarray(batch_const, np.uint64).reshape(self.L)
        lib().of_buckler_eval_circuit(self.buf, rank, len(constraints), ptr(to, lp), ptr(cf), ptr(pi, lp),
                                      ptr(wo, lp), ptr(wi, lp), ptr(bc), ptr(w), ptr(pwa), ptr(out))
        return out

    def tables(self, N, cyclic=False):
        """(tw [N,L], twinv [N,L], ninv [L]) as np.uint64 (Montgomery), or raises."""
        tw = np.zeros((N, self.L), np.uint64)
        twi = np.zeros((N, self.L), np.uint64)
        ninv = np.zeros(self.L, np.uint64)
        fn = lib().of_cyclic_tables if cyclic else lib().of_cyclotomic_tables
        rc = fn(self.buf, N, ptr(tw), ptr(twi), ptr(ninv))
        if rc == -1:
            raise ValueError("rank must be a power of two")
        if rc:
            raise ValueError("NTT not supported")
        return tw, twi, ninv

    def ntt_fwd(self, a, tw):
        """a: np.uint64 [batch, N, L] -> new array"""
        a = np.ascontiguousarray(a, dtype=np.uint64)
        out = np.empty_like(a)
        lib().of_ntt_fwd(self.buf, ptr(out), ptr(a), ptr(np.ascontiguousarray(tw)), a.shape[-2],
                         a.size // (a.shape[-2] * self.L))
        return out

    def ntt_inv(self, a, twi, ninv):
        a = np.ascontiguousarray(a, dtype=np.uint64)
        out = np.empty_like(a)
        lib().of_ntt_inv(self.buf, ptr(out), ptr(a), ptr(np.ascontiguousarray(twi)), ptr(np.ascontiguousarray(ninv)),
                         a.shape[-2], a.size // (a.shape[-2] * self.L))
        return out

    VEC_OPS = {"add": 0, "sub": 1, "neg": 2, "mul": 3, "smul": 4, "mul_add": 5, "mul_sub": 6,
               "smul_add": 7, "smul_sub": 8}

    def vec(self, op, out, a, b=None):
        """in-place on `out` (np.uint64 [n, L]); matches rg_vec semantics."""
        n = out.size // self.L
        lib().of_vec(self.buf, self.VEC_OPS[op], ptr(out), ptr(a), ptr(b), n)
        return out


class OfJindoParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ["rank", "rows", "cols", "slots", "exp", "d", "in_msis", "out_msis", "mlwe", "dcmp",
                 "log_in_cut", "log_out_cut"]] + [
        ("base", ctypes.c_uint64), ("nq", ctypes.c_int), ("nqo", ctypes.c_int),
        ("q", ctypes.c_uint64 * 4), ("qo", ctypes.c_uint64 * 4), ("field_limbs", ctypes.c_int),
        ("field_q", ctypes.c_uint64 * 16)]


def make_params_struct(P, field_q, cls=OfJindoParams):
    s = cls()
    for k, a in [("rank", "rank"), ("rows", "rows"), ("cols", "cols"), ("slots", "slots"), ("exp", "exp"),
                 ("d", "d"), ("in_msis", "in_msis"), ("out_msis", "out_msis"), ("mlwe", "mlwe"),
                 ("dcmp", "in_com_dcmp_len"), ("log_in_cut", "log_in_cut"), ("log_out_cut", "log_out_cut")]:
        setattr(s, k, int(P[a] if isinstance(P, dict) else getattr(P, a)))
    g = (lambda k: P[k]) if isinstance(P, dict) else (lambda k: getattr(P, k))
    s.base = g("base")
    q, qo = list(g("q")), list(g("qo"))
    s.nq, s.nqo = len(q), len(qo)
    for i, x in enumerate(q):
        s.q[i] = x
    for i, x in enumerate(qo):
        s.qo[i] = x
    L = (field_q.bit_length() + 63) // 64
    s.field_limbs = L
    for i in range(L):
        s.field_q[i] = (field_q >> (64 * i)) & ((1 << 64) - 1)
    return s


class CJindo:
    """C-oracle commit with injected randomness (same layouts as rg_jindo_commit)."""

    def __init__(self, P, field_q):
        self.P = P
        self.ps = make_params_struct(P, field_q)
        self.h = lib().of_jindo_create(ctypes.byref(self.ps))
        if not self.h:
            raise ValueError("bad jindo params")
        self.L = self.ps.field_limbs

    def __del__(self):
        if getattr(self, "h", None):
            lib().of_jindo_destroy(self.h)
            self.h = None

    def shapes(self):
        s = self.ps
        nm = s.in_msis + s.mlwe
        return dict(incom=(s.dcmp, s.nqo, s.d), enc=(s.cols + 1, s.rows, s.nq, s.d),
                    mlwe=(s.cols + 1, nm, s.nq, s.d), com=(s.out_msis, s.nq, s.d))

    def commit(self, ck_in, ck_mlwe, ck_out, v, last_row, mask, enc_noise, mlwe_noise):
        sh = self.shapes()
        o = {k: np.zeros(v_, np.uint64) for k, v_ in sh.items()}
        args = [np.ascontiguousarray(x) for x in (ck_in, ck_mlwe, ck_out, v, last_row, mask)]
        en = np.ascontiguousarray(enc_noise, dtype=np.int64)
        mn = np.ascontiguousarray(mlwe_noise, dtype=np.int64)
        rc = lib().of_jindo_commit(
            ctypes.c_void_p(self.h), ptr(args[0]), ptr(args[1]), ptr(args[2]), ptr(args[3]),
            ctypes.c_long(args[3].shape[0]), ptr(args[4]), ptr(args[5]), ptr(en, i64p), ptr(mn, i64p),
            ptr(o["incom"]), ptr(o["enc"]), ptr(o["mlwe"]), ptr(o["com"]))
        if rc:
            raise ValueError("len(v) > params.rank")
        return o

    def commit_core(self, ck_in, ck_mlwe, ck_out, enc, mlwe):
        """The Ajtai core of Commit (prover.go:144-202) from the NTT-domain Opening.Encode/MLWE."""
        sh = self.shapes()
        o = {k: np.zeros(sh[k], np.uint64) for k in ("incom", "com")}
        a = [np.ascontiguousarray(x, dtype=np.uint64) for x in (ck_in, ck_mlwe, ck_out, enc, mlwe)]
        lib().of_jindo_commit_core(ctypes.c_void_p(self.h), *[ptr(x) for x in a], ptr(o["incom"]), ptr(o["com"]))
        return o

    def sample(self, sd, delta, seeds, first, v):
        """The randomness of v.shape[0] commits (of_jindo_sample): sd = the six standard deviations
        (ecd, ecd_blind, mask, mask_blind, mlwe, mask_mlwe), delta = deltaInv, seeds = 192 bytes."""
        s = self.ps
        B, nv = v.shape[0], v.shape[1]
        nm = s.in_msis + s.mlwe
        o = dict(last_row=np.zeros((B, s.cols * s.slots, self.L), np.uint64),
                 mask=np.zeros((B, s.rows, s.slots, self.L), np.uint64),
                 enc_noise=np.zeros((B, s.cols + 1, s.rows, s.d), np.int64),
                 mlwe_noise=np.zeros((B, s.cols + 1, nm, s.d), np.int64))
        sdv = (ctypes.c_double * 6)(*sd)
        dv = (ctypes.c_double * len(delta))(*delta)
        vv = np.ascontiguousarray(v, np.uint64)
        rc = lib().of_jindo_sample(ctypes.c_void_p(self.h), sdv, dv, bytes(seeds), first, B, ptr(vv), nv,
                                   ptr(o["last_row"]), ptr(o["mask"]), ptr(o["enc_noise"], i64p),
                                   ptr(o["mlwe_noise"], i64p))
        if rc:
            raise RuntimeError("of_jindo_sample: libcrypto unavailable")
        return o

    # ---- Prover.Evaluate core (prover.go:205-324), challenges injected ----
    def eval_shapes(self):
        s = self.ps
        nm = s.in_msis + s.mlwe
        return dict(ob_incom=(s.dcmp, s.nqo, s.d), ob_enc=(s.cols + 1, s.rows, s.nq, s.d),
                    ob_mlwe=(s.cols + 1, nm, s.nq, s.d), partial=(s.cols + 1, s.nq, s.d),
                    pf_enc=(s.rows, s.nq, s.d), pf_mlwe=(nm, s.nq, s.d))

    def eval_batch(self, incom, enc, mlwe, bq, bo):
        """openBatch = sum_i open[i] * batch[i]; inputs carry a leading batch dimension."""
        sh = self.eval_shapes()
        o = {k: np.zeros(sh[k], np.uint64) for k in ("ob_incom", "ob_enc", "ob_mlwe")}
        a = [np.ascontiguousarray(x, dtype=np.uint64) for x in (incom, enc, mlwe, bq, bo)]
        lib().of_jindo_eval_batch(ctypes.c_void_p(self.h), ctypes.c_long(a[0].shape[0]), *[ptr(x) for x in a],
                                  ptr(o["ob_incom"]), ptr(o["ob_enc"]), ptr(o["ob_mlwe"]))
        return o

    def eval_partial(self, ob_enc, left):
        out = np.zeros(self.eval_shapes()["partial"], np.uint64)
        a = [np.ascontiguousarray(x, dtype=np.uint64) for x in (ob_enc, left)]
        lib().of_jindo_eval_partial(ctypes.c_void_p(self.h), ptr(a[0]), ptr(a[1]), ptr(out))
        return out

    def eval_respond(self, ob_enc, ob_mlwe, chals):
        sh = self.eval_shapes()
        pe, pm = np.zeros(sh["pf_enc"], np.uint64), np.zeros(sh["pf_mlwe"], np.uint64)
        a = [np.ascontiguousarray(x, dtype=np.uint64) for x in (ob_enc, ob_mlwe, chals)]
        lib().of_jindo_eval_respond(ctypes.c_void_p(self.h), ptr(a[0]), ptr(a[1]), ptr(a[2]), ptr(pe), ptr(pm))
        return pe, pm

    # ---- Verifier.Verify (verifier.go:50-282), challenges injected ----
    def verify(self, ck, batch, com, bq, bo, chals, left, right, y, pf_incom, pf_partial, pf_enc, pf_mlwe,
               in_com_dcmp_two_nm, res_two_nm):
        """Returns dict(ok, flags=[outer, inner, consistency, eval], outer_sq, inner_sq (ints),
        eval_lhs, eval_rhs (Montgomery limbs)).  bq/bo may be None when batch == 1."""
        res = np.zeros(20, np.uint64)
        flags = (ctypes.c_int * 4)()
        ev = np.zeros(2 * self.L, np.uint64)
        z = np.zeros(1, np.uint64)
        a = [np.ascontiguousarray(x, dtype=np.uint64) if x is not None else z
             for x in (ck[0], ck[1], ck[2], com, bq, bo, chals, left, right, y, pf_incom, pf_partial, pf_enc, pf_mlwe)]
        ok = lib().of_jindo_verify(ctypes.c_void_p(self.h), ptr(a[0]), ptr(a[1]), ptr(a[2]), ctypes.c_long(batch),
                                   *[ptr(x) for x in a[3:]], float(in_com_dcmp_two_nm), float(res_two_nm), ptr(res),
                                   flags, ptr(ev))
        word = lambda w: sum(int(x) << (64 * i) for i, x in enumerate(w))
        return dict(ok=bool(ok), flags=[bool(f) for f in flags], outer_sq=word(res[:10]), inner_sq=word(res[10:]),
                    eval_lhs=ev[:self.L].copy(), eval_rhs=ev[self.L:].copy())

    def encode_challenge(self, ring, b16):
        """encodeChallengeTo (utils.go:20-46) of 16 bytes into ringQ (ring 0) or ringQOut (1)."""
        s = self.ps
        out = np.zeros((s.nqo if ring else s.nq, s.d), np.uint64)
        lib().of_jindo_encode_challenge(ctypes.c_void_p(self.h), int(ring), bytes(b16), ptr(out))
        return out

    def encode(self, v):
        """Encoder.encode (encoder.go:105-117) of <= slots Montgomery elements [n][L]."""
        s = self.ps
        out = np.zeros((s.nq, s.d), np.uint64)
        vv = np.ascontiguousarray(v, dtype=np.uint64)
        lib().of_jindo_encode(ctypes.c_void_p(self.h), ptr(vv), int(vv.shape[0]), ptr(out))
        return out


def norm_below(S, nm):
    """oracle.c norm_below: Float64(isqrt(S)) < nm decided by S < K^2 (verifier.go:278-281)"""
    w = np.array([(S >> (64 * i)) & ((1 << 64) - 1) for i in range(10)], np.uint64)
    return bool(lib().of_norm_below(ptr(w), float(nm)))


def uniform_words(seed, inst, first, n):
    """UniformSampler.Sample() words [first, first + n) of instance `inst` (oracle.c)."""
    out = np.zeros(n, np.uint64)
    if lib().of_uniform_words(bytes(seed), len(seed), inst, first, n, ptr(out)):
        raise RuntimeError("libcrypto unavailable")
    return out


def sampler_draws(kind, seeds, sigma, center, n, per_inst=256):
    """n draws of one reference sampler (oracle.c of_sampler_draws): kind "twin_cdt", "cosac" or
    "rounded"; seeds = 64 bytes (the sampler's UniformSampler seed, then COSAC's rounded one)."""
    k = {"twin_cdt": 0, "cosac": 1, "rounded": 2}[kind]
    out = np.zeros(n, np.int64)
    if lib().of_sampler_draws(k, bytes(seeds), float(sigma), float(center), n, per_inst,
                              out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))):
        raise RuntimeError("libcrypto unavailable")
    return out
