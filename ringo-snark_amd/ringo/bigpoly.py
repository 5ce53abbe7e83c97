"""bigpoly mirror (math/bigpoly) over libringo.

Host-side objects hold numpy uint64 arrays laid out like a contiguous []zp.Uint: [N][L] limbs
of Montgomery-form elements.  Every arithmetic call goes through the C ABI (include/ringo.h);
the shape/domain checks that Go performs before computing stay here with the reference's panic
messages (math/bigpoly/poly.go:106-121, base_op.go:133-205, ntt.go:27-37,154-164).

Device-resident entry points (`*_dev`) accept anything exposing `data_ptr()` (torch tensors)
or raw integer addresses, plus an optional HIP stream handle.
"""
import ctypes

import numpy as np

from ._lib import check, lib, ptr, vp


class RingoPanic(Exception):
    """Raised where the Go reference panics; str(e) is the reference's message."""


_WORD_DTYPES = ("torch.int64", "torch.uint64")


def _addr(x, words=None):
    """Device address of a buffer of 64-bit words.  Tensors must be contiguous, of a 64-bit
    integer dtype, on the current GPU and (when `words` is given) hold at least that many
    words; anything else raises RingoPanic instead of letting the kernel read a strided view,
    another GPU's memory or past the end.  Raw int addresses are taken as they are."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if not hasattr(x, "data_ptr"):
        raise TypeError("device buffer must be a tensor or an int address")
    if str(x.dtype) not in _WORD_DTYPES:
        raise RingoPanic(f"device buffer dtype {x.dtype}: need 64-bit words (int64/uint64)")
    if not x.is_contiguous():
        raise RingoPanic("device buffer is not contiguous")
    if x.device.type != "cuda":
        raise RingoPanic(f"device buffer on {x.device}, need the GPU")
    import torch
    if x.device.index != torch.cuda.current_device():
        raise RingoPanic(f"device buffer on {x.device}, current device is cuda:{torch.cuda.current_device()}")
    if words is not None and x.numel() < words:
        raise RingoPanic(f"device buffer holds {x.numel()} words, need {words}")
    return x.data_ptr()


def _stream(s):
    if s is None:
        return None
    if isinstance(s, int):
        return s
    return getattr(s, "cuda_stream", s)


class Field:
    """The element type E (math/bignum/bignum.go:8-31): modulus q, L = ceil(bits/64) limbs,
    Montgomery R = 2^(64L)."""

    def __init__(self, q, limbs=None):
        self.q = int(q)
        self.L = limbs or (self.q.bit_length() + 63) // 64
        ql = np.array([(self.q >> (64 * i)) & ((1 << 64) - 1) for i in range(self.L)], dtype=np.uint64)
        h = vp()
        st = lib().rg_field_create(self.L, ptr(ql), ctypes.byref(h))
        if st != 0:
            raise RingoPanic("invalid modulus")
        self.h = h
        self._L = lib()

    def __del__(self):
        if getattr(self, "h", None) and getattr(self, "_L", None):  # the CDLL bound at creation
            self._L.rg_field_destroy(self.h)  # (module globals may already be gone at interpreter exit)
            self.h = None

    def constants(self):
        qinv = ctypes.c_uint64()
        r2 = np.zeros(self.L, np.uint64)
        one = np.zeros(self.L, np.uint64)
        check(lib().rg_field_constants(self.h, ctypes.byref(qinv), ptr(r2), ptr(one)))
        return qinv.value, r2, one

    # conversions (host only; used to build inputs) -----------------------------------------
    def to_limbs(self, values):
        values = list(values)
        out = np.zeros((len(values), self.L), np.uint64)
        m = (1 << 64) - 1
        for i, v in enumerate(values):
            for j in range(self.L):
                out[i, j] = (int(v) >> (64 * j)) & m
        return out

    def from_limbs(self, arr):
        a = np.asarray(arr, np.uint64).reshape(-1, self.L)
        return [sum(int(a[i, j]) << (64 * j) for j in range(self.L)) for i in range(a.shape[0])]

    def mont(self, values):
        """plain integers -> Montgomery limbs (SetBigInt)"""
        R = 1 << (64 * self.L)
        return self.to_limbs([(int(v) % self.q) * R % self.q for v in values])

    def unmont(self, arr):
        Rinv = pow(1 << (64 * self.L), -1, self.q)
        return [v * Rinv % self.q for v in self.from_limbs(arr)]

    def random(self, n, rng):
        """n uniform Montgomery-form elements (MustSetRandom analogue, seeded)"""
        words = rng.integers(0, 2 ** 63, size=(n, self.L), dtype=np.int64).astype(np.uint64) * 2
        words += rng.integers(0, 2, size=(n, self.L), dtype=np.int64).astype(np.uint64)
        vals = [v % self.q for v in self.from_limbs(words)]
        return self.to_limbs(vals)


class _Transformer:
    negacyclic = None

    def __init__(self, field, rank, tables=None):
        if rank <= 0 or rank & (rank - 1):
            raise RingoPanic("rank must be a power of two")  # ntt.go:27-29,154-156
        self.field = field
        self.rank = rank
        h = vp()
        if tables is None:
            st = lib().rg_ntt_create(field.h, rank, 1 if self.negacyclic else 0, ctypes.byref(h))
        else:
            tw, twi, ninv = (np.ascontiguousarray(t, np.uint64) for t in tables)
            st = lib().rg_ntt_create_from_tables(field.h, rank, 1 if self.negacyclic else 0, ptr(tw), ptr(twi),
                                                 ptr(ninv), ctypes.byref(h))
        if st == -3:
            raise RingoPanic("NTT not supported")  # ntt.go:35-37,162-164
        check(st)
        self.h = h
        self._L = lib()

    def __del__(self):
        if getattr(self, "h", None) and getattr(self, "_L", None):  # the CDLL bound at creation
            self._L.rg_ntt_destroy(self.h)  # (module globals may already be gone at interpreter exit)
            self.h = None

    def Rank(self):
        return self.rank

    def tables(self):
        L = self.field.L
        tw = np.zeros((self.rank, L), np.uint64)
        twi = np.zeros((self.rank, L), np.uint64)
        ninv = np.zeros(L, np.uint64)
        check(lib().rg_ntt_tables(self.h, ptr(tw), ptr(twi), ptr(ninv)))
        return tw, twi, ninv

    def _host(self, fn, vOut, v):
        v = np.ascontiguousarray(v, np.uint64)
        if v.size % (self.rank * self.field.L):
            raise RingoPanic("inconsistent input(s)")
        batch = v.size // (self.rank * self.field.L)
        out = vOut if (vOut is not None and vOut.flags.c_contiguous and vOut.dtype == np.uint64) else np.empty_like(v)
        check(fn(self.h, ptr(out), ptr(v), batch))
        if vOut is not None and out is not vOut:
            vOut[...] = out
        return out

    def FwdNTTTo(self, vOut, v):
        """FwdNTTTo (ntt.go:98-115 / 206-223); v, vOut: [..., rank, L]; batched if leading dims."""
        return self._host(lib().rg_ntt_fwd, vOut, v)

    def InvNTTTo(self, vOut, v):
        """InvNTTTo (ntt.go:118-136 / 226-244)."""
        return self._host(lib().rg_ntt_inv, vOut, v)

    def fwd_dev(self, d_out, d_in, batch, stream=None):
        w = batch * self.rank * self.field.L
        check(lib().rg_ntt_fwd_dev(self.h, _addr(d_out, w), _addr(d_in, w), batch, _stream(stream)))

    def inv_dev(self, d_out, d_in, batch, stream=None):
        w = batch * self.rank * self.field.L
        check(lib().rg_ntt_inv_dev(self.h, _addr(d_out, w), _addr(d_in, w), batch, _stream(stream)))


class CyclotomicTransformer(_Transformer):
    """Negacyclic NTT over Z_q[X]/(X^N+1) (ntt.go:143-203)."""
    negacyclic = True


class CyclicTransformer(_Transformer):
    """Cyclic NTT over Z_q[X]/(X^N-1) (ntt.go:16-95)."""
    negacyclic = False


def NewCyclotomicTransformer(field, rank):
    return CyclotomicTransformer(field, rank)


def NewCyclicTransformer(field, rank):
    return CyclicTransformer(field, rank)


class Poly:
    """Poly[E] (poly.go:11-14): Coeffs [rank][L] Montgomery limbs + IsNTT flag."""

    def __init__(self, field, rank, is_ntt=False, coeffs=None):
        self.field = field
        self.Coeffs = np.zeros((rank, field.L), np.uint64) if coeffs is None else np.ascontiguousarray(coeffs, np.uint64)
        self.IsNTT = is_ntt

    def Rank(self):
        return self.Coeffs.shape[0]

    def CopyFrom(self, p0):  # poly.go:44-61
        self.Coeffs[...] = p0.Coeffs
        self.IsNTT = p0.IsNTT

    def Clear(self):
        self.Coeffs[...] = 0

    def Evaluate(self, x):  # poly.go:64-76
        """p(x) for x one element ([L] Montgomery limbs); rg_poly_evaluate."""
        if self.IsNTT:
            raise RingoPanic("Evaluate: p is in NTT form")
        out = np.zeros(self.field.L, np.uint64)
        xx = np.ascontiguousarray(x, np.uint64).reshape(self.field.L)
        check(lib().rg_poly_evaluate(self.field.h, ptr(self.Coeffs), self.Rank(), ptr(xx), ptr(out)))
        return out


_OPS = {"add": 0, "sub": 1, "neg": 2, "mul": 3, "smul": 4, "mul_add": 5, "mul_sub": 6, "smul_add": 7, "smul_sub": 8}


class _BaseOperator:
    """baseOperator (base_op.go:10-207)."""

    def __init__(self, field, rank, ntt):
        self.field = field
        self.rank = rank
        self.ntt = ntt

    def NewPoly(self, is_ntt):
        return Poly(self.field, self.rank, is_ntt)

    def Rank(self):
        return self.rank

    # checks (poly.go:106-121) --------------------------------------------------------------
    def _unary(self, pOut, p):
        if pOut.Rank() != self.rank or p.Rank() != self.rank:
            raise RingoPanic("inconsistent input(s)")

    def _binary(self, pOut, p0, p1):
        if pOut.Rank() != self.rank or p0.Rank() != self.rank or p1.Rank() != self.rank:
            raise RingoPanic("inconsistent input(s)")
        if p0.IsNTT != p1.IsNTT:
            raise RingoPanic("inconsistent input(s)")

    def _vec(self, op, pOut, a, b):
        n = self.rank
        check(lib().rg_vec(self.field.h, _OPS[op], ptr(pOut.Coeffs), ptr(a), ptr(b), n))

    # ops -----------------------------------------------------------------------------------
    def AddTo(self, pOut, p0, p1):  # base_op.go:49-55
        self._binary(pOut, p0, p1)
        self._vec("add", pOut, p0.Coeffs, p1.Coeffs)
        pOut.IsNTT = p0.IsNTT

    def SubTo(self, pOut, p0, p1):  # base_op.go:64-70
        self._binary(pOut, p0, p1)
        self._vec("sub", pOut, p0.Coeffs, p1.Coeffs)
        pOut.IsNTT = p0.IsNTT

    def NegTo(self, pOut, p):  # base_op.go:79-85
        self._unary(pOut, p)
        self._vec("neg", pOut, p.Coeffs, None)
        pOut.IsNTT = p.IsNTT

    def ScalarMulTo(self, pOut, p, c):  # base_op.go:94-100
        self._unary(pOut, p)
        self._vec("smul", pOut, p.Coeffs, np.ascontiguousarray(c, np.uint64).reshape(-1))
        pOut.IsNTT = p.IsNTT

    def ScalarMulAddTo(self, pOut, p, c):  # base_op.go:102-112
        self._unary(pOut, p)
        self._vec("smul_add", pOut, p.Coeffs, np.ascontiguousarray(c, np.uint64).reshape(-1))
        pOut.IsNTT = p.IsNTT

    def ScalarMulSubTo(self, pOut, p, c):  # base_op.go:114-124
        self._unary(pOut, p)
        self._vec("smul_sub", pOut, p.Coeffs, np.ascontiguousarray(c, np.uint64).reshape(-1))
        pOut.IsNTT = p.IsNTT

    def _mul_check(self, pOut, p0, p1):
        self._binary(pOut, p0, p1)
        if not p0.IsNTT or not p1.IsNTT:
            raise RingoPanic("input(s) not in NTT domain")  # base_op.go:135-137

    def MulTo(self, pOut, p0, p1):  # base_op.go:133-142
        self._mul_check(pOut, p0, p1)
        self._vec("mul", pOut, p0.Coeffs, p1.Coeffs)
        pOut.IsNTT = True

    def MulAddTo(self, pOut, p0, p1):  # base_op.go:144-157
        self._mul_check(pOut, p0, p1)
        self._vec("mul_add", pOut, p0.Coeffs, p1.Coeffs)
        pOut.IsNTT = True

    def MulSubTo(self, pOut, p0, p1):  # base_op.go:159-172
        self._mul_check(pOut, p0, p1)
        self._vec("mul_sub", pOut, p0.Coeffs, p1.Coeffs)
        pOut.IsNTT = True

    def NTTTo(self, pOut, p):  # base_op.go:181-190
        self._unary(pOut, p)
        if p.IsNTT:
            raise RingoPanic("input already in NTT domain")
        self.ntt.FwdNTTTo(pOut.Coeffs, p.Coeffs)
        pOut.IsNTT = True

    def InvNTTTo(self, pOut, p):  # base_op.go:199-207
        self._unary(pOut, p)
        if not p.IsNTT:
            raise RingoPanic("input not in NTT domain")
        self.ntt.InvNTTTo(pOut.Coeffs, p.Coeffs)
        pOut.IsNTT = False

    # allocating forms (base_op.go:42-197)
    def Add(self, p0, p1):
        o = self.NewPoly(p0.IsNTT)
        self.AddTo(o, p0, p1)
        return o

    def Sub(self, p0, p1):
        o = self.NewPoly(p0.IsNTT)
        self.SubTo(o, p0, p1)
        return o

    def Neg(self, p):
        o = self.NewPoly(p.IsNTT)
        self.NegTo(o, p)
        return o

    def ScalarMul(self, p, c):
        o = self.NewPoly(p.IsNTT)
        self.ScalarMulTo(o, p, c)
        return o

    def Mul(self, p0, p1):
        o = self.NewPoly(True)
        self.MulTo(o, p0, p1)
        return o

    def NTT(self, p):
        o = self.NewPoly(True)
        self.NTTTo(o, p)
        return o

    def InvNTT(self, p):
        o = self.NewPoly(False)
        self.InvNTTTo(o, p)
        return o


class CyclotomicEvaluator(_BaseOperator):
    """NewCyclotomicEvaluator (cyclotomic.go:15-20)."""

    def Aut(self, p, idx):  # cyclotomic.go:22-27
        o = self.NewPoly(p.IsNTT)
        self.AutTo(o, p, idx)
        return o

    def AutTo(self, pOut, p, idx):  # cyclotomic.go:29-47 (autTo / autNTTTo)
        self._unary(pOut, p)
        if idx % 2 == 0:
            raise RingoPanic("AutTo: idx must be odd")
        src = p.Coeffs.copy() if pOut is p else p.Coeffs  # the reference works through a pooled buffer
        check(lib().rg_poly_aut(self.field.h, self.rank, int(idx), 1 if p.IsNTT else 0, ptr(pOut.Coeffs), ptr(src)))
        pOut.IsNTT = p.IsNTT


    def ModSwitch(self, pBig, qBig):  # cyclotomic.go:91-96
        o = self.NewPoly(False)
        self.ModSwitchTo(o, pBig, qBig)
        return o

    def ModSwitchTo(self, pOut, pBig, qBig):  # cyclotomic.go:98-124
        """pBig: rank Python ints (any sign, e.g. PolyToBigintCentered output), qBig > 0: each
        coefficient to round(p q / qBig) mod q (rg_poly_modswitch), pOut in the coefficient domain."""
        if len(pBig) != self.rank:
            raise RingoPanic("input size not consistent")
        qBig = int(qBig)
        if qBig <= 0:
            raise RingoPanic("qBig must be positive")
        bits = max([qBig.bit_length()] + [abs(int(x)).bit_length() for x in pBig]) + 1  # + sign bit
        w = (bits + 63) // 64
        if w > 8:
            raise RingoPanic("ModSwitch: operands wider than 511 bits are not supported")
        mask = (1 << (64 * w)) - 1
        words = np.array([[((int(x) & mask) >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(w)] for x in pBig],
                         dtype=np.uint64).reshape(self.rank, w)
        qw = np.array([(qBig >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(w)], dtype=np.uint64)
        check(lib().rg_poly_modswitch(self.field.h, self.rank, ptr(words), w, ptr(qw), ptr(pOut.Coeffs)))
        pOut.IsNTT = False


class CyclicEvaluator(_BaseOperator):
    """NewCyclicEvaluator (cyclic.go:11-16)."""

    def QuoRemByVanishing(self, p, N):  # cyclic.go:18-37
        if p.Rank() != self.rank:
            raise RingoPanic("inputs not consistent")
        if p.IsNTT:
            raise RingoPanic("input in NTT domain")
        if N < 0:
            raise RingoPanic("index out of range")  # Go: quo.Coeffs[i-N] with N < 0
        quo, rem = self.NewPoly(False), self.NewPoly(False)
        check(lib().rg_poly_quorem_vanishing(self.field.h, self.rank, int(N), ptr(quo.Coeffs), ptr(rem.Coeffs),
                                             ptr(p.Coeffs)))
        return quo, rem


def NewCyclotomicEvaluator(field, rank):
    return CyclotomicEvaluator(field, rank, CyclotomicTransformer(field, rank))


def NewCyclicEvaluator(field, rank):
    return CyclicEvaluator(field, rank, CyclicTransformer(field, rank))


def vec_dev(field, op, d_out, d_a, d_b, n, stream=None):
    """rg_vec_dev: device-resident pointwise op over n elements."""
    w = n * field.L
    wb = None if op == "neg" else (field.L if op.startswith("smul") else w)
    check(lib().rg_vec_dev(field.h, _OPS[op], _addr(d_out, w), _addr(d_a, w), _addr(d_b, wb), n, _stream(stream)))
