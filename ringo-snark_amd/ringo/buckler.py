"""buckler mirror: the Buckler prover's per-witness device work over
libringo -- the Encoder (buckler/encoder.go) and ArithmeticConstraint / Prover.evalCircuit
(buckler/constraint.go, buckler/prover.go:355-379).  Same names and argument meaning as the
reference; MustSetRandom draws are injected (`rand=`), as everywhere in this library.

    enc = NewEncoder(F, rank, embRank)                 # newEncoder (encoder.go:15-20)
    p = enc.RandEncode(w, rand=r)                      # RandEncode (encoder.go:42-54)
    c = ArithmeticConstraint(F); c.AddTerm(None, a, b) # constraint.go:15-53
    out = EvalCircuit(F, batchConst, [c], wEcdNTT, pwEcdNTT)   # prover.go:355-379
"""
import ctypes

import numpy as np

from ._lib import check, lib, ptr, vp
from .bigpoly import NewCyclicTransformer, Poly, RingoPanic, _addr, _stream


class Encoder:
    """Encoder[E] (buckler/encoder.go:9-12): a CyclicTransformer at the witness rank and the
    embedding rank of the output polynomials."""

    def __init__(self, field, rank, embed_rank):
        self.field = field
        self.ntt = NewCyclicTransformer(field, rank)
        self.embedRank = embed_rank

    def Encode(self, v):  # encoder.go:24-28
        pOut = Poly(self.field, self.embedRank, False)
        self.EncodeTo(pOut, v)
        return pOut

    def EncodeTo(self, pOut, v):  # encoder.go:32-38
        self._encode(pOut, v, None)

    def RandEncode(self, v, rand):  # encoder.go:42-46
        pOut = Poly(self.field, self.embedRank, False)
        self.RandEncodeTo(pOut, v, rand)
        return pOut

    def RandEncodeTo(self, pOut, v, rand):  # encoder.go:50-54; rand = the MustSetRandom draw
        self._encode(pOut, v, rand)

    def _encode(self, pOut, v, rand):
        L, rank = self.field.L, self.ntt.Rank()
        v = np.ascontiguousarray(np.asarray(v, np.uint64).reshape(-1, L)[:rank])  # v[:e.ntt.Rank()]
        if v.shape[0] < rank:
            raise RingoPanic("index out of range")  # Go slices past len(v)
        if pOut.Rank() < rank + (1 if rand is not None else 0):
            raise RingoPanic("index out of range")
        r = None if rand is None else np.ascontiguousarray(np.asarray(rand, np.uint64).reshape(L))
        out = np.zeros((pOut.Rank(), L), np.uint64)
        check(lib().rg_buckler_encode(self.ntt.h, pOut.Rank(), ptr(out), ptr(v), ptr(r)))
        pOut.Coeffs[...] = out
        pOut.IsNTT = False

    def encode_dev(self, d_out, d_v, batch, d_rand=None, d_scratch=None, stream=None):
        """rg_buckler_encode_dev: `batch` witnesses [batch][rank][L] -> [batch][embedRank][L]."""
        L, rank = self.field.L, self.ntt.Rank()
        sw = self.scratch_bytes(batch) // 8
        check(lib().rg_buckler_encode_dev(self.ntt.h, self.embedRank, _addr(d_out, batch * self.embedRank * L),
                                          _addr(d_v, batch * rank * L), batch,
                                          _addr(d_rand, batch * L) if d_rand is not None else None,
                                          _addr(d_scratch, sw) if d_scratch is not None else None, _stream(stream)))

    def scratch_bytes(self, batch):
        return lib().rg_buckler_encode_scratch_bytes(self.ntt.h, batch)


def NewEncoder(field, rank, embed_rank):
    return Encoder(field, rank, embed_rank)


class ArithmeticConstraint:
    """ArithmeticConstraint[E] (constraint.go:6-12).  Witnesses and public witnesses are given by
    their witnessToID numbers; coefficients are Montgomery elements ([L] words)."""

    def __init__(self, field):
        self.field = field
        self.coeffs, self.hasCoeffPublicWitness, self.coeffsPublicWitness, self.witness = [], [], [], []
        self.wRank = 0

    def _const(self, v):
        return np.asarray(self.field.mont([v % self.field.q]), np.uint64).reshape(self.field.L)

    def AddTerm(self, coeffPublicWitness, *witness):  # constraint.go:15-21
        self.AddTermWithConst(self._const(1), coeffPublicWitness, *witness)

    def SubTerm(self, coeffPublicWitness, *witness):  # constraint.go:23-29
        self.AddTermWithConst(self._const(-1), coeffPublicWitness, *witness)

    def AddTermWithConst(self, coeff, coeffPublicWitness, *witness):  # constraint.go:31-53
        self.coeffs.append(np.asarray(coeff, np.uint64).reshape(self.field.L))
        self.hasCoeffPublicWitness.append(coeffPublicWitness is not None)
        self.coeffsPublicWitness.append(0 if coeffPublicWitness is None else int(coeffPublicWitness))
        self.witness.append([int(w) for w in witness])
        self.wRank = max(self.wRank, len(witness))

    def maxRank(self, rank):  # constraint.go:56-70
        maxDeg = 0
        for i, ws in enumerate(self.witness):
            deg = (rank - 1 if self.hasCoeffPublicWitness[i] else 0) + len(ws) * rank
            maxDeg = max(maxDeg, deg)
        return maxDeg + 1


class Circuit:
    """A set of constraints uploaded once (rg_buckler_circuit_create): the program evalCircuit walks."""

    def __init__(self, field, constraints):
        self.field = field
        L = field.L
        term_off, coeffs, pw, wit_off, wit = [0], [], [], [0], []
        for c in constraints:
            for i in range(len(c.coeffs)):
                coeffs.append(c.coeffs[i])
                pw.append(c.coeffsPublicWitness[i] if c.hasCoeffPublicWitness[i] else -1)
                wit.extend(c.witness[i])
                wit_off.append(len(wit))
            term_off.append(len(pw))
        self.n_w = 1 + max(wit, default=-1)
        self.n_pw = 1 + max(pw, default=-1)
        sz = ctypes.c_size_t
        to = (sz * len(term_off))(*term_off)
        wo = (sz * len(wit_off))(*wit_off)
        wi = (ctypes.c_uint64 * max(1, len(wit)))(*wit)
        pi = (ctypes.c_longlong * max(1, len(pw)))(*pw)
        cf = np.ascontiguousarray(np.array(coeffs, np.uint64).reshape(-1, L) if coeffs else np.zeros((1, L), np.uint64))
        h = vp()
        st = lib().rg_buckler_circuit_create(field.h, len(constraints), to, ptr(cf), pi, wo, wi, ctypes.byref(h))
        if st == -1:
            raise RingoPanic("inconsistent input(s)")
        check(st)
        self.h = h
        self._L = lib()

    def __del__(self):
        if getattr(self, "h", None) and getattr(self, "_L", None):  # the CDLL bound at creation
            self._L.rg_buckler_circuit_destroy(self.h)  # (module globals may already be gone at interpreter exit)
            self.h = None

    def eval_dev(self, rank, d_batch_const, d_w, n_w, d_pw, n_pw, d_out, stream=None):
        """rg_buckler_eval_circuit_dev (device-resident wEcdNTT [n_w][rank][L], pwEcdNTT [n_pw][rank][L])."""
        L = self.field.L
        check(lib().rg_buckler_eval_circuit_dev(self.h, rank, _addr(d_batch_const, L),
                                                _addr(d_w, n_w * rank * L) if n_w else None, n_w,
                                                _addr(d_pw, n_pw * rank * L) if n_pw else None, n_pw,
                                                _addr(d_out, rank * L), _stream(stream)))


def EvalCircuit(field, batchConst, constraints, wEcdNTT, pwEcdNTT):
    """Prover.evalCircuit (prover.go:355-379): wEcdNTT / pwEcdNTT are lists of NTT-domain Polys
    (or [n][rank][L] arrays); returns the NTT-domain Poly."""
    L = field.L
    circ = Circuit(field, constraints)

    def stack(ps):
        if ps is None or len(ps) == 0:
            return None, 0
        if isinstance(ps, np.ndarray):
            return np.ascontiguousarray(ps, np.uint64), ps.shape[0]
        for p in ps:
            if not p.IsNTT:
                raise RingoPanic("input not in NTT domain")  # base_op.go:133-142 MulTo
        return np.ascontiguousarray(np.stack([p.Coeffs for p in ps]), np.uint64), len(ps)

    w, n_w = stack(wEcdNTT)
    pw, n_pw = stack(pwEcdNTT)
    rank = (w if w is not None else pw).shape[-2] if (w is not None or pw is not None) else 0
    if n_w < circ.n_w or n_pw < circ.n_pw:
        raise RingoPanic("index out of range")
    out = Poly(field, rank, True)
    bc = np.ascontiguousarray(np.asarray(batchConst, np.uint64).reshape(L))
    res = np.zeros((rank, L), np.uint64)
    check(lib().rg_buckler_eval_circuit(circ.h, rank, ptr(bc), ptr(w), n_w, ptr(pw), n_pw, ptr(res)))
    out.Coeffs[...] = res
    return out
