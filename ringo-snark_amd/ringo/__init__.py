"""ringo -- Python mirror of ringo-snark's hot-path interface over libringo (HIP, gfx950).

Mirrors the reference's Go surface (math/bigpoly, jindo) with the same names, argument
meaning and panics (raised as RingoPanic with the reference's message), so the parity tests
read like the reference's own tests:

    F   = Field(q)                                   # bignum.Uint[E]
    ev  = NewCyclotomicEvaluator(F, rank)            # bigpoly/cyclotomic.go:15
    p   = ev.NewPoly(False); ev.NTTTo(p, p)          # base_op.go:181
    prv = jindo.NewProver(params, crs)               # jindo/prover.go:28
    com, open_ = prv.Commit(v, randomness)          # prover.go:45 (randomness injected)
"""
from ._lib import RingoError, lib  # noqa: F401
from .bigpoly import (CyclicTransformer, CyclotomicTransformer, Field, NewCyclicEvaluator,  # noqa: F401
                      NewCyclicTransformer, NewCyclotomicEvaluator, NewCyclotomicTransformer, Poly,
                      RingoPanic)
from . import buckler, jindo  # noqa: F401
