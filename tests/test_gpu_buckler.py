"""GPU parity: the Buckler prover's device work (rg_buckler_*: Encoder.EncodeTo / RandEncodeTo
buckler/encoder.go:32-54, Prover.evalCircuit buckler/prover.go:355-379) vs the C oracle,
bit-exact, through the Python mirror (host entry points) and the batched device forms."""
import numpy as np
import pytest

import coracle as co
import ringo
from ringo import buckler
from ringo.bigpoly import RingoPanic

pytestmark = pytest.mark.gpu


def _rand(F, n, rng):
    return F.random(n, rng).reshape(n, F.L)


@pytest.mark.parametrize("key", ["p63", "mult_zp", "jindo_zp", "zp440"])
@pytest.mark.parametrize("rank,emb", [(1 << 12, 1 << 13), (1 << 10, (1 << 10) + 1), (1 << 14, 1 << 16), (8, 16),
                                      (1 << 15, 1 << 16)])
def test_encode_matches_oracle(fields, key, rank, emb):
    q = fields[key]
    F = ringo.Field(q)
    cf = co.CField(q)
    rng = np.random.default_rng(rank + emb)
    enc = buckler.NewEncoder(F, rank, emb)
    v = _rand(F, rank, rng)
    p = enc.Encode(v)
    assert not p.IsNTT and p.Rank() == emb
    assert (p.Coeffs == cf.buckler_encode(v, emb)).all()
    r = _rand(F, 1, rng)[0]
    pr = enc.RandEncode(v, rand=r)
    assert (pr.Coeffs == cf.buckler_encode(v, emb, rnd=r)).all()


@pytest.mark.parametrize("key", ["p63", "mult_zp", "jindo_zp"])
@pytest.mark.parametrize("batch", [1, 3, 16])
def test_encode_dev_batch(fields, key, batch):
    import torch
    q = fields[key]
    F = ringo.Field(q)
    cf = co.CField(q)
    L = F.L
    rank, emb = 1 << 12, 1 << 13
    rng = np.random.default_rng(batch)
    enc = buckler.NewEncoder(F, rank, emb)
    v = _rand(F, batch * rank, rng).reshape(batch, rank, L)
    r = _rand(F, batch, rng)
    dv = torch.from_numpy(v.view(np.int64)).cuda()
    dr = torch.from_numpy(r.view(np.int64)).cuda()
    dout = torch.full((batch, emb, L), -1, dtype=torch.int64, device="cuda")
    scr = torch.empty(max(1, enc.scratch_bytes(batch) // 8), dtype=torch.int64, device="cuda")
    for rand in (None, dr):
        enc.encode_dev(dout, dv, batch, d_rand=rand, d_scratch=scr)
        torch.cuda.synchronize()
        got = dout.cpu().numpy().view(np.uint64)
        for b in range(batch):
            want = cf.buckler_encode(v[b], emb, rnd=None if rand is None else r[b])
            assert (got[b] == want).all(), b


def test_encode_dev_batch_q255_split(fields):
    """The witness rank at the Jindo default prime with a batch of 9: the batched cyclic InvNTT at
    rank 2^15 runs as two halves (4 + 5 polynomials) on the caller's stream and the plan's helper
    stream (ntt_l4_fast.hip run_split).  Witnesses 0, 4 (the first half's last) and 8 against the
    oracle, with and without the random coefficient."""
    import torch
    q = fields["jindo_zp"]
    F = ringo.Field(q)
    cf = co.CField(q)
    L = F.L
    rank, emb, batch = 1 << 15, 1 << 16, 9
    rng = np.random.default_rng(915)
    enc = buckler.NewEncoder(F, rank, emb)
    v = _rand(F, batch * rank, rng).reshape(batch, rank, L)
    r = _rand(F, batch, rng)
    dv = torch.from_numpy(v.view(np.int64)).cuda()
    dr = torch.from_numpy(r.view(np.int64)).cuda()
    dout = torch.full((batch, emb, L), -1, dtype=torch.int64, device="cuda")
    scr = torch.empty(max(1, enc.scratch_bytes(batch) // 8), dtype=torch.int64, device="cuda")
    for rand in (None, dr):
        enc.encode_dev(dout, dv, batch, d_rand=rand, d_scratch=scr)
        torch.cuda.synchronize()
        got = dout.cpu().numpy().view(np.uint64)
        for b in (0, 4, 8):
            want = cf.buckler_encode(v[b], emb, rnd=None if rand is None else r[b])
            assert (got[b] == want).all(), b


def test_encode_panics(fields):
    F = ringo.Field(fields["p63"])
    enc = buckler.NewEncoder(F, 64, 64)
    enc.Encode(_rand(F, 64, np.random.default_rng(0)))  # EncodeTo fills all 64 coefficients
    with pytest.raises(RingoPanic):  # RandEncode writes Coeffs[rank]: index out of range
        enc.RandEncode(_rand(F, 64, np.random.default_rng(0)), rand=_rand(F, 1, np.random.default_rng(1))[0])
    # a negacyclic plan is not an Encoder's transformer
    T = ringo.NewCyclotomicTransformer(F, 64)
    out = np.zeros((128, 1), np.uint64)
    v = np.zeros((64, 1), np.uint64)
    assert ringo.lib().rg_buckler_encode(T.h, 128, out.ctypes.data_as(ringo._lib.u64p),
                                         v.ctypes.data_as(ringo._lib.u64p), None) == -1


def _circuit(F, rng, nw, npw):
    c0 = buckler.ArithmeticConstraint(F)
    c0.AddTerm(None, 0, 1)      # a * b
    c0.SubTerm(None, 2)         # - c
    c1 = buckler.ArithmeticConstraint(F)
    c1.AddTermWithConst(_rand(F, 1, rng)[0], 1 % npw, 3, 0)  # k * pw * d * a
    c1.AddTerm(0, 2, 2, 2)      # pw0 * c^3
    c1.AddTermWithConst(_rand(F, 1, rng)[0], None)  # a constant term
    c2 = buckler.ArithmeticConstraint(F)                  # no terms
    c3 = buckler.ArithmeticConstraint(F)
    c3.AddTerm(None, nw - 1)
    return [c0, c1, c2, c3]


def _oracle_cons(cons):
    return [[(c.coeffs[i], c.coeffsPublicWitness[i] if c.hasCoeffPublicWitness[i] else None, c.witness[i])
             for i in range(len(c.coeffs))] for c in cons]


@pytest.mark.parametrize("key", ["p63", "mult_zp", "jindo_zp", "zp440"])
@pytest.mark.parametrize("rank", [1 << 6, 1 << 13, 1000])
def test_eval_circuit_matches_oracle(fields, key, rank):
    q = fields[key]
    F = ringo.Field(q)
    cf = co.CField(q)
    L = F.L
    rng = np.random.default_rng(rank)
    nw, npw = 5, 2
    cons = _circuit(F, rng, nw, npw)
    w = [ringo.Poly(F, rank, True, _rand(F, rank, rng)) for _ in range(nw)]
    pw = [ringo.Poly(F, rank, True, _rand(F, rank, rng)) for _ in range(npw)]
    bc = _rand(F, 1, rng)[0]
    got = buckler.EvalCircuit(F, bc, cons, w, pw)
    assert got.IsNTT
    want = cf.buckler_eval_circuit(_oracle_cons(cons), bc, np.stack([p.Coeffs for p in w]),
                                   np.stack([p.Coeffs for p in pw]))
    assert (got.Coeffs == want).all()
    # device form on the same data
    import torch
    circ = buckler.Circuit(F, cons)
    dw = torch.from_numpy(np.stack([p.Coeffs for p in w]).view(np.int64)).cuda()
    dpw = torch.from_numpy(np.stack([p.Coeffs for p in pw]).view(np.int64)).cuda()
    dbc = torch.from_numpy(bc.view(np.int64).copy()).cuda()
    dout = torch.zeros((rank, L), dtype=torch.int64, device="cuda")
    circ.eval_dev(rank, dbc, dw, nw, dpw, npw, dout)
    torch.cuda.synchronize()
    assert (dout.cpu().numpy().view(np.uint64) == want).all()


def test_eval_circuit_index_checks(fields):
    F = ringo.Field(fields["p63"])
    rng = np.random.default_rng(0)
    cons = _circuit(F, rng, 5, 2)
    w = [ringo.Poly(F, 64, True, _rand(F, 64, rng)) for _ in range(4)]  # witness 4 missing
    pw = [ringo.Poly(F, 64, True, _rand(F, 64, rng)) for _ in range(2)]
    with pytest.raises(RingoPanic):
        buckler.EvalCircuit(F, _rand(F, 1, rng)[0], cons, w, pw)
    c = buckler.ArithmeticConstraint(F)
    c.AddTermWithConst(np.array([F.q], np.uint64), None, 0)  # coefficient not reduced
    with pytest.raises(RingoPanic):
        buckler.Circuit(F, [c])


def test_witness_pipeline_end_to_end(fields):
    """The prover's per-witness flow (prover.go:147-150, 355-379): RandEncode every witness,
    NTT at embRank (CyclicEvaluator), evalCircuit -- all on the device -- vs the oracle chain."""
    import torch
    q = fields["mult_zp"]
    F = ringo.Field(q)
    cf = co.CField(q)
    L = F.L
    rank, emb, nw = 1 << 12, 1 << 13, 3
    rng = np.random.default_rng(5)
    enc = buckler.NewEncoder(F, rank, emb)
    T = ringo.NewCyclicTransformer(F, emb)
    v = _rand(F, nw * rank, rng).reshape(nw, rank, L)
    r = _rand(F, nw, rng)
    dv = torch.from_numpy(v.view(np.int64)).cuda()
    dr = torch.from_numpy(r.view(np.int64)).cuda()
    decd = torch.empty((nw, emb, L), dtype=torch.int64, device="cuda")
    scr = torch.empty(enc.scratch_bytes(nw) // 8, dtype=torch.int64, device="cuda")
    enc.encode_dev(decd, dv, nw, d_rand=dr, d_scratch=scr)
    T.fwd_dev(decd, decd, nw)
    c = buckler.ArithmeticConstraint(F)
    c.AddTerm(None, 0, 1)
    c.SubTerm(None, 2)
    circ = buckler.Circuit(F, [c])
    bc = _rand(F, 1, rng)[0]
    dbc = torch.from_numpy(bc.view(np.int64).copy()).cuda()
    dout = torch.empty((emb, L), dtype=torch.int64, device="cuda")
    circ.eval_dev(emb, dbc, decd, nw, None, 0, dout)
    torch.cuda.synchronize()
    tw, _, _ = cf.tables(emb, cyclic=True)
    wn = np.stack([cf.ntt_fwd(cf.buckler_encode(v[i], emb, rnd=r[i])[None], tw)[0] for i in range(nw)])
    assert (decd.cpu().numpy().view(np.uint64) == wn).all()
    want = cf.buckler_eval_circuit(_oracle_cons([c]), bc, wn, None)
    assert (dout.cpu().numpy().view(np.uint64) == want).all()
