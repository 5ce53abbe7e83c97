"""GPU parity: the remaining bigpoly operators (rg_poly_*: QuoRemByVanishing cyclic.go:18-37,
AutTo cyclotomic.go:29-86, Poly.Evaluate poly.go:64-76, ModSwitchTo cyclotomic.go:97-124) vs the C
oracle (ModSwitch: vs pyref.mod_switch's big-integer restatement), bit-exact, through the
Python mirror of the reference's evaluators (host entry points) and the batched device forms."""
import numpy as np
import pytest

import coracle as co
import ringo
from ringo.bigpoly import RingoPanic

pytestmark = pytest.mark.gpu


def _rand(F, n, rng):
    return F.random(n, rng).reshape(n, F.L)


@pytest.mark.parametrize("key", ["p63", "mult_zp", "jindo_zp", "zp440"])
@pytest.mark.parametrize("rank,N", [(1 << 12, 1 << 11), (1 << 12, 1000), (1 << 12, 1), (1 << 12, 0),
                                    (1 << 12, 1 << 12), (1 << 12, 5000), (1 << 16, 1 << 15)])
def test_quorem_vanishing(fields, key, rank, N):
    q = fields[key]
    F = ringo.Field(q)
    cf = co.CField(q)
    ev = ringo.NewCyclicEvaluator(F, rank)
    p = ev.NewPoly(False)
    p.Coeffs[...] = _rand(F, rank, np.random.default_rng(N))
    quo, rem = ev.QuoRemByVanishing(p, N)
    wq, wr = cf.quorem_vanishing(p.Coeffs, N)
    assert (quo.Coeffs == wq).all() and (rem.Coeffs == wr).all()


def test_quorem_panics(fields):
    F = ringo.Field(fields["p63"])
    ev = ringo.NewCyclicEvaluator(F, 64)
    with pytest.raises(RingoPanic, match="input in NTT domain"):
        ev.QuoRemByVanishing(ev.NewPoly(True), 8)
    with pytest.raises(RingoPanic, match="inputs not consistent"):
        ev.QuoRemByVanishing(ringo.NewCyclicEvaluator(F, 32).NewPoly(False), 8)


@pytest.mark.parametrize("key", ["p63", "mult_zp", "jindo_zp"])
@pytest.mark.parametrize("idx", [1, 3, 5, 2 * (1 << 12) - 1, -7, 3 * 2 * (1 << 12) + 9, 12345])
@pytest.mark.parametrize("ntt", [False, True])
def test_aut(fields, key, idx, ntt):
    q = fields[key]
    F = ringo.Field(q)
    cf = co.CField(q)
    rank = 1 << 12
    ev = ringo.NewCyclotomicEvaluator(F, rank)
    p = ev.NewPoly(ntt)
    p.Coeffs[...] = _rand(F, rank, np.random.default_rng(idx & 0xffff))
    out = ev.Aut(p, idx)
    assert out.IsNTT == ntt
    assert (out.Coeffs == cf.aut(p.Coeffs, idx, ntt)).all()
    ev.AutTo(p, p, idx)  # aliasing, as the reference allows through its pooled buffer
    assert (p.Coeffs == out.Coeffs).all()


def test_aut_even_index_panics(fields):
    F = ringo.Field(fields["p63"])
    ev = ringo.NewCyclotomicEvaluator(F, 64)
    with pytest.raises(RingoPanic, match="AutTo: idx must be odd"):
        ev.Aut(ev.NewPoly(False), 4)


@pytest.mark.parametrize("key", ["p63", "mult_zp", "jindo_zp", "zp880"])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 4097, 1 << 16])
def test_evaluate(fields, key, n):
    q = fields[key]
    F = ringo.Field(q)
    cf = co.CField(q)
    rng = np.random.default_rng(n)
    p = ringo.Poly(F, n, False, _rand(F, n, rng))
    x = _rand(F, 1, rng)[0]
    assert (p.Evaluate(x) == cf.evaluate(p.Coeffs, x)).all()


def test_batched_device_forms(fields):
    import torch
    from ringo._lib import lib, check
    q = fields["jindo_zp"]
    F = ringo.Field(q)
    cf = co.CField(q)
    rank, B, N, idx = 1 << 12, 5, 1 << 10, 7
    rng = np.random.default_rng(1)
    host = _rand(F, B * rank, rng).reshape(B, rank, F.L)
    dev = torch.device("cuda")
    d = torch.from_numpy(host.view(np.int64).copy()).to(dev)
    quo, rem, aut = torch.empty_like(d), torch.empty_like(d), torch.empty_like(d)
    check(lib().rg_poly_quorem_vanishing_dev(F.h, rank, N, quo.data_ptr(), rem.data_ptr(), d.data_ptr(), B, None))
    check(lib().rg_poly_aut_dev(F.h, rank, idx, 1, aut.data_ptr(), d.data_ptr(), B, None))
    torch.cuda.synchronize()
    for b in range(B):
        wq, wr = cf.quorem_vanishing(host[b], N)
        assert (quo[b].cpu().numpy().view(np.uint64) == wq).all()
        assert (rem[b].cpu().numpy().view(np.uint64) == wr).all()
        assert (aut[b].cpu().numpy().view(np.uint64) == cf.aut(host[b], idx, True)).all()
    # rem may alias p
    check(lib().rg_poly_quorem_vanishing_dev(F.h, rank, N, quo.data_ptr(), d.data_ptr(), d.data_ptr(), B, None))
    torch.cuda.synchronize()
    assert torch.equal(d, rem)


@pytest.mark.parametrize("key", ["p63", "mult_zp", "bfv_zp", "jindo_zp", "zp440", "zp880"])
@pytest.mark.parametrize("qbits", [2, 62, 64, 130, 255, 300, 509])
def test_mod_switch(fields, key, qbits):
    """CyclotomicEvaluator.ModSwitch on centred inputs (the bfv example's PolyToBigintCentered,
    examples/bfv/main.go:152-155), the range ends, exact ties and values beyond qBig."""
    import pyref
    q = fields[key]
    F = ringo.Field(q)
    rank = 1 << 10
    rng = np.random.default_rng(qbits)
    qbig = (int.from_bytes(rng.bytes(64), "little") % (1 << qbits)) | (1 << (qbits - 1)) | (qbits & 1)
    ps = [int.from_bytes(rng.bytes(72), "little") % qbig - (qbig >> 1) for _ in range(rank)]
    edge = [0, 1, -1, qbig - 1, -(qbig - 1), qbig >> 1, -(qbig >> 1), (qbig + 1) >> 1, -((qbig + 1) >> 1),
            3 * qbig + 5, -(3 * qbig) - 1]
    ps[:len(edge)] = edge
    ev = ringo.NewCyclotomicEvaluator(F, rank)
    out = ev.ModSwitch(ps, qbig)
    assert not out.IsNTT
    rinv = pow(1 << (64 * F.L), -1, q)
    got = [x * rinv % q for x in co.from_limbs(out.Coeffs)]
    assert got == pyref.mod_switch(ps, qbig, q)


def test_mod_switch_panics(fields):
    F = ringo.Field(fields["p63"])
    ev = ringo.NewCyclotomicEvaluator(F, 64)
    with pytest.raises(RingoPanic, match="input size not consistent"):
        ev.ModSwitch([1] * 63, 97)
