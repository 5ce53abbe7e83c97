"""GPU parity: libringo's bigpoly NTT / vec ops vs the C oracle (oracle/oracle.c), bit-exact.

Mirrors what the reference exercises through bigpoly (math/bigpoly/ntt.go, vec.go,
base_op.go): every generated field of the reference, cyclic and negacyclic transformers,
ranks from 2 to 2^16 (the wide fields through ntt_wide_pass up to Buckler's 2^15 / 2^16),
batched, aliasing out == in."""
import numpy as np
import pytest

import coracle as co
import ringo

pytestmark = pytest.mark.gpu

CASES = [  # (field, logN list)
    ("p63", [3, 5, 6, 8, 10, 12, 13, 16]),
    ("jindo_zp", [3, 6, 8, 11, 12, 16]),
    ("zp110", [3, 8, 12, 13]),
    ("mult_zp", [4, 10]),
    ("zp220", [5, 9, 14]),
    ("bfv_zp", [8]),
    ("zp440", [1, 3, 8, 10, 11, 15, 16]),
    ("zp880", [2, 6, 9, 13, 15, 16]),
]


@pytest.mark.parametrize("name,logns", CASES)
@pytest.mark.parametrize("negacyclic", [True, False])
def test_ntt_matches_oracle(fields, name, logns, negacyclic):
    q = fields[name]
    F = ringo.Field(q)
    cf = co.CField(q)
    rng = np.random.default_rng(1234)
    for logn in logns:
        N = 1 << logn
        batch = 3 if logn <= 12 else 2
        T = (ringo.CyclotomicTransformer if negacyclic else ringo.CyclicTransformer)(F, N)
        tw, twi, ninv = T.tables()
        otw, otwi, oninv = cf.tables(N, cyclic=not negacyclic)
        assert (tw == otw).all() and (twi == otwi).all() and (ninv == oninv).all(), (name, logn)
        a = F.random(batch * N, rng).reshape(batch, N, F.L)
        want = cf.ntt_fwd(a, otw)
        got = T.FwdNTTTo(None, a)
        assert (got == want).all(), (name, logn, "fwd")
        back = T.InvNTTTo(None, got)
        assert (back == a).all(), (name, logn, "inv roundtrip")
        want_inv = cf.ntt_inv(a, otwi, oninv)  # inverse of arbitrary input
        got_inv = T.InvNTTTo(None, a)
        assert (got_inv == want_inv).all(), (name, logn, "inv")


@pytest.mark.parametrize("name", ["p63", "jindo_zp", "zp110", "mult_zp", "zp440", "zp880"])
def test_vec_ops_match_oracle(fields, name):
    q = fields[name]
    F = ringo.Field(q)
    cf = co.CField(q)
    rng = np.random.default_rng(7)
    n = 4099
    a = F.random(n, rng)
    b = F.random(n, rng)
    c = F.random(1, rng)
    a[:3] = 0  # edge values: 0, 1 (Montgomery R), q-1
    b[0] = F.mont([q - 1])[0]
    for op in ["add", "sub", "neg", "mul", "smul", "mul_add", "mul_sub", "smul_add", "smul_sub"]:
        base = F.random(n, rng)
        want = base.copy()
        got = base.copy()
        bb = c[0] if op.startswith("smul") else b
        cf.vec(op, want, a, np.ascontiguousarray(bb))
        ringo._lib.check(ringo.lib().rg_vec(F.h, ringo.bigpoly._OPS[op], ringo._lib.ptr(got), ringo._lib.ptr(a),
                                            ringo._lib.ptr(np.ascontiguousarray(bb)), n))
        assert (got == want).all(), (name, op)


@pytest.mark.parametrize("batch", [1, 3, 16, 17, 32])
def test_ntt_2e16_batches_match_oracle(fields, batch):
    """Degree 2^16 at the config-2 prime: the lazy two-pass kernels (ntt64.hpp) with both ROW
    tilings (16 rows of one poly, and the same row of 16 polys when batch % 16 == 0), in place
    and out of place, device-resident entry points, forward vs the C oracle and inverse."""
    import torch

    q = fields["p63"]
    N = 1 << 16
    F = ringo.Field(q)
    cf = co.CField(q)
    T = ringo.CyclotomicTransformer(F, N)
    tw, twi, ninv = cf.tables(N)
    rng = np.random.default_rng(batch)
    a = F.random(batch * N, rng).reshape(batch, N, 1)
    a[0, :4, 0] = [0, 1, q - 1, q - 2]  # edge residues
    want = cf.ntt_fwd(a, tw)
    dev = torch.device("cuda", 0)
    x = torch.from_numpy(a.view(np.int64).reshape(-1).copy()).to(dev)
    y = torch.empty_like(x)
    T.fwd_dev(y, x, batch)  # out of place
    torch.cuda.synchronize()
    assert (y.cpu().numpy().view(np.uint64).reshape(batch, N, 1) == want).all()
    assert torch.equal(x.cpu(), torch.from_numpy(a.view(np.int64).reshape(-1)))  # input untouched
    T.inv_dev(y, y, batch)  # in place
    torch.cuda.synchronize()
    assert (y.cpu().numpy().view(np.uint64).reshape(batch, N, 1) == a).all()
    want_inv = cf.ntt_inv(a, twi, ninv)  # inverse of an arbitrary (canonical) input
    T.inv_dev(x, x, batch)
    torch.cuda.synchronize()
    assert (x.cpu().numpy().view(np.uint64).reshape(batch, N, 1) == want_inv).all()


@pytest.mark.parametrize("logn,negacyclic", [(16, True), (16, False), (15, True), (15, False)])
@pytest.mark.parametrize("batch", [1, 4, 5])
def test_ntt_2e16_q255_matches_oracle(fields, batch, logn, negacyclic):
    """Degree 2^16 and 2^15 at the Jindo default prime (4 limbs, q = 1 mod 2^64): the ntt256
    kernels (N = 2^15: a 7-stage COL pass of 128-point columns, 8 per tile; both ROW tilings: same
    row of 4 polys when batch % 4 == 0, else 4 rows of one poly), cyclic (Buckler's encoder) and
    negacyclic, forward vs the C oracle, inverse round trip and inverse of arbitrary input."""
    q = fields["jindo_zp"]
    N = 1 << logn
    F = ringo.Field(q)
    cf = co.CField(q)
    T = (ringo.CyclotomicTransformer if negacyclic else ringo.CyclicTransformer)(F, N)
    tw, twi, ninv = cf.tables(N, cyclic=not negacyclic)
    rng = np.random.default_rng(100 + batch)
    a = F.random(batch * N, rng).reshape(batch, N, F.L)
    a[0, 0] = F.mont([q - 1])[0]
    got = T.FwdNTTTo(None, a)
    assert (got == cf.ntt_fwd(a, tw)).all()
    assert (T.InvNTTTo(None, got) == a).all()
    assert (T.InvNTTTo(None, a) == cf.ntt_inv(a, twi, ninv)).all()


def test_empty_batches_are_noops(fields):
    """Empty inputs: the reference's loops over zero polynomials / elements do nothing
    (ntt.go:98-136 over a batch of none, vec.go:9-121 with n = 0). The device entry points
    must return OK without launching, and leave the output buffer untouched."""
    import torch

    q = fields["p63"]
    F = ringo.Field(q)
    T = ringo.CyclotomicTransformer(F, 1 << 16)
    dev = torch.device("cuda", 0)
    sentinel = torch.full((8,), 12345, dtype=torch.int64, device=dev)
    T.fwd_dev(sentinel, sentinel, 0)
    T.inv_dev(sentinel, sentinel, 0)
    L = ringo.lib()
    ringo._lib.check(L.rg_vec_dev(F.h, ringo.bigpoly._OPS["mul"], sentinel.data_ptr(), sentinel.data_ptr(),
                                  sentinel.data_ptr(), 0, None))
    torch.cuda.synchronize()
    assert (sentinel.cpu() == 12345).all()


def test_ntt_2e16_full_batch_spot_check(fields):
    """The headline's full configs[1] batch (1024 polynomials, 512 MiB, in place as bench.py runs
    it): polynomials 0, 511 and 1023 of the forward transform against the C oracle, then the
    inverse restores all 1024 bit-exactly.  Inputs are generated on the device (SplitMix64-like
    hash of the word index mod p) so the host only materialises the three checked polynomials."""
    import torch
    q = fields["p63"]
    N, B = 1 << 16, 1024
    F = ringo.Field(q)
    cf = co.CField(q)
    T = ringo.CyclotomicTransformer(F, N)
    tw, _, _ = cf.tables(N)
    idx = torch.arange(B * N, dtype=torch.int64, device="cuda")
    z = idx * 0x9E3779B97F4A7C15 + 0x52494E47
    z = (z ^ ((z >> 30) & ((1 << 34) - 1))) * 0xBF58476D1CE4E5B9
    z = (z ^ ((z >> 27) & ((1 << 37) - 1))) * 0x94D049BB133111EB
    z = (z ^ ((z >> 31) & ((1 << 33) - 1))) & ((1 << 62) - 1)
    x = torch.remainder(z, q)  # < 2^62 < p: already canonical, kept as remainder for clarity
    picks = [0, 511, 1023]
    a = np.stack([x[i * N:(i + 1) * N].cpu().numpy().view(np.uint64) for i in picks]).reshape(3, N, 1)
    ref = x.clone()
    T.fwd_dev(x, x, B)
    torch.cuda.synchronize()
    want = cf.ntt_fwd(a, tw)
    for j, i in enumerate(picks):
        got = x[i * N:(i + 1) * N].cpu().numpy().view(np.uint64).reshape(N, 1)
        assert (got == want[j]).all(), i
    T.inv_dev(x, x, B)
    torch.cuda.synchronize()
    assert torch.equal(x, ref)


def test_ntt_2e16_q255_bench_batch_spot_check(fields):
    """configs[3]'s full L = 4 batch as bench.py's l4 line runs it (64 polynomials of 2^16
    Montgomery words at the Jindo default prime, 128 MiB, in place): polynomials 0, 37 and 63 of
    the forward transform against the C oracle, then the inverse restores all 64 bit-exactly.
    Covers the ntt256_pass same-row-of-4 ROW tiling at the batch the bench times."""
    import torch
    q = fields["jindo_zp"]
    N, B = 1 << 16, 64
    F = ringo.Field(q)
    cf = co.CField(q)
    T = ringo.CyclotomicTransformer(F, N)
    tw, _, _ = cf.tables(N)
    assert q > 1 << 254  # words below 2^254 are canonical residues (valid Montgomery forms)
    rng = np.random.default_rng(255)
    a = rng.integers(0, 2 ** 64, size=(B, N, F.L), dtype=np.uint64)
    a[:, :, 3] >>= np.uint64(2)
    a[63, N - 1] = F.mont([q - 1])[0]
    x = torch.from_numpy(a.view(np.int64).reshape(-1).copy()).cuda()
    ref = x.clone()
    T.fwd_dev(x, x, B)
    torch.cuda.synchronize()
    picks = [0, 37, 63]
    want = cf.ntt_fwd(np.ascontiguousarray(a[picks]), tw)
    got = x.cpu().numpy().view(np.uint64).reshape(B, N, F.L)
    for j, i in enumerate(picks):
        assert (got[i] == want[j]).all(), i
    T.inv_dev(x, x, B)
    torch.cuda.synchronize()
    assert torch.equal(x, ref)


@pytest.mark.parametrize("logn", [16, 15])
def test_ntt_q255_split_halves_match_oracle(fields, logn):
    """From 8 polynomials up ntt256_run runs the batch as two halves, the second on the plan's
    helper stream (ntt_l4_fast.hip run_split): batches 8 (4 + 4, both halves on the same-row-of-4
    ROW tiling), 9 (4 + 5: the second half on the 4-rows-of-one-poly tiling) and 14 (8 + 6), on a
    side stream, out of place then in place, every polynomial against the C oracle.  Then two
    streams share the plan with interleaved transforms (the fork/join events are per plan)."""
    import torch
    q = fields["jindo_zp"]
    N = 1 << logn
    F = ringo.Field(q)
    cf = co.CField(q)
    T = ringo.CyclotomicTransformer(F, N)
    tw, twi, ninv = cf.tables(N)
    side = torch.cuda.Stream()
    for B in (8, 9, 14):
        rng = np.random.default_rng(1000 + B + logn)
        a = F.random(B * N, rng).reshape(B, N, F.L)
        x = torch.from_numpy(a.view(np.int64).reshape(-1).copy()).cuda()
        y = torch.empty_like(x)
        torch.cuda.synchronize()
        T.fwd_dev(y, x, B, stream=side)
        T.inv_dev(x, y, B, stream=side)  # y -> x: ordered behind the forward's helper half
        side.synchronize()
        assert (y.cpu().numpy().view(np.uint64).reshape(B, N, F.L) == cf.ntt_fwd(a, tw)).all(), B
        assert (x.cpu().numpy().view(np.uint64).reshape(B, N, F.L) == a).all(), B
        T.inv_dev(x, x, B, stream=side)
        side.synchronize()
        assert (x.cpu().numpy().view(np.uint64).reshape(B, N, F.L) == cf.ntt_inv(a, twi, ninv)).all(), B
    B = 12
    rng = np.random.default_rng(77 + logn)
    a = F.random(2 * B * N, rng).reshape(2, B, N, F.L)
    xs = [torch.from_numpy(a[i].view(np.int64).reshape(-1).copy()).cuda() for i in range(2)]
    sts = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    for _ in range(3):
        for i in range(2):
            T.fwd_dev(xs[i], xs[i], B, stream=sts[i])
        for i in range(2):
            T.inv_dev(xs[i], xs[i], B, stream=sts[i])
    torch.cuda.synchronize()
    for i in range(2):
        assert (xs[i].cpu().numpy().view(np.uint64).reshape(B, N, F.L) == a[i]).all(), i


@pytest.mark.parametrize("name,B", [("zp440", 32), ("zp880", 16)])
def test_ntt_2e16_wide_bench_batch_spot_check(fields, name, B):
    """The wide Buckler fields at the batch bench.py's wide_ntt_* lines time (zp440 x 32,
    zp880 x 16 polynomials of 2^16, in place; buckler_test.go:163-222 runs these fields): three
    polynomials of the forward transform against the C oracle, so a forward that is consistently
    wrong cannot hide behind the bench's fwd-then-inv self-check, then the in-place inverse
    restores all B bit-exactly."""
    import torch
    q = fields[name]
    N = 1 << 16
    F = ringo.Field(q)
    cf = co.CField(q)
    T = ringo.CyclotomicTransformer(F, N)
    tw, _, _ = cf.tables(N)
    rng = np.random.default_rng(440 + B)
    a = F.random(B * N, rng).reshape(B, N, F.L)
    a[B - 1, N - 1] = F.mont([q - 1])[0]  # the largest residue
    x = torch.from_numpy(a.view(np.int64).reshape(-1).copy()).cuda()
    ref = x.clone()
    T.fwd_dev(x, x, B)
    torch.cuda.synchronize()
    picks = [0, B // 2 + 1, B - 1]
    want = cf.ntt_fwd(np.ascontiguousarray(a[picks]), tw)
    got = x.cpu().numpy().view(np.uint64).reshape(B, N, F.L)
    for j, i in enumerate(picks):
        assert (got[i] == want[j]).all(), (name, i)
    T.inv_dev(x, x, B)
    torch.cuda.synchronize()
    assert torch.equal(x, ref)


@pytest.mark.parametrize("name,logn", [("p63", 16), ("zp440", 10), ("zp880", 9), ("jindo_zp", 8)])
def test_from_tables_honours_rank_inv(fields, name, logn):
    """rg_ntt_create_from_tables takes Go's tables verbatim, rankInv included (ntt.go:86-87,
    194-195 set it to N^-1; InvNTTTo multiplies by whatever the transformer holds,
    ntt.go:242-243).  A plan built with another canonical rank_inv must scale by it, on every
    kernel family: the wide fields' per-stage-halving pass only computes N^-1, so such a plan
    takes the per-stage inverse instead."""
    q = fields[name]
    N = 1 << logn
    F = ringo.Field(q)
    cf = co.CField(q)
    T0 = ringo.CyclotomicTransformer(F, N)
    tw, twi, ninv = T0.tables()
    rinv = F.mont([pow(3 * N, -1, q)])[0]  # (3N)^-1: a third of the reference's scaling
    T = ringo.CyclotomicTransformer(F, N, tables=(tw, twi, rinv))
    rng = np.random.default_rng(logn)
    a = F.random(2 * N, rng).reshape(2, N, F.L)
    got = T.InvNTTTo(None, a)
    assert (got == cf.ntt_inv(a, twi, rinv)).all(), name
    assert not (got == T0.InvNTTTo(None, a)).all()
    assert (T.FwdNTTTo(None, a) == T0.FwdNTTTo(None, a)).all()
