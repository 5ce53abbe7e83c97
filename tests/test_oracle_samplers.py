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
import math
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


# ---- goodness of fit against the exact distributions (pin the float paths by
# distribution).  Each case draws 10^6 samples of ONE reference sampler from the C restatement
# (fixed seeds: deterministic) and runs a chi-square test against the exact pmf, with bins merged
# until every expected count is >= 20.

def _chi2_p(x, support, pmf):
    """p-value of draws `x` (ints) against pmf over `support` (consecutive ints; the mass outside
    goes to the two end bins)."""
    from scipy.stats import chi2
    lo = support[0]
    counts = np.bincount(np.clip(x - lo, 0, len(support) - 1), minlength=len(support)).astype(np.float64)
    exp_ = pmf / pmf.sum() * len(x)
    obs_b, exp_b, co_, ce = [], [], 0.0, 0.0
    for o, e in zip(counts, exp_):
        co_ += o
        ce += e
        if ce >= 20:
            obs_b.append(co_)
            exp_b.append(ce)
            co_, ce = 0.0, 0.0
    obs_b[-1] += co_
    exp_b[-1] += ce
    obs_b, exp_b = np.array(obs_b), np.array(exp_b)
    stat = ((obs_b - exp_b) ** 2 / exp_b).sum()
    return chi2.sf(stat, len(obs_b) - 1), len(obs_b)


def _seeds2(tag):
    return hashlib.sha256(tag + b"0").digest() + hashlib.sha256(tag + b"1").digest()


def _dgauss(support, sigma, c):
    z = support.astype(np.float64) - c
    return np.exp(-z * z / (2 * sigma * sigma))


N_DRAWS = 1_000_000


@pytest.mark.parametrize("center", [0.0, 0.3, -2.71, 0.5 + 1 / 256, 1e5 + 0.83])
def test_twin_cdt_chi_square(center):
    """TwinCDTGaussianSampler.Sample(center) (gaussian_twin_cdt.go:77-111) at ecdStdDev.  The
    reference returns table c0's value on every draw: where the two tables disagree its fallback
    sums the exp terms over x <= the INDEX v0 (sic: values -tailHi .. v0, not .. v0 + tailLo), so
    p < cdf always holds.  The distribution is therefore D_{Z, sigma, floor(c) + c0/128} with
    c0 = floor(128 frac(c)): the centre quantised down to the 1/128 grid."""
    sigma = PARAMS["t16_b4096"]["ecd_sd"]
    x = co.sampler_draws("twin_cdt", _seeds2(b"cdt%r" % center), sigma, center, N_DRAWS)
    fl = np.floor(center)
    mu = fl + np.floor(128 * (center - fl)) / 128
    support = np.arange(int(fl) - 60, int(fl) + 62)
    p, nb = _chi2_p(x, support, _dgauss(support, sigma, mu))
    assert nb > 20 and p > 1e-3, (p, nb)
    # and the unquantised centre is the wrong model where the quantisation step is large
    if center == 0.5 + 1 / 256:
        assert abs(x.mean() - mu) < 4 * sigma / np.sqrt(N_DRAWS)


# The reference's normFloat (gaussian_rounded.go:22-116) as its tables define it: xn[0] and fn[0]
# are never set (0), so layer 1's wedge test U (fn[0] - fn[1]) < f(x) - fn[1] always passes and
# the top strip |x| < xn[1] = 0.2723 comes out UNIFORM at density fn[1] + v / xn[1] (~1.0)
# instead of following exp(-x^2/2); every other layer is the exact ziggurat (area v each).
RN = 3.442619855899


def _zig_top():
    nrm = lambda x: math.exp(-0.5 * x * x)
    v = RN * nrm(RN) + math.sqrt(math.pi / 2) * math.erfc(RN / math.sqrt(2))
    x = RN
    for _ in range(126):  # xn[126] .. xn[1]
        x = math.sqrt(-2 * math.log(v / x + nrm(x)))
    return x, v


def _nf():
    from scipy.stats import norm
    xn1, v = _zig_top()
    ctop = math.exp(-0.5 * xn1 * xn1) + v / xn1
    zn = math.sqrt(2 * math.pi) * (1 - (norm.cdf(xn1) - norm.cdf(-xn1))) + 2 * xn1 * ctop
    return xn1, lambda x: np.where(np.abs(x) < xn1, ctop, np.exp(-0.5 * x * x)) / zn


_GL = np.polynomial.legendre.leggauss(24)


def _integ(lo, hi, f, kinks):
    """row-wise integral of f over [lo, hi], Gauss-Legendre on the pieces between kink points"""
    pts = np.sort(np.concatenate([lo[:, None], hi[:, None], np.clip(kinks, lo[:, None], hi[:, None])], axis=1), axis=1)
    tot = np.zeros(len(lo))
    for j in range(pts.shape[1] - 1):
        a, b = pts[:, j], pts[:, j + 1]
        y = ((a + b) / 2)[:, None] + ((b - a) / 2)[:, None] * _GL[0][None, :]
        tot += (b - a) / 2 * (f(y) * _GL[1][None, :]).sum(axis=1)
    return tot


def _go_round(x):  # math.Round: half away from zero
    return float(np.sign(x) * np.floor(abs(x) + 0.5))


def _rounded_pmf(support, sigma, c):
    """P(round(c + sigma normFloat) = k)"""
    xn1, nf = _nf()
    kinks = np.tile([-xn1, xn1], (len(support), 1))
    return _integ((support - 0.5 - c) / sigma, (support + 0.5 - c) / sigma, nf, kinks)


def _cosac_pmf(support, sigma, center):
    """The distribution gaussian_cosac.go:22-57 samples, exactly: r < rho(cFrac) / (sqrt(2 pi) sigma)
    returns cInt; otherwise the loop's candidate yRound (= round(y) -+ 1 for b = 0 / 1, y = sigma
    normFloat) is kept on its side (b = 0: yRound <= 0.5, b = 1: yRound >= -0.5 -- so yRound = 0
    is reachable from BOTH sides, sic) and accepted with min(1, exp(-((yRound + cFrac)^2 - y^2) /
    2 sigma^2)); P(loop returns k) = q(k) / sum q with q(k) = 1/2 sum over its sides of the integral
    of density(y) * acceptance over the y that round onto k."""
    xn1, nf = _nf()
    ci = _go_round(center)
    cf = ci - center
    kk = (support - ci).astype(np.float64)
    a = np.abs(kk + cf)
    s = sigma * xn1
    f = lambda y: nf(y / sigma) / sigma * np.minimum(1.0, np.exp((y * y - a[:, None] ** 2) / (2 * sigma * sigma)))
    kinks = np.stack([-a, a, np.full(len(a), -s), np.full(len(a), s)], axis=1)
    q = 0.5 * (np.where(kk <= 0, _integ(kk + 0.5, kk + 1.5, f, kinks), 0.0) +
               np.where(kk >= 0, _integ(kk - 1.5, kk - 0.5, f, kinks), 0.0))
    p1 = min(1.0, math.exp(-cf * cf / (2 * sigma * sigma)) / (math.sqrt(2 * math.pi) * sigma))
    return (1 - p1) * q / q.sum() + np.where(kk == 0, p1, 0.0)


@pytest.mark.parametrize("sigma,center", [(1.0, 0.2), (3.2, 0.37), (3.2, -5.5), (6.77, 12.25),
                                          (1733.2479139039056, -0.3), (1733.2479139039056, 1234.9)])
def test_cosac_chi_square(sigma, center):
    """COSACSampler.Sample(center, sigma) (gaussian_cosac.go:22-57), its rounded sampler's
    normFloat included, against the exact distribution of the reference's algorithm (_cosac_pmf)."""
    x = co.sampler_draws("cosac", _seeds2(b"cosac%r%r" % (sigma, center)), sigma, center, N_DRAWS)
    half = int(np.ceil(7 * sigma)) + 2
    support = np.arange(int(_go_round(center)) - half, int(_go_round(center)) + half + 1)
    p, nb = _chi2_p(x, support, _cosac_pmf(support, sigma, center))
    assert nb > 8 and p > 1e-3, (p, nb)
    if sigma == 3.2 and center == 0.37:
        # the same draws are far from the textbook D_{Z, sigma, c} (cInt is over-weighted), so
        # the test tells the reference's algorithm from the ideal one
        p0, _ = _chi2_p(x, support, _dgauss(support, sigma, center))
        assert p0 < 1e-12


@pytest.mark.parametrize("sigma,center", [(1.0, 0.0), (2.0, 0.3), (2451.1013707864035, 0.0)])
def test_rounded_chi_square(sigma, center):
    """RoundedGaussianSampler.Sample(center, sigma) (gaussian_rounded.go:77-125) = round(c + sigma
    normFloat), against the reference's normFloat density (uniform top strip; tail and wedges
    exact), integrated over each rounding cell."""
    x = co.sampler_draws("rounded", _seeds2(b"rnd%r%r" % (sigma, center)), sigma, center, N_DRAWS)
    half = int(np.ceil(6 * sigma)) + 2
    support = np.arange(-half, half + 1)
    p, nb = _chi2_p(x, support, _rounded_pmf(support, sigma, center))
    assert nb > 8 and p > 1e-3, (p, nb)
    # the tail branch (|N| > rn), against the normal tail mass
    from scipy.stats import norm
    t = np.abs(x - center) > RN * sigma + 1
    want = 2 * norm.sf(RN + 1 / sigma) * len(x) * (_nf()[1](np.array([RN + 1.0]))[0] / norm.pdf(RN + 1.0))
    assert abs(t.sum() - want) < 5 * np.sqrt(want), (t.sum(), want)
