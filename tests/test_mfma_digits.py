"""CPU check of the arithmetic behind mac_mfma.hip (the Jindo Ajtai MAC on the matrix cores):
the key's balanced base-256 digits, byte-reversed and shifted into the A operand of each digit
diagonal, the opening's bytes offset by 0x80 (read as int8), the per-(lk, j) correction and the
signed 128-bit fold give (sum_t A[t] B[t]) 2^-64 mod q exactly, as mac_kernel computes it (prover.go:149-157, the summed MulCoeffsMontgomeryThenAdd).

This restates the kernel's byte-level formulation in Python (no GPU); the GPU kernel itself is
checked bit for bit against the oracle by tests/test_gpu_jindo.py (test_mac_paths_agree and the
commit parity tests) and by tools/ubench/mac_mfma_check."""
import random

import pytest

PRIMES = [  # the configs' ring primes: configs[4] inner / outer, configs[2], examples/mult
    (288230376151736833, 545), (288230376151748609, 545), (18014398509485569, 144),
    (68719484929, 161), (34359753217, 65), (1125899906844161, 162),
]


def nb_of(q):
    """digits per residue (mac_mfma_nb): q < 2^(8 NB - 2)"""
    return max(4, ((q - 1).bit_length() + 2 + 7) // 8)


def sbyte(x):
    x &= 255
    return x - 256 if x >= 128 else x


def key_word(x, NB):
    """balanced digits of x, byte-reversed within NB bytes (mac_mfma_key_kernel)"""
    v, R = x, 0
    for k in range(NB):
        dg = v & 255
        if dg >= 128:
            dg -= 256
        v = (v - dg) >> 8
        R |= (dg & 255) << (8 * (NB - 1 - k))
    assert v == 0
    return R


def mac_digits(q, A, B):
    """one output of mac_mfma_kernel: diagonals D_s over (term, digit) pairs, then the fold"""
    NB = nb_of(q)
    bxor = sum(0x80 << (8 * k) for k in range(NB - 1))
    D = [0] * (2 * NB - 1)
    for a, b in zip(A, B):
        R, bp = key_word(a, NB), b ^ bxor
        for s in range(2 * NB - 1):
            sh = NB - 1 - s
            av = (R >> (8 * sh)) if sh >= 0 else (R << (-8 * sh)) & (2**64 - 1)
            D[s] += sum(sbyte(av >> (8 * i)) * sbyte(bp >> (8 * i)) for i in range(8))
    assert all(abs(d) < 2**31 for d in D)  # int32 accumulators
    S = sum(d << (8 * s) for s, d in enumerate(D))
    assert abs(S) < 2**126  # the signed 128-bit fold (mac_mfma_nb's bound)
    lo, hi = S & (2**64 - 1), S >> 64
    rinv = pow(2, -64, q)
    corr = (bxor % q) * (sum(A) % q) * rinv % q
    return (lo * rinv + hi + corr) % q


@pytest.mark.parametrize("q,T", PRIMES)
def test_digit_diagonals_equal_montgomery_sum(q, T):
    rng = random.Random(q ^ T)
    for trial in range(3):
        t = T if trial == 0 else rng.randrange(1, T + 1)
        pick = lambda: rng.choice([0, 1, q - 1, q - 2, rng.randrange(q)])  # noqa: E731
        A = [pick() for _ in range(t)]
        B = [pick() for _ in range(t)]
        want = sum(a * b for a, b in zip(A, B)) * pow(2, -64, q) % q
        assert mac_digits(q, A, B) == want


@pytest.mark.parametrize("q,T", PRIMES[:2])
def test_extreme_words(q, T):
    """all-(q-1) key and opening: the largest diagonals and fold the configs[4] shape reaches"""
    A, B = [q - 1] * T, [q - 1] * T
    assert mac_digits(q, A, B) == (q - 1) ** 2 * T * pow(2, -64, q) % q
