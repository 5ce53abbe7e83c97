"""CPU: the divide-and-conquer base-b digit split (ringo-snark_amd/csrc/digits_dc.hpp, used by
digits_kernel on the device) compiled for the host with g++ from the same source and compared with
Python integers: Encoder.Encode's digits (jindo/encoder.go:125-136: exp - 1 remainders of repeated
division by b, then the final quotient, which may exceed b).  Both configs shapes: the 255-bit
jindo modulus (L = 4, exp 16, b = 60272) and examples/mult's 128-bit field (L = 2, exp 8,
b = 60256); edge values (0, q - 1, powers of b and their neighbours, every Barrett boundary) and
seeded random values.  The commit parity tests pin the device build of the same code."""
import ctypes
import json
import os
import random
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "ringo-snark_amd", "csrc")
PARAMS = json.load(open(os.path.join(HERE, "golden", "jindo_params.json")))

HARNESS = r"""
#include "digits_dc.hpp"
extern "C" int dc_run(uint64_t base, int exp, int L, int qbits, const uint64_t* c, long n, uint32_t* out) {
  const rg::DigitDc K = rg::dc_constants(base, exp, L, qbits);
  if (K.exp != exp) return 1;
  for (long i = 0; i < n; ++i) {
    uint32_t* o = out + i * exp;
    auto put = [&](int j, uint32_t d) { o[j] = d; };
    if (L == 4) {
      const uint64_t w[4] = {c[4 * i], c[4 * i + 1], c[4 * i + 2], c[4 * i + 3]};
      rg::dc_digits<4>(w, K, put);
    } else {
      const uint64_t w[2] = {c[2 * i], c[2 * i + 1]};
      rg::dc_digits<2>(w, K, put);
    }
  }
  return 0;
}
extern "C" int dc_check(uint64_t base, int exp, int L, int qbits) {
  return rg::dc_constants(base, exp, L, qbits).exp;
}
"""


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("dc")
    src, so = d / "dc.cpp", d / "libdc.so"
    src.write_text(HARNESS)
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-I", CSRC, str(src), "-o", str(so)], check=True)
    L = ctypes.CDLL(str(so))
    L.dc_run.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_long,
                         ctypes.c_void_p]
    L.dc_check.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    return L


def _ref(c, b, exp):
    out = []
    for _ in range(exp - 1):
        out.append(c % b)
        c //= b
    out.append(c)
    return out


def _shapes():
    seen = {}
    for name, P in PARAMS.items():
        q = int(P["field_q_hex"], 16)
        L = (q.bit_length() + 63) // 64
        seen[(P["base"], P["exp"], L, q)] = name
    return sorted(seen.items(), key=lambda x: x[1])


# the BASELINE configs' fields (q255: configs[2]-[4], examples/mult: configs[0]) must take the fast
# path; the zp package's other fields (exp 4 .. 64 as Buckler's Jindo fields) keep the device's
# general long division, pinned by tests/test_gpu_jindo_fields.py
CONFIG_BASES = {60272, 60256}


@pytest.mark.parametrize("shape", _shapes(), ids=lambda s: s[1])
def test_digits_dc_matches_integers(lib, shape):
    (b, exp, L, q), _ = shape
    got = lib.dc_check(b, exp, L, q.bit_length())
    if b in CONFIG_BASES:
        assert got == exp  # every configs field takes the fast path
    assert got in (0, exp)
    if got == 0:
        return
    B2, B4 = b * b, b ** 4
    vals = {0, 1, q - 1, q - 2, b - 1, b, B2 - 1, B2, B4 - 1, B4, B4 + 1}
    for k in range(exp + 2):
        for d in (-2, -1, 0, 1):
            vals.add(b ** k + d)
            vals.add(q - b ** k + d)
    for m in range(1, 9):  # multiples of the split points, where a Barrett quotient is exact
        vals.update({m * B4 - 1, m * B4, (q // B4) * B4 - m})
        if exp == 16:
            vals.update({m * b ** 8 - 1, m * b ** 8, (q // b ** 8) * b ** 8 - m})
    rng = random.Random(7)
    vals.update(rng.randrange(q) for _ in range(100000))
    vals.update(rng.randrange(1 << rng.randrange(1, q.bit_length())) for _ in range(20000))  # short values
    vals = sorted(v for v in vals if 0 <= v < q)
    words = np.array([[(v >> (64 * i)) & ((1 << 64) - 1) for i in range(L)] for v in vals], dtype=np.uint64)
    out = np.zeros((len(vals), exp), dtype=np.uint32)
    assert lib.dc_run(b, exp, L, q.bit_length(), words.ctypes.data, len(vals), out.ctypes.data) == 0
    for i, v in enumerate(vals):
        assert out[i].tolist() == _ref(v, b, exp), v


def test_digits_dc_refuses_other_shapes(lib):
    """Outside its preconditions dc_constants returns exp = 0 and digits_kernel keeps the general
    long division: b^2 not in (2^31, 2^32), b^8 < 2^127 at L = 4, exp or L other than 16/4, 8/2."""
    assert lib.dc_check(60272, 16, 4, 255) == 16
    assert lib.dc_check(60256, 8, 2, 128) == 8
    assert lib.dc_check(40000, 16, 4, 255) == 0   # b^2 < 2^31
    assert lib.dc_check(65537, 16, 4, 255) == 0   # b^2 >= 2^32
    assert lib.dc_check(60000, 16, 4, 255) == 0   # b^8 < 2^127
    assert lib.dc_check(60272, 16, 4, 256) == 0   # q too wide for H < 2^128
    assert lib.dc_check(60272, 15, 4, 255) == 0
    assert lib.dc_check(60272, 8, 2, 129) == 0
