// digits_dc.hpp -- the base-b digits of Encoder.Encode (jindo/encoder.go:125-136: exp - 1 remainders
// of repeated division by b, then the last quotient) by divide and conquer, for the two field
// shapes of the configs: L = 4 words with exp = 16 (the 255-bit jindo modulus, b = 60272) and
// L = 2 with exp = 8 (examples/mult's 128-bit field, b = 60256).
//
// Round 5's digits_kernel divided the whole value by b^2 seven times (a predicated 8-word long
// division per pass: ~1,500 VALU per element).  Here the value is split once by B8 = b^8, each
// half by B4 = b^4, each quarter by B2 = b^2 and each eighth by b:
//   c = H B8 + Lo (Barrett, mu8 = floor(2^256 / B8) = 2^128 + m1 2^64 + m0)
//   Lo = L1 B4 + L0,  H = H1 B4 + H0 (Barrett, mu4 = floor(2^128 / B4) = 2^64 + u0)
//   64-bit quarters < B4 = xh B2 + xl (divstep by B2), 32-bit eighths < B2 = d1 b + d0
// Each Barrett quotient is Q or Q - 1 (the dropped fraction is below 1), so one conditional
// correction makes it exact.  Preconditions (checked on the host, DigitDc::exp = 0 otherwise):
// b^2 in (2^31, 2^32), B4 > 2^63, and for L = 4: B8 >= 2^127 and q < 2^255, so that H < 2^128, the
// top quarter H1 < 2^65 and its top eighth G < 2^34; the last digit floor(c / b^(exp-1)) = G / b
// may exceed b, as the reference's last quotient does.
//
// RG_HD: the same source is compiled for the host by tests/test_digits_dc.py and checked there
// against Python integers on edge and random values.
#pragma once
#include <stdint.h>

#include "field.hpp"

namespace rg {

struct DigitDc {
  uint64_t b, b2, b2inv, binv;  // base, b^2, floor(2^64 / b^2), floor(2^64 / b)
  uint64_t b4, u0;              // B4 = b^4, floor(2^128 / B4) - 2^64
  uint64_t b8lo, b8hi, m0, m1;  // B8 = b^8, floor(2^256 / B8) - 2^128
  int exp;                      // 16 (L = 4), 8 (L = 2), 0: the general loop
};

RG_HD uint32_t dc_umulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

// (r 2^32 + n0) / B2 for r < B2, B2 in (2^31, 2^32): floor(2^64 / B2) = 2^32 + B0, so
// hi64(num (2^32 + B0)) = r + hi32(r B0 + n0 + hi32(n0 B0)) (three 32-bit products)
RG_HD uint32_t dc_div_b2(uint32_t r, uint32_t n0, const DigitDc& K, uint32_t& rem) {
  const uint32_t B0 = (uint32_t)K.b2inv;
  const uint64_t t = mad64(r, B0, (uint64_t)n0 + dc_umulhi(n0, B0));
  uint32_t qt = r + (uint32_t)(t >> 32);
  uint64_t rm = (((uint64_t)r << 32) | n0) - (uint64_t)qt * K.b2;
  if (rm >= K.b2) {
    rm -= K.b2;
    ++qt;
  }
  rem = (uint32_t)rm;
  return qt;
}

// num / b for num < b 2^32 (quotient < 2^32): hi64(num floor(2^64 / b)) is Q or Q - 1
RG_HD uint32_t dc_div_b(uint64_t num, const DigitDc& K, uint32_t& rem) {
  uint64_t qt = mul_hi(num, K.binv);
  uint64_t rm = num - qt * K.b;
  if (rm >= K.b) {
    rm -= K.b;
    ++qt;
  }
  rem = (uint32_t)rm;
  return (uint32_t)qt;
}

// N = n1 2^64 + n0 (< 2^128) = Q B4 + r, Q = q1 2^64 + q0 (q1 <= 1 when B4 > 2^63), r < B4
RG_HD void dc_split_b4(uint64_t n0, uint64_t n1, const DigitDc& K, uint64_t& q0, uint32_t& q1, uint64_t& r) {
  // floor(N mu4 / 2^128) with N mu4 = N u0 + N 2^64: limbs 2 and 3 of
  // n0 u0 + (n1 u0 + n0) 2^64 + n1 2^128
  uint64_t a0, a1, b0, b1;
  mul_wide(n0, K.u0, a0, a1);
  mul_wide(n1, K.u0, b0, b1);
  uint32_t c1 = 0, c2 = 0;
  const uint64_t s1 = addc(a1, b0, c1);
  addc(s1, n0, c2);  // limb 1: only its carries matter
  uint32_t c3 = 0;
  const uint64_t s2 = addc(b1, n1, c3);
  uint32_t c4 = 0;
  uint64_t e0 = addc(s2, (uint64_t)(c1 + c2), c4);
  uint32_t e1 = c3 + c4;
  // r = N - Q B4 mod 2^128 (the true remainder is < 2 B4 < 2^65)
  uint64_t p0, p1;
  mul_wide(e0, K.b4, p0, p1);
  p1 += e1 ? K.b4 : 0;
  uint32_t br = 0;
  uint64_t r0 = subb(n0, p0, br);
  const uint64_t r1 = n1 - p1 - br;
  if (r1 != 0 || r0 >= K.b4) {
    r0 -= K.b4;
    e0 += 1;
    e1 += e0 == 0;
  }
  q0 = e0;
  q1 = e1;
  r = r0;
}

// c (4 words, < 2^255) = H B8 + Lo, H = (h1, h0) < 2^128, Lo = (l1, l0) < B8
RG_HD void dc_split_b8(const uint64_t c[4], const DigitDc& K, uint64_t& h0, uint64_t& h1, uint64_t& l0,
                       uint64_t& l1) {
  // S = c (m0 + m1 2^64) + c 2^128; Q = floor(S / 2^256) = limbs 4, 5
  uint64_t s[6] = {0, 0, c[0], c[1], c[2], c[3]};
  auto row = [&](int off, uint64_t m) {
    uint64_t carry = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint64_t lo, hi;
      mul_wide(c[i], m, lo, hi);
      uint32_t k1 = 0, k2 = 0;
      lo = addc(lo, carry, k1);
      s[off + i] = addc(s[off + i], lo, k2);
      carry = hi + k1 + k2;  // hi <= 2^64 - 2
    }
#pragma unroll
    for (int k = off + 4; k < 6; ++k) {
      uint32_t k3 = 0;
      s[k] = addc(s[k], carry, k3);
      carry = k3;
    }
  };
  row(0, K.m0);
  row(1, K.m1);
  uint64_t q0 = s[4], q1 = s[5];
  // Lo = c - Q B8 mod 2^192 (the true remainder is < 2 B8 < 2^129)
  uint64_t a0, a1, b0, b1, e0, e1;
  mul_wide(q0, K.b8lo, a0, a1);
  mul_wide(q0, K.b8hi, b0, b1);
  mul_wide(q1, K.b8lo, e0, e1);
  uint32_t k1 = 0, k2 = 0;
  uint64_t t1 = addc(a1, b0, k1);
  t1 = addc(t1, e0, k2);
  const uint64_t t2 = b1 + e1 + q1 * K.b8hi + k1 + k2;
  uint32_t br = 0;
  uint64_t r0 = subb(c[0], a0, br);
  uint64_t r1 = subb(c[1], t1, br);
  const uint64_t r2 = c[2] - t2 - br;
  if (r2 != 0 || r1 > K.b8hi || (r1 == K.b8hi && r0 >= K.b8lo)) {
    uint32_t b2 = 0;
    r0 = subb(r0, K.b8lo, b2);
    r1 = subb(r1, K.b8hi, b2);
    q0 += 1;
    q1 += q0 == 0;
  }
  h0 = q0;
  h1 = q1;
  l0 = r0;
  l1 = r1;
}

// digits pos .. pos + 3 of a quarter X < B4
template <class Put>
RG_HD void dc_quarter(uint64_t X, int pos, const DigitDc& K, Put& put) {
  uint32_t xl, d;
  const uint32_t xh = dc_div_b2((uint32_t)(X >> 32), (uint32_t)X, K, xl);
  put(pos + 1, dc_div_b(xl, K, d));
  put(pos, d);
  put(pos + 3, dc_div_b(xh, K, d));
  put(pos + 2, d);
}
// digits pos .. pos + 3 of the top quarter (q1 2^64 + q0 < 2^65); the last is the unbounded quotient
template <class Put>
RG_HD void dc_top(uint64_t q0, uint32_t q1, int pos, const DigitDc& K, Put& put) {
  uint32_t r1, g0, d;
  const uint32_t gh = dc_div_b2(q1, (uint32_t)(q0 >> 32), K, r1);
  const uint32_t gl = dc_div_b2(r1, (uint32_t)q0, K, g0);
  put(pos + 1, dc_div_b(g0, K, d));
  put(pos, d);
  put(pos + 3, dc_div_b(((uint64_t)gh << 32) | gl, K, d));
  put(pos + 2, d);
}

// c: the canonical value, L = 4 (exp 16) or L = 2 (exp 8) words; put(j, digit j)
template <int L, class Put>
RG_HD void dc_digits(const uint64_t (&c)[L], const DigitDc& K, Put put) {
  if constexpr (L == 4) {
    uint64_t h0, h1, l0, l1, q0, r;
    uint32_t q1;
    dc_split_b8(c, K, h0, h1, l0, l1);
    dc_split_b4(l0, l1, K, q0, q1, r);  // Lo < B8: its quotient < B4 (q1 = 0)
    dc_quarter(r, 0, K, put);
    dc_quarter(q0, 4, K, put);
    dc_split_b4(h0, h1, K, q0, q1, r);
    dc_quarter(r, 8, K, put);
    dc_top(q0, q1, 12, K, put);
  } else {
    uint64_t q0, r;
    uint32_t q1;
    dc_split_b4(c[0], c[1], K, q0, q1, r);
    dc_quarter(r, 0, K, put);
    dc_top(q0, q1, 4, K, put);
  }
}

// host: the constants, or exp = 0 when a precondition fails (q_bits: bit length of the modulus)
inline DigitDc dc_constants(uint64_t base, int exp, int L, int q_bits) {
  DigitDc K{};
  K.exp = 0;
  const uint64_t b2 = base * base;
  if (base < 2 || (b2 >> 32) != 0 || b2 <= (1ull << 31)) return K;
  K.b = base;
  K.b2 = b2;
  K.b2inv = (uint64_t)(((unsigned __int128)1 << 64) / b2);
  K.binv = (uint64_t)(((unsigned __int128)1 << 64) / base);
  K.b4 = b2 * b2;
  if (K.b4 <= (1ull << 63)) return K;
  const unsigned __int128 mu4 = ~(unsigned __int128)0 / K.b4;  // B4 is no power of two: = floor(2^128 / B4)
  if ((uint64_t)(mu4 >> 64) != 1) return K;
  K.u0 = (uint64_t)mu4;
  if (L == 2 && exp == 8 && q_bits <= 128) {
    K.exp = 8;
    return K;
  }
  if (L != 4 || exp != 16 || q_bits > 255) return K;
  const unsigned __int128 B8 = (unsigned __int128)K.b4 * K.b4;
  if ((uint64_t)(B8 >> 127) != 1) return K;  // B8 in [2^127, 2^128)
  K.b8lo = (uint64_t)B8;
  K.b8hi = (uint64_t)(B8 >> 64);
  // floor(2^256 / B8) - 2^128 = floor((2^128 - B8) 2^128 / B8): long division, one bit at a time
  const unsigned __int128 D = (unsigned __int128)0 - B8;  // 2^128 - B8 < B8
  unsigned __int128 rem = D, quo = 0;
  for (int i = 0; i < 128; ++i) {
    const bool top = (rem >> 127) != 0;  // 2 rem overflows 128 bits
    rem <<= 1;
    const bool ge = top || rem >= B8;
    if (ge) rem -= B8;  // wraps correctly when top is set (the true 2 rem - B8 < B8 < 2^128)
    quo = (quo << 1) | (ge ? 1 : 0);
  }
  K.m0 = (uint64_t)quo;
  K.m1 = (uint64_t)(quo >> 64);
  K.exp = 16;
  return K;
}

}  // namespace rg
