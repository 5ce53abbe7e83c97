// field.hpp -- modular arithmetic for gfx950 (and the host side of the library).
//
// Semantics: gnark-crypto generated Montgomery fields, R = 2^(64L), every result fully
// reduced to [0, q) (jindo/internal/zp/element.go:397-466, element_purego.go:46-213).  Because
// all values are canonical residues, any exact algorithm gives bit-identical limbs; the
// kernels therefore pick the cheapest exact form per case:
//   * L = 1 twiddle products use Shoup's precomputed-quotient multiply: mont(v, w*R) ==
//     v*w mod q, computed as v*w - floor(v*w'/2^64)*q with w' = floor(w*2^64/q).
//   * L >= 2 products use word-level CIOS Montgomery on 64-bit limbs built from
//     v_mad_u64_u32 (32x32+64 -> 64), the gfx950 integer multiply primitive (half rate:
//     measured 4-5 cycles per wave64 instruction vs 2 for v_add_u32, tools/ubench).
//   * Lattigo RNS limbs (single words < 2^61) use Shoup for constant operands and a
//     Barrett-free 2^64-Montgomery (MRed) for data x data products, as ring.MulCoeffsMontgomery.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RG_HD __host__ __device__ __forceinline__
#else
#define RG_HD inline
#endif

namespace rg {

// ------------------------------------------------------------------------------------------
// 64-bit building blocks
// ------------------------------------------------------------------------------------------
RG_HD uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }

// full 64x64 -> 128 product from four v_mad_u64_u32
RG_HD void mul_wide(uint64_t a, uint64_t b, uint64_t& lo, uint64_t& hi) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
  uint64_t t0 = mad64(a0, b0, 0);
  uint64_t t1 = mad64(a1, b0, t0 >> 32);
  uint64_t t2 = mad64(a0, b1, (uint32_t)t1);
  hi = mad64(a1, b1, (t1 >> 32) + (t2 >> 32));
  lo = (t2 << 32) | (uint32_t)t0;
#else
  unsigned __int128 p = (unsigned __int128)a * b;
  lo = (uint64_t)p;
  hi = (uint64_t)(p >> 64);
#endif
}

RG_HD uint64_t mul_hi(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
  uint64_t t1 = mad64(a1, b0, __umulhi(a0, b0));
  uint64_t t2 = mad64(a0, b1, (uint32_t)t1);
  return mad64(a1, b1, (t1 >> 32) + (t2 >> 32));
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

// lo 64 bits of a*b (one v_mad_u64_u32 + two v_mul_lo_u32)
RG_HD uint64_t mul_lo(uint64_t a, uint64_t b) { return a * b; }

// add with carry-in/out
RG_HD uint64_t addc(uint64_t a, uint64_t b, uint32_t& c) {
  uint64_t s = a + b;
  uint32_t c1 = s < a;
  uint64_t r = s + c;
  uint32_t c2 = r < s;
  c = c1 | c2;
  return r;
}
RG_HD uint64_t subb(uint64_t a, uint64_t b, uint32_t& br) {
  uint64_t d = a - b;
  uint32_t b1 = a < b;
  uint64_t r = d - br;
  uint32_t b2 = d < br;
  br = b1 | b2;
  return r;
}

// ------------------------------------------------------------------------------------------
// single-word modulus helpers (q < 2^63)
// ------------------------------------------------------------------------------------------
RG_HD uint64_t mod_add(uint64_t a, uint64_t b, uint64_t q) {
  uint64_t s = a + b;  // < 2q < 2^64
  return s >= q ? s - q : s;
}
RG_HD uint64_t mod_sub(uint64_t a, uint64_t b, uint64_t q) { return a >= b ? a - b : a + q - b; }
RG_HD uint64_t mod_neg(uint64_t a, uint64_t q) { return a ? q - a : 0; }

// Shoup: y * w mod q with wp = floor(w * 2^64 / q); y < 2^64, w < q < 2^63 -> canonical
RG_HD uint64_t shoup_mul(uint64_t y, uint64_t w, uint64_t wp, uint64_t q) {
  uint64_t qh = mul_hi(y, wp);
  uint64_t r = y * w - qh * q;  // in [0, 2q)
  return r >= q ? r - q : r;
}
// lazy variant: result in [0, 2q)
RG_HD uint64_t shoup_mul_lazy(uint64_t y, uint64_t w, uint64_t wp, uint64_t q) {
  return y * w - mul_hi(y, wp) * q;
}

// 2^64-Montgomery reduction for one word (Lattigo MRed semantics): a*b*2^-64 mod q,
// qinv = -q^-1 mod 2^64, q < 2^63.  Canonical output.
RG_HD uint64_t mont_mul1(uint64_t a, uint64_t b, uint64_t q, uint64_t qinv) {
  uint64_t lo, hi;
  mul_wide(a, b, lo, hi);
  uint64_t m = lo * qinv;
  uint64_t mh = mul_hi(m, q);
  // (a*b + m*q) / 2^64 = hi + mh + carry(lo + m*q_lo64); lo + (m*q mod 2^64) == 0 mod 2^64,
  // so the carry is 1 iff lo != 0.
  uint64_t r = hi + mh + (lo != 0);
  return r >= q ? r - q : r;
}

// host-side helpers ---------------------------------------------------------------------
inline uint64_t h_mulmod(uint64_t a, uint64_t b, uint64_t q) {
  return (uint64_t)((unsigned __int128)a * b % q);
}
inline uint64_t h_powmod(uint64_t a, uint64_t e, uint64_t q) {
  uint64_t r = 1 % q;
  a %= q;
  while (e) {
    if (e & 1) r = h_mulmod(r, a, q);
    a = h_mulmod(a, a, q);
    e >>= 1;
  }
  return r;
}
inline uint64_t h_shoup(uint64_t w, uint64_t q) {
  return (uint64_t)(((unsigned __int128)w << 64) / q);
}
inline uint64_t h_qinv_neg(uint64_t q0) {
  uint64_t inv = 1;
  for (int i = 0; i < 7; ++i) inv *= 2 - q0 * inv;
  return 0 - inv;
}

// ------------------------------------------------------------------------------------------
// multi-limb Montgomery field (L 64-bit limbs), parameters passed by value to kernels
// ------------------------------------------------------------------------------------------
template <int L>
struct FieldParams {
  uint64_t q[L];
  uint64_t qinv;  // -q^-1 mod 2^64
};

template <int L>
RG_HD bool geq_q(const uint64_t* a, const FieldParams<L>& F) {
#pragma unroll
  for (int i = L - 1; i >= 0; --i) {
    if (a[i] != F.q[i]) return a[i] > F.q[i];
  }
  return true;
}

// z = x + y mod q (element.go:397-413); x, y < q
template <int L>
RG_HD void f_add(uint64_t* z, const uint64_t* x, const uint64_t* y, const FieldParams<L>& F) {
  uint64_t s[L], t[L];
  uint32_t c = 0, br = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) s[i] = addc(x[i], y[i], c);
#pragma unroll
  for (int i = 0; i < L; ++i) t[i] = subb(s[i], F.q[i], br);
  // s >= q  <=>  carry out, or no borrow in s - q
  bool use_t = c || !br;
#pragma unroll
  for (int i = 0; i < L; ++i) z[i] = use_t ? t[i] : s[i];
}

// z = x - y mod q (element.go:437-451)
template <int L>
RG_HD void f_sub(uint64_t* z, const uint64_t* x, const uint64_t* y, const FieldParams<L>& F) {
  uint64_t d[L], t[L];
  uint32_t br = 0, c = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) d[i] = subb(x[i], y[i], br);
#pragma unroll
  for (int i = 0; i < L; ++i) t[i] = addc(d[i], F.q[i], c);
#pragma unroll
  for (int i = 0; i < L; ++i) z[i] = br ? t[i] : d[i];
}

// z = -x mod q (element.go:454-466)
template <int L>
RG_HD void f_neg(uint64_t* z, const uint64_t* x, const FieldParams<L>& F) {
  uint64_t orv = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) orv |= x[i];
  uint32_t br = 0;
  uint64_t t[L];
#pragma unroll
  for (int i = 0; i < L; ++i) t[i] = subb(F.q[i], x[i], br);
#pragma unroll
  for (int i = 0; i < L; ++i) z[i] = orv ? t[i] : 0;
}

// z = x * y * R^-1 mod q, CIOS on 64-bit limbs (element_purego.go:46-213); x, y < q.
// General form with an (L+2)-word accumulator, so it is exact also for moduli without a
// spare top bit (examples/mult/zp: a full 128-bit q).
template <int L>
RG_HD void f_mul(uint64_t* z, const uint64_t* x, const uint64_t* y, const FieldParams<L>& F) {
  uint64_t t[L + 2];
#pragma unroll
  for (int i = 0; i < L + 2; ++i) t[i] = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {  // t += x[i] * y
      uint64_t lo, hi;
      mul_wide(x[i], y[j], lo, hi);
      uint32_t c = 0;
      lo = addc(lo, t[j], c);
      hi += c;
      c = 0;
      lo = addc(lo, carry, c);
      hi += c;
      t[j] = lo;
      carry = hi;
    }
    uint32_t c = 0;
    t[L] = addc(t[L], carry, c);
    t[L + 1] = c;
    // m = t0 * qinv; t = (t + m*q) / 2^64
    uint64_t m = t[0] * F.qinv;
    uint64_t lo, hi;
    mul_wide(m, F.q[0], lo, hi);
    uint32_t c0 = 0;
    addc(lo, t[0], c0);
    carry = hi + c0;
#pragma unroll
    for (int j = 1; j < L; ++j) {
      mul_wide(m, F.q[j], lo, hi);
      uint32_t cc = 0;
      lo = addc(lo, t[j], cc);
      hi += cc;
      cc = 0;
      lo = addc(lo, carry, cc);
      hi += cc;
      t[j - 1] = lo;
      carry = hi;
    }
    c = 0;
    t[L - 1] = addc(t[L], carry, c);
    t[L] = t[L + 1] + c;
  }
  uint64_t s[L];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) s[i] = subb(t[i], F.q[i], br);
  bool use_s = t[L] || !br;
#pragma unroll
  for (int i = 0; i < L; ++i) z[i] = use_s ? s[i] : t[i];
}

// Element container (registers)
template <int L>
struct Elem {
  uint64_t v[L];
};

}  // namespace rg
