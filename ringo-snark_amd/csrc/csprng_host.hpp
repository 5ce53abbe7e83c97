// csprng_host.hpp -- host-side setup of the device samplers (math/csprng, jindo/encoder.go):
// AES-256 key schedule and T-table for the AES-CTR UniformSampler, the TwinCDT tables
// (gaussian_twin_cdt.go:13-37), the ziggurat tables of the rounded-Gaussian sampler
// (gaussian_rounded.go:22-52) and the encoder's deltaInv constants (encoder.go:50-67), the last
// computed exactly as Go's big.Float does (round-to-nearest-even at prec = bitlen(p) after every
// operation, then Float64()).
//
// Floating point: these follow the Go expressions operation by operation in IEEE double with no
// contraction (the host build has no FMA instructions; `fp contract(off)` makes it explicit).
// libm's exp/log/erfc may differ from Go's math package in the last ulp, which moves a table
// entry by a few units of 2^-53 relative: parity with Go there is unpinned.
#pragma once
#include <stdint.h>
#include <string.h>

#include <cmath>
#include <vector>

namespace rg {

#pragma clang fp contract(off)

// ---- AES-256 (FIPS-197) ------------------------------------------------------------------
inline uint8_t gf_mul(uint8_t a, uint8_t b) {
  uint8_t p = 0;
  for (int i = 0; i < 8; ++i) {
    if (b & 1) p ^= a;
    const bool hi = a & 0x80;
    a <<= 1;
    if (hi) a ^= 0x1b;
    b >>= 1;
  }
  return p;
}
inline void aes_sbox(uint8_t s[256]) {
  for (int x = 0; x < 256; ++x) {
    uint8_t inv = 0;
    if (x)
      for (int y = 1; y < 256; ++y)
        if (gf_mul((uint8_t)x, (uint8_t)y) == 1) {
          inv = (uint8_t)y;
          break;
        }
    uint8_t r = inv;
    for (int i = 1; i < 5; ++i) r ^= (uint8_t)((inv << i) | (inv >> (8 - i)));
    s[x] = r ^ 0x63;
  }
}
// Te0[x] = (2 S[x], S[x], S[x], 3 S[x]) as big-endian bytes of one word
inline void aes_te0(uint32_t te[256]) {
  uint8_t s[256];
  aes_sbox(s);
  for (int x = 0; x < 256; ++x)
    te[x] = ((uint32_t)gf_mul(s[x], 2) << 24) | ((uint32_t)s[x] << 16) | ((uint32_t)s[x] << 8) | gf_mul(s[x], 3);
}
// AES-256 key schedule: 60 big-endian round-key words
inline void aes256_expand(const uint8_t key[32], uint32_t rk[60]) {
  uint8_t s[256];
  aes_sbox(s);
  auto sub = [&](uint32_t w) {
    return ((uint32_t)s[w >> 24] << 24) | ((uint32_t)s[(w >> 16) & 255] << 16) | ((uint32_t)s[(w >> 8) & 255] << 8) |
           s[w & 255];
  };
  for (int i = 0; i < 8; ++i)
    rk[i] = ((uint32_t)key[4 * i] << 24) | ((uint32_t)key[4 * i + 1] << 16) | ((uint32_t)key[4 * i + 2] << 8) | key[4 * i + 3];
  uint8_t rc = 1;
  for (int i = 8; i < 60; ++i) {
    uint32_t t = rk[i - 1];
    if (i % 8 == 0) {
      t = sub((t << 8) | (t >> 24)) ^ ((uint32_t)rc << 24);
      rc = gf_mul(rc, 2);
    } else if (i % 8 == 4) {
      t = sub(t);
    }
    rk[i] = rk[i - 8] ^ t;
  }
}

// ---- TwinCDT tables (gaussian_twin_cdt.go:13-37) ------------------------------------------
// Go's float64 -> uint64 conversion on amd64 for x >= 2^63 is uint64(int64(x - 2^63)) | 1<<63;
// the one out-of-range value computeCDT can produce (cdf rounding to exactly 1.0, so
// Round(cdf * 2^64) = 2^64) therefore converts to 2^63 there.
inline uint64_t go_f2u64(double x) {
  const double two63 = 9223372036854775808.0;
  if (x < two63) return (uint64_t)(int64_t)x;
  const double y = x - two63;
  const int64_t z = y < two63 ? (int64_t)y : INT64_MIN;  // CVTTSD2SQ: out of range -> 0x8000...
  return (uint64_t)z | 0x8000000000000000ull;
}
inline std::vector<uint64_t> compute_cdt(double center, double sigma) {
  const int64_t tail_hi = (int64_t)std::ceil(9.0 * sigma);  // tailCut = 9
  const int64_t tail_lo = -tail_hi;
  std::vector<uint64_t> t((size_t)(tail_hi - tail_lo + 1));
  double cdf = 0.0;
  const double norm = std::sqrt(2.0 * M_PI) * sigma;
  int i = 0;
  for (int64_t x = tail_lo; x <= tail_hi; ++x, ++i) {
    const double xf = (double)x;
    const double rho = std::exp(-(xf - center) * (xf - center) / (2.0 * sigma * sigma)) / norm;
    cdf += rho;
    t[i] = cdf > 1.0 ? UINT64_MAX : go_f2u64(std::round(cdf * 18446744073709551616.0));
  }
  return t;
}

// ---- ziggurat tables (gaussian_rounded.go:9-52), blockSize 128, floatPrec 52 -------------
struct Ziggurat {
  uint64_t kn[128];
  double wn[128], fn[128];
};
inline Ziggurat make_ziggurat() {
  const double rn = 3.442619855899;
  auto normal = [](double x) { return std::exp(-0.5 * x * x); };
  auto normal_integral = [](double x) { return std::sqrt(M_PI / 2.0) * std::erfc(x / std::sqrt(2.0)); };
  auto normal_inv = [](double x) { return std::sqrt(-2.0 * std::log(x)); };
  Ziggurat Z;
  memset(&Z, 0, sizeof(Z));
  const double v = rn * normal(rn) + normal_integral(rn);
  double xn[128] = {0};
  xn[127] = rn;
  for (int i = 126; i >= 1; --i) xn[i] = normal_inv(v / xn[i + 1] + normal(xn[i + 1]));
  const double scale = 4503599627370496.0;  // 1 << floatPrec
  for (int i = 1; i < 128; ++i) {
    Z.kn[i] = go_f2u64((xn[i - 1] / xn[i]) * scale);
    Z.wn[i] = xn[i] / scale;
    Z.fn[i] = normal(xn[i]);
  }
  Z.kn[0] = go_f2u64((rn * normal(rn) / v) * scale);
  Z.wn[0] = (v / normal(rn)) / scale;
  return Z;
}

// ---- deltaInv (encoder.go:50-67) with big.Float semantics ----------------------------------
// A tiny arbitrary-precision binary float: value = (neg ? -1 : 1) * m * 2^e, m < 2^prec.
struct BigU {  // little-endian 32-bit words
  std::vector<uint32_t> w;
  int bits() const {
    for (int i = (int)w.size() - 1; i >= 0; --i)
      if (w[i]) return 32 * i + 32 - __builtin_clz(w[i]);
    return 0;
  }
  bool bit(int i) const { return i >= 0 && (size_t)(i >> 5) < w.size() && ((w[i >> 5] >> (i & 31)) & 1); }
  bool any_below(int i) const {  // any set bit in [0, i)
    for (int k = 0; k < i; ++k)
      if (bit(k)) return true;
    return false;
  }
  void shr(int s) {
    std::vector<uint32_t> o(w.size(), 0);
    for (int i = 0; i < (int)w.size() * 32; ++i)
      if (bit(i + s)) o[i >> 5] |= 1u << (i & 31);
    w = o;
  }
  void add1() {
    for (auto& x : w)
      if (++x) return;
    w.push_back(1);
  }
  void mul32(uint32_t b) {
    uint64_t c = 0;
    for (auto& x : w) {
      const uint64_t t = (uint64_t)x * b + c;
      x = (uint32_t)t;
      c = t >> 32;
    }
    if (c) w.push_back((uint32_t)c);
  }
};
// round m to `prec` significant bits, nearest even; returns the exponent shift applied
inline int round_to(BigU& m, int prec) {
  const int nb = m.bits();
  if (nb <= prec) return 0;
  const int s = nb - prec;
  const bool half = m.bit(s - 1), rest = m.any_below(s - 1);
  m.shr(s);
  if (half && (rest || m.bit(0))) {
    m.add1();
    if (m.bits() > prec) {
      m.shr(1);
      return s + 1;
    }
  }
  return s;
}
// deltaInv[i] for p = base^exp + 1: the big.Float chain of newEncoder, Float64() of each term,
// zeroed below 2^-50 / (base * exp)
inline std::vector<double> compute_delta_inv(uint64_t base, int exp) {
  BigU p;
  p.w = {1};
  for (int i = 0; i < exp; ++i) p.mul32((uint32_t)base);
  const int pbits_pow = p.bits();  // bitlen(b^exp): prec of bFloat
  p.add1();
  const int prec = p.bits();  // prec of pFloat, and of every result (encoder.go:51-57)
  (void)pbits_pow;
  // 1 / p at prec bits: floor(2^K / p) with K = prec + bitlen(p) + 2, then rounded
  const int K = 2 * prec + 2;
  BigU num;
  num.w.assign((size_t)(K / 32 + 2), 0);
  BigU q;
  q.w.assign(num.w.size(), 0);
  // bit-serial long division of 2^K by p
  BigU r;
  r.w.assign(p.w.size() + 1, 0);
  auto r_geq_p = [&]() {
    for (int i = (int)std::max(r.w.size(), p.w.size()) - 1; i >= 0; --i) {
      const uint32_t a = i < (int)r.w.size() ? r.w[i] : 0, b = i < (int)p.w.size() ? p.w[i] : 0;
      if (a != b) return a > b;
    }
    return true;
  };
  auto r_sub_p = [&]() {
    int64_t br = 0;
    for (size_t i = 0; i < r.w.size(); ++i) {
      int64_t t = (int64_t)r.w[i] - (i < p.w.size() ? p.w[i] : 0) - br;
      br = t < 0;
      r.w[i] = (uint32_t)(t + (br << 32));
    }
  };
  for (int i = K; i >= 0; --i) {
    // r = 2 r + bit_i(2^K)
    uint32_t c = (i == K) ? 1 : 0;
    for (auto& x : r.w) {
      const uint32_t nc = x >> 31;
      x = (x << 1) | c;
      c = nc;
    }
    if (r_geq_p()) {
      r_sub_p();
      q.w[i >> 5] |= 1u << (i & 31);
    }
  }
  // 1/p = q * 2^-K + rem: round (q with sticky remainder) to prec bits
  bool sticky = false;
  for (auto x : r.w) sticky |= x != 0;
  int e = -K;
  {
    const int nb = q.bits();
    const int s = nb - prec;
    const bool half = q.bit(s - 1), rest = q.any_below(s - 1) || sticky;
    q.shr(s);
    e += s;
    if (half && (rest || q.bit(0))) {
      q.add1();
      if (q.bits() > prec) {
        q.shr(1);
        ++e;
      }
    }
  }
  const double thr = std::exp2(-50.0) / ((double)base * (double)exp);
  std::vector<double> out;
  BigU m = q;
  for (int i = 0; i < exp; ++i) {
    // Float64(): round m to 53 bits, value = -(m53 * 2^(e + s))
    BigU m53 = m;
    const int s = round_to(m53, 53);
    uint64_t mm = 0;
    for (int k = 1; k >= 0; --k) mm = (mm << 32) | (k < (int)m53.w.size() ? m53.w[k] : 0);
    double d = -std::ldexp((double)mm, e + s);
    if (std::fabs(d) < thr) d = 0.0;
    out.push_back(d);
    m.mul32((uint32_t)base);  // pFloatInv.Mul(pFloatInv, bFloat): exact product, rounded to prec
    e += round_to(m, prec);
  }
  return out;
}

#pragma clang fp contract(on)

}  // namespace rg
