// csprng.hpp -- the reference's samplers (math/csprng) on gfx950.
//
// UniformSampler (uniform.go:38-100): key = SHA-384(seed)[0:32], IV = [32:48], AES-256-CTR
// with a 128-bit big-endian counter; Sample() reads little-endian u64 words out of an 8192-byte
// buffer that every refill XORs the next keystream chunk into (XORKeyStream(buf, buf)), so word
// w of chunk c is KS_0[w] ^ ... ^ KS_c[w].  On the device a sampler INSTANCE is a window of one
// domain's counter space: instance n (any u64) starts at counter IV + n * 2^24 (a 128-bit sum) and is exactly the Go
// UniformSampler whose IV is that counter.  Words are computed on demand (one AES block per two
// words); an instance rarely reads past its first 1024 words, and when it does the XOR of the
// earlier chunks is recomputed.
//
// AES-256 runs from T-tables Te0 and Te1 = ror8 Te0 held in LDS, replicated 32 times so that lane
// l reads replica l % 32 (conflict-free) at byte offset (x << 8) | (Te1 ? 0x80 : 0) | ((l % 32) << 2),
// which one v_perm forms from the state word: 64 KiB per workgroup.
// Keys come from kernel arguments (SGPRs) or LDS.
//
// Samplers (each a literal restatement, floats in IEEE double without contraction):
//   TwinCDT.Sample        gaussian_twin_cdt.go:77-112 (tables from the host, global memory)
//   RoundedGaussian       gaussian_rounded.go:77-125 (normFloat ziggurat, tables from the host)
//   COSAC.Sample          gaussian_cosac.go:22-57
//   Uint.SetRandom        jindo/internal/zp/element.go:299-343 (crypto/rand -> a domain window)
#pragma once
#include <stdint.h>

#include "ntt64.hpp"

namespace rg {

constexpr int kAesRep = 32;              // replicas of Te0 and Te1: lane l reads replica l % 32
constexpr int kAesLds = 256 * kAesRep * 2;  // u32 words: per x, 32 x Te0[x] then 32 x Te1[x] (64 KiB)
constexpr int kWinShift = 24;            // blocks per sampler instance: 2^24 (256 MiB of keystream)
constexpr int kKeyWords = 128;           // an AES key staged in LDS: rk[60], iv[4], rol16(rk)[60], pad

struct AesKey {
  uint32_t rk[60];
  uint32_t iv[4];  // big-endian words, iv[0] most significant
};

#if defined(__HIPCC__)
#pragma clang fp contract(off)

__device__ __forceinline__ uint32_t ror32(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
// a ^ b ^ c in one instruction (gfx950 v_bitop3_b32, truth table 0x96); the compiler does not
// form it from xor chains
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// fill the workgroup's LDS T-tables: Te0[x] of replica r at byte (x << 8) | (r << 2), Te1[x] =
// ror8 Te0[x] at (x << 8) | 0x80 | (r << 2) (call by all threads, then sync)
__device__ __forceinline__ void aes_lds_fill(uint32_t* lds, const uint32_t* te0) {
  for (int i = threadIdx.x; i < kAesLds; i += blockDim.x) {
    const uint32_t t = te0[i >> 6];
    lds[i] = (i & 32) ? ror32(t, 8) : t;
  }
}
// stage one key (round keys, IV, round keys rotated left by 16) in LDS: kKeyWords words
__device__ __forceinline__ void aes_key_fill(uint32_t* dst, const AesKey& k) {
  for (int i = threadIdx.x; i < kKeyWords; i += blockDim.x)
    dst[i] = i < 60 ? k.rk[i] : i < 64 ? k.iv[i - 60] : i < 124 ? ror32(k.rk[i - 64], 16) : 0u;
}

// Key sources: a key in LDS (per-lane pointer: lanes may use different keys) or a kernel
// argument whose words the compiler keeps in SGPRs.
struct LdsKey {
  const uint32_t* p;
  __device__ __forceinline__ uint32_t rk(int i) const { return p[i]; }
  __device__ __forceinline__ uint32_t iv(int i) const { return p[60 + i]; }
  __device__ __forceinline__ uint32_t rkr(int i) const { return p[64 + i]; }  // rol16(rk[i])
};
struct ArgKey {
  const AesKey& k;
  __device__ __forceinline__ uint32_t rk(int i) const { return k.rk[i]; }
  __device__ __forceinline__ uint32_t iv(int i) const { return k.iv[i]; }
  __device__ __forceinline__ uint32_t rkr(int i) const { return ror32(k.rk[i], 16); }
};

// T-table lookup of byte `B` of s: the LDS byte offset (byte << 8) | lo is one v_perm (byte 1 <-
// s.byte B, byte 0 <- lo, bytes 2-3 <- 0) with lo = (lane % 32) << 2 for Te0, | 0x80 for Te1;
// ds_read_b32 bank = lane % 32: conflict-free
template <int B>
__device__ __forceinline__ uint32_t te_b(const uint32_t* lds, uint32_t s, uint32_t lo) {
  const uint32_t off = __builtin_amdgcn_perm(s, lo, 0x0C0C0000u | ((4u + B) << 8));
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + off);
}

// AES-256 of the counter block IV + n, n = nhi 2^64 + nlo (128-bit big-endian add, as Go's
// crypto/cipher CTR increments the whole block); returns the 16 keystream bytes as 4 big-endian words.
// Round column: Te0[a] ^ ror8 Te0[b] ^ ror16 Te0[c] ^ ror24 Te0[d] ^ k
//             = Te0[a] ^ Te1[b] ^ ror16(Te0[c] ^ Te1[d] ^ rol16 k)   (rotation is linear in ^)
// = 4 v_perm + 2 v_bitop3 + 1 rotate per column.
template <class K>
__device__ __forceinline__ void aes_ctr(const K& key, uint64_t nhi, uint64_t nlo, const uint32_t* lds, uint32_t out[4]) {
  const uint32_t l0 = (threadIdx.x & 31u) << 2, l1 = l0 | 0x80u;
  const uint64_t ivlo = ((uint64_t)key.iv(2) << 32) | key.iv(3), ivhi = ((uint64_t)key.iv(0) << 32) | key.iv(1);
  const uint64_t lo = ivlo + nlo;
  const uint64_t hi = ivhi + nhi + (lo < nlo ? 1u : 0u);
  uint32_t s0 = (uint32_t)(hi >> 32) ^ key.rk(0), s1 = (uint32_t)hi ^ key.rk(1), s2 = (uint32_t)(lo >> 32) ^ key.rk(2),
           s3 = (uint32_t)lo ^ key.rk(3);
  auto col = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t kr) {
    return xor3(te_b<3>(lds, a, l0), te_b<2>(lds, b, l1), ror32(xor3(te_b<1>(lds, c, l0), te_b<0>(lds, d, l1), kr), 16));
  };
#pragma unroll
  for (int r = 1; r < 14; ++r) {
    const uint32_t t0 = col(s0, s1, s2, s3, key.rkr(4 * r));
    const uint32_t t1 = col(s1, s2, s3, s0, key.rkr(4 * r + 1));
    const uint32_t t2 = col(s2, s3, s0, s1, key.rkr(4 * r + 2));
    const uint32_t t3 = col(s3, s0, s1, s2, key.rkr(4 * r + 3));
    s0 = t0;
    s1 = t1;
    s2 = t2;
    s3 = t3;
  }
  // final round: S-box bytes (byte 2 of Te0[x] is S[x]) gathered with v_perm, no MixColumns
  auto fin = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
    const uint32_t ab = __builtin_amdgcn_perm(te_b<3>(lds, a, l0), te_b<2>(lds, b, l0), 0x06020C0Cu);
    const uint32_t cd = __builtin_amdgcn_perm(te_b<1>(lds, c, l0), te_b<0>(lds, d, l0), 0x0C0C0602u);
    return xor3(ab, cd, k);
  };
  out[0] = fin(s0, s1, s2, s3, key.rk(56));
  out[1] = fin(s1, s2, s3, s0, key.rk(57));
  out[2] = fin(s2, s3, s0, s1, key.rk(58));
  out[3] = fin(s3, s0, s1, s2, key.rk(59));
}

// Two blocks of one key in lockstep: each round issues both blocks' 32 table lookups together
// (twice the loads in flight of one block) and reads the round key once for both.
template <class K>
__device__ __forceinline__ void aes_ctr_x2(const K& key, uint64_t hi0, uint64_t lo0, uint64_t hi1, uint64_t lo1,
                                           const uint32_t* lds, uint32_t o0[4], uint32_t o1[4]) {
  const uint32_t l0 = (threadIdx.x & 31u) << 2, l1 = l0 | 0x80u;
  const uint64_t ivlo = ((uint64_t)key.iv(2) << 32) | key.iv(3), ivhi = ((uint64_t)key.iv(0) << 32) | key.iv(1);
  const uint64_t c0 = ivlo + lo0, c1 = ivlo + lo1;
  const uint64_t h0 = ivhi + hi0 + (c0 < lo0 ? 1u : 0u), h1 = ivhi + hi1 + (c1 < lo1 ? 1u : 0u);
  const uint32_t k0 = key.rk(0), k1 = key.rk(1), k2 = key.rk(2), k3 = key.rk(3);
  uint32_t a0 = (uint32_t)(h0 >> 32) ^ k0, a1 = (uint32_t)h0 ^ k1, a2 = (uint32_t)(c0 >> 32) ^ k2, a3 = (uint32_t)c0 ^ k3;
  uint32_t b0 = (uint32_t)(h1 >> 32) ^ k0, b1 = (uint32_t)h1 ^ k1, b2 = (uint32_t)(c1 >> 32) ^ k2, b3 = (uint32_t)c1 ^ k3;
  auto col = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t kr) {
    return xor3(te_b<3>(lds, a, l0), te_b<2>(lds, b, l1), ror32(xor3(te_b<1>(lds, c, l0), te_b<0>(lds, d, l1), kr), 16));
  };
#pragma unroll
  for (int r = 1; r < 14; ++r) {
    const uint32_t r0 = key.rkr(4 * r), r1 = key.rkr(4 * r + 1), r2 = key.rkr(4 * r + 2), r3 = key.rkr(4 * r + 3);
    const uint32_t ta0 = col(a0, a1, a2, a3, r0), tb0 = col(b0, b1, b2, b3, r0);
    const uint32_t ta1 = col(a1, a2, a3, a0, r1), tb1 = col(b1, b2, b3, b0, r1);
    const uint32_t ta2 = col(a2, a3, a0, a1, r2), tb2 = col(b2, b3, b0, b1, r2);
    const uint32_t ta3 = col(a3, a0, a1, a2, r3), tb3 = col(b3, b0, b1, b2, r3);
    a0 = ta0; a1 = ta1; a2 = ta2; a3 = ta3;
    b0 = tb0; b1 = tb1; b2 = tb2; b3 = tb3;
  }
  auto fin = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
    const uint32_t ab = __builtin_amdgcn_perm(te_b<3>(lds, a, l0), te_b<2>(lds, b, l0), 0x06020C0Cu);
    const uint32_t cd = __builtin_amdgcn_perm(te_b<1>(lds, c, l0), te_b<0>(lds, d, l0), 0x0C0C0602u);
    return xor3(ab, cd, k);
  };
  const uint32_t f0 = key.rk(56), f1 = key.rk(57), f2 = key.rk(58), f3 = key.rk(59);
  o0[0] = fin(a0, a1, a2, a3, f0);
  o1[0] = fin(b0, b1, b2, b3, f0);
  o0[1] = fin(a1, a2, a3, a0, f1);
  o1[1] = fin(b1, b2, b3, b0, f1);
  o0[2] = fin(a2, a3, a0, a1, f2);
  o1[2] = fin(b2, b3, b0, b1, f2);
  o0[3] = fin(a3, a0, a1, a2, f3);
  o1[3] = fin(b3, b0, b1, b2, f3);
}

// The two little-endian u64 keystream words of block `off` of instance `inst`'s window, i.e. of
// counter block IV + inst 2^24 + off.  inst 2^24 is formed in 128 bits (hi = inst >> 40): an
// instance number up to 2^64 - 1 never wraps onto another instance's window (oracle.c uni_init).
template <class K>
__device__ __forceinline__ void ks_words(const K& key, uint64_t inst, uint64_t off, const uint32_t* lds, uint64_t& w0,
                                         uint64_t& w1) {
  const uint64_t wlo = inst << kWinShift, lo = wlo + off;
  const uint64_t hi = (inst >> (64 - kWinShift)) + (lo < wlo ? 1u : 0u);
  uint32_t o[4];
  aes_ctr(key, hi, lo, lds, o);
  w0 = (uint64_t)bswap32(o[0]) | ((uint64_t)bswap32(o[1]) << 32);
  w1 = (uint64_t)bswap32(o[2]) | ((uint64_t)bswap32(o[3]) << 32);
}
__device__ __forceinline__ void ks_words(const AesKey& K, uint64_t inst, uint64_t off, const uint32_t* lds, uint64_t& w0,
                                         uint64_t& w1) {
  ks_words(ArgKey{K}, inst, off, lds, w0, w1);
}

// blocks off0 and off1 of one instance's window (ks_words for both, in lockstep)
template <class K>
__device__ __forceinline__ void ks_words_x2(const K& key, uint64_t inst, uint64_t off0, uint64_t off1,
                                            const uint32_t* lds, uint64_t w[4]) {
  const uint64_t wlo = inst << kWinShift, lo0 = wlo + off0, lo1 = wlo + off1, whi = inst >> (64 - kWinShift);
  uint32_t a[4], b[4];
  aes_ctr_x2(key, whi + (lo0 < wlo ? 1u : 0u), lo0, whi + (lo1 < wlo ? 1u : 0u), lo1, lds, a, b);
  w[0] = (uint64_t)bswap32(a[0]) | ((uint64_t)bswap32(a[1]) << 32);
  w[1] = (uint64_t)bswap32(a[2]) | ((uint64_t)bswap32(a[3]) << 32);
  w[2] = (uint64_t)bswap32(b[0]) | ((uint64_t)bswap32(b[1]) << 32);
  w[3] = (uint64_t)bswap32(b[2]) | ((uint64_t)bswap32(b[3]) << 32);
}

// word `p` of the Sample() stream of instance `inst` (uniform.go:64-82): chunk c = KS_0 ^ ... ^ KS_c
__device__ __noinline__ uint64_t uniform_word_at(LdsKey key, const uint32_t* lds, uint64_t inst, uint64_t p) {
  const uint64_t c = p >> 10, o = p & 1023u;
  uint64_t x = 0;
  for (uint64_t i = 0; i <= c; ++i) {
    uint64_t w0, w1;
    ks_words(key, inst, ((i << 10) + o) / 2, lds, w0, w1);
    x ^= (o & 1) ? w1 : w0;
  }
  return x;
}

// One UniformSampler instance (window `inst` of the domain): Sample(), SampleFloat()
struct Uniform {
  LdsKey key;
  const uint32_t* lds;
  uint64_t inst;  // the instance (its window starts at block inst 2^24)
  uint64_t pos;   // next word
  uint64_t spare;
  bool have_spare;

  __device__ __forceinline__ void init(const uint32_t* key_lds, const uint32_t* l, uint64_t instance) {
    key.p = key_lds;
    lds = l;
    inst = instance;
    pos = 0;
    have_spare = false;
  }
  __device__ uint64_t word_at(uint64_t p) const { return uniform_word_at(key, lds, inst, p); }
  __device__ __forceinline__ uint64_t sample() {
    uint64_t r;
    if (have_spare) {
      r = spare;
      have_spare = false;
    } else if (pos < 1024 && !(pos & 1)) {
      uint64_t w0, w1;
      ks_words(key, inst, pos / 2, lds, w0, w1);
      r = w0;
      spare = w1;
      have_spare = true;
    } else {
      r = word_at(pos);
    }
    ++pos;
    return r;
  }
  __device__ __forceinline__ double sample_float() {  // uniform.go:95-100: (Sample() mod 2^52) / 2^52
    return (double)(sample() & 0xFFFFFFFFFFFFFull) * 2.220446049250313e-16;
  }
};

// slices.BinarySearch(table, u): smallest i with table[i] >= u; found -> i - 1 (twin_cdt.go:88-95)
__device__ __forceinline__ int64_t cdt_search(const uint64_t* t, int n, uint64_t u) {
  int i = 0, j = n;
  while (i < j) {
    const int h = (int)((unsigned)(i + j) >> 1);
    if (t[h] < u)
      i = h + 1;
    else
      j = h;
  }
  return (i < n && t[i] == u) ? i - 1 : i;
}

struct CdtDev {
  const uint64_t* tables;  // [128][size]
  const uint8_t* guide;    // [128][257]: lower_bound of t * 2^56 (size <= 255), or null
  int size;
  int64_t tail_lo;
  double sigma;
};

// TwinCDTGaussianSampler.Sample(center) with the instance's next word u (twin_cdt.go:77-112)
__device__ int64_t twin_cdt(const CdtDev& C, double center, uint64_t u) {
  const double c_floor = floor(center);
  const double c_frac = center - c_floor;
  const int64_t c0 = (int64_t)floor(128.0 * c_frac) % 128;
  const int64_t c1 = (int64_t)ceil(128.0 * c_frac) % 128;
  const int64_t v0 = cdt_search(C.tables + c0 * C.size, C.size, u);
  const int64_t v1 = c1 == c0 ? v0 : cdt_search(C.tables + c1 * C.size, C.size, u);
  if (v0 == v1) return v0 + (int64_t)c_floor + C.tail_lo;
  double cdf = 0.0;
  const double norm = sqrt(2.0 * M_PI) * C.sigma;
  for (int64_t x = C.tail_lo; x <= v0; ++x) {  // sic: x runs over values up to the INDEX v0
    const double xf = (double)x;
    cdf += exp(-(xf - c_frac) * (xf - c_frac) / (2.0 * C.sigma * C.sigma)) / norm;
  }
  const double p = __ull2double_rn(u) / 18446744073709551616.0;
  return (p < cdf ? v0 : v1) + C.tail_lo + (int64_t)c_floor;
}

struct ZigDev {
  const uint64_t* kn;
  const double* wn;
  const double* fn;
};

// RoundedGaussianSampler.normFloat (gaussian_rounded.go:77-116)
__device__ double norm_float(const ZigDev& Z, Uniform& U) {
  const double rn = 3.442619855899;
  for (;;) {
    const uint64_t r = U.sample();
    const uint64_t b = r >> 63;
    const uint32_t i = (uint32_t)(r & 127u);
    const uint64_t j = (r >> 7) & 0xFFFFFFFFFFFFFull;
    const double x = (double)(int64_t)((j ^ (0ull - b)) + b) * Z.wn[i];
    if (j < Z.kn[i]) return x;
    if (i == 0) {
      double u, v;
      for (;;) {
        u = -log(U.sample_float()) * (1.0 / rn);
        v = -log(U.sample_float());
        if (v + v >= u * u) break;
      }
      u += rn;
      return b == 1 ? -u : u;
    }
    const double f0 = Z.fn[i - 1], f1 = Z.fn[i];
    if (U.sample_float() * (f0 - f1) < exp(-0.5 * x * x) - f1) return x;
  }
}

// RoundedGaussianSampler.Sample(center, stdDev) (gaussian_rounded.go:118-125)
__device__ __forceinline__ int64_t rounded_gauss(const ZigDev& Z, Uniform& U, double center, double sd) {
  return (int64_t)round(center + norm_float(Z, U) * sd);
}

// COSACSampler.Sample(center, stdDev) (gaussian_cosac.go:22-57): `base` is the sampler's own
// UniformSampler, `rnd` the one inside its RoundedGaussianSampler
__device__ int64_t cosac(const ZigDev& Z, Uniform& base, Uniform& rnd, double center, double sd) {
  const double c_int = round(center);
  const double c_frac = c_int - center;
  const double r = base.sample_float();
  if (r < exp(-(c_frac * c_frac) / (2.0 * sd * sd)) / (sqrt(2.0 * M_PI) * sd)) return (int64_t)c_int;
  for (;;) {
    const double y = sd * norm_float(Z, rnd);
    const uint64_t b = base.sample() & 1;
    double y_round;
    bool cmp;
    if (b == 0) {
      y_round = round(y) - 1.0;
      cmp = y_round <= 0.5;
    } else {
      y_round = round(y) + 1.0;
      cmp = y_round >= -0.5;
    }
    if (cmp) {
      const double rr = base.sample_float();
      if (rr < exp(-((y_round + c_frac) * (y_round + c_frac) - y * y) / (2.0 * sd * sd)))
        return (int64_t)y_round + (int64_t)c_int;
    }
  }
}

#pragma clang fp contract(on)
#endif  // __HIPCC__

}  // namespace rg
