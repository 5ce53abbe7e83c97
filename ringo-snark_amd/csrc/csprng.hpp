// csprng.hpp -- the reference's samplers (math/csprng) on gfx950.
//
// UniformSampler (uniform.go:38-100): key = SHA-384(seed)[0:32], IV = [32:48], AES-256-CTR
// with a 128-bit big-endian counter; Sample() reads little-endian u64 words out of an 8192-byte
// buffer that every refill XORs the next keystream chunk into (XORKeyStream(buf, buf)), so word
// w of chunk c is KS_0[w] ^ ... ^ KS_c[w].  On the device a sampler INSTANCE is a window of one
// domain's counter space: instance n starts at counter IV + n * 2^24 and is exactly the Go
// UniformSampler whose IV is that counter.  Words are computed on demand (one AES block per two
// words); an instance rarely reads past its first 1024 words, and when it does the XOR of the
// earlier chunks is recomputed.
//
// AES-256 runs from a T-table held in LDS, replicated 32 times so that lane l always reads
// bank l & 31 (conflict-free): 32 KiB per workgroup.
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

constexpr int kAesLds = 256 * 32;  // u32 words of the replicated T-table
constexpr int kWinShift = 24;      // blocks per sampler instance: 2^24 (256 MiB of keystream)

struct AesKey {
  uint32_t rk[60];
  uint32_t iv[4];  // big-endian words, iv[0] most significant
};

#if defined(__HIPCC__)
#pragma clang fp contract(off)

__device__ __forceinline__ uint32_t ror32(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// fill the workgroup's LDS T-table copy (call by all threads, then __syncthreads)
__device__ __forceinline__ void aes_lds_fill(uint32_t* lds, const uint32_t* te0) {
  for (int i = threadIdx.x; i < kAesLds; i += blockDim.x) lds[i] = te0[i >> 5];
}

__device__ __forceinline__ uint32_t te(const uint32_t* lds, uint32_t x, uint32_t lane) { return lds[(x << 5) | lane]; }

// AES-256 of the counter block IV + n; returns the 16 keystream bytes as 4 big-endian words
__device__ __forceinline__ void aes_ctr(const AesKey& K, uint64_t n, const uint32_t* lds, uint32_t out[4]) {
  const uint32_t lane = threadIdx.x & 31u;
  const uint64_t lo = (((uint64_t)K.iv[2] << 32) | K.iv[3]) + n;
  const uint64_t hi = (((uint64_t)K.iv[0] << 32) | K.iv[1]) + (lo < n ? 1u : 0u);
  uint32_t s0 = (uint32_t)(hi >> 32) ^ K.rk[0], s1 = (uint32_t)hi ^ K.rk[1], s2 = (uint32_t)(lo >> 32) ^ K.rk[2],
           s3 = (uint32_t)lo ^ K.rk[3];
#pragma unroll
  for (int r = 1; r < 14; ++r) {
    const uint32_t t0 = te(lds, s0 >> 24, lane) ^ ror32(te(lds, (s1 >> 16) & 255u, lane), 8) ^
                        ror32(te(lds, (s2 >> 8) & 255u, lane), 16) ^ ror32(te(lds, s3 & 255u, lane), 24) ^ K.rk[4 * r];
    const uint32_t t1 = te(lds, s1 >> 24, lane) ^ ror32(te(lds, (s2 >> 16) & 255u, lane), 8) ^
                        ror32(te(lds, (s3 >> 8) & 255u, lane), 16) ^ ror32(te(lds, s0 & 255u, lane), 24) ^
                        K.rk[4 * r + 1];
    const uint32_t t2 = te(lds, s2 >> 24, lane) ^ ror32(te(lds, (s3 >> 16) & 255u, lane), 8) ^
                        ror32(te(lds, (s0 >> 8) & 255u, lane), 16) ^ ror32(te(lds, s1 & 255u, lane), 24) ^
                        K.rk[4 * r + 2];
    const uint32_t t3 = te(lds, s3 >> 24, lane) ^ ror32(te(lds, (s0 >> 16) & 255u, lane), 8) ^
                        ror32(te(lds, (s1 >> 8) & 255u, lane), 16) ^ ror32(te(lds, s2 & 255u, lane), 24) ^
                        K.rk[4 * r + 3];
    s0 = t0;
    s1 = t1;
    s2 = t2;
    s3 = t3;
  }
  // final round: S-box bytes (byte 2 of Te0[x] is S[x]), no MixColumns
  auto sb = [&](uint32_t x) { return (te(lds, x, lane) >> 16) & 255u; };
  out[0] = ((sb(s0 >> 24) << 24) | (sb((s1 >> 16) & 255u) << 16) | (sb((s2 >> 8) & 255u) << 8) | sb(s3 & 255u)) ^ K.rk[56];
  out[1] = ((sb(s1 >> 24) << 24) | (sb((s2 >> 16) & 255u) << 16) | (sb((s3 >> 8) & 255u) << 8) | sb(s0 & 255u)) ^ K.rk[57];
  out[2] = ((sb(s2 >> 24) << 24) | (sb((s3 >> 16) & 255u) << 16) | (sb((s0 >> 8) & 255u) << 8) | sb(s1 & 255u)) ^ K.rk[58];
  out[3] = ((sb(s3 >> 24) << 24) | (sb((s0 >> 16) & 255u) << 16) | (sb((s1 >> 8) & 255u) << 8) | sb(s2 & 255u)) ^ K.rk[59];
}

// the two little-endian u64 keystream words of block n
__device__ __forceinline__ void ks_words(const AesKey& K, uint64_t n, const uint32_t* lds, uint64_t& w0, uint64_t& w1) {
  uint32_t o[4];
  aes_ctr(K, n, lds, o);
  w0 = (uint64_t)bswap32(o[0]) | ((uint64_t)bswap32(o[1]) << 32);
  w1 = (uint64_t)bswap32(o[2]) | ((uint64_t)bswap32(o[3]) << 32);
}

// One UniformSampler instance (window `inst` of the domain): Sample(), SampleFloat()
struct Uniform {
  const AesKey* K;
  const uint32_t* lds;
  uint64_t base;  // first block of the window
  uint64_t pos;   // next word
  uint64_t spare;
  bool have_spare;

  __device__ __forceinline__ void init(const AesKey& key, const uint32_t* l, uint64_t inst) {
    K = &key;
    lds = l;
    base = inst << kWinShift;
    pos = 0;
    have_spare = false;
  }
  // word `p` of the instance's Sample() stream (uniform.go:64-82)
  __device__ uint64_t word_at(uint64_t p) const {
    const uint64_t c = p >> 10, o = p & 1023u;
    uint64_t x = 0;
    for (uint64_t i = 0; i <= c; ++i) {  // chunk c = KS_0 ^ ... ^ KS_c (c = 0 in practice)
      uint64_t w0, w1;
      ks_words(*K, base + ((i << 10) + o) / 2, lds, w0, w1);
      x ^= (o & 1) ? w1 : w0;
    }
    return x;
  }
  __device__ __forceinline__ uint64_t sample() {
    uint64_t r;
    if (have_spare) {
      r = spare;
      have_spare = false;
    } else if (pos < 1024 && !(pos & 1)) {
      uint64_t w0, w1;
      ks_words(*K, base + pos / 2, lds, w0, w1);
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
