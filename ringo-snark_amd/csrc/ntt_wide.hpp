// ntt_wide.hpp -- LDS-tiled pass kernel for the wide Buckler fields (zp440: L = 7, zp880: L = 14
// 64-bit limbs), the NTT math/bigpoly/ntt.go:98-136,206-244 runs for buckler_test.go:163-222.
//
// Cost model.  A 14-limb Montgomery product is ~3,100 half-rate VALU operations, so at these
// widths the transform is bound by the multiplier, not by HBM: a 2^16-point zp880 transform is
// ~0.5 G wave-lane multiplies against 7.3 MB of data.  What the one-launch-per-stage kernel
// (ntt_stage_kernel) wasted was 16 HBM round trips per transform plus a 64-bit-limb CIOS with
// explicit compare-based carries.  Here:
//   * passes of P <= 8 stages (N = 2^16: COL 8 + ROW 8, N = 2^15: 7 + 8, N <= 2^8: one pass):
//     a workgroup loads `cpt` sub-transforms (2^P points at stride S) into limb-planar LDS, runs
//     the P radix-2 stages with one butterfly per thread per step and a barrier between stages,
//     and writes the tile back -- HBM sees one read and one write per element per pass;
//   * the product is Montgomery on 28-bit digits (mont28), product scanning with one 64-bit column
//     accumulator: one v_mad_u64_u32 per partial product and no carry handling (the round-4
//     32-bit-digit form, a v_mad_u64_u32 plus a v_addc per product, is
//     tools/experiments/wide_mont32.patch);
//   * every value stays canonical in [0, q) (one conditional subtract per add / sub / product:
//     ~3 D operations against ~4 D^2 for the product), so limbs equal the reference's.
// Twiddles are the reference's Montgomery tables tw[m + i] / twInv[m + i], read from L2.  The
// inverse halves every stage ((u + v) / 2, (u - v) twInv[m + i] / 2 from a halved copy of the
// table) instead of multiplying by N^-1 after the last one: log N halvings are N^-1, a halving is
// ~3 D operations, and the butterfly keeps ONE product site (a second one for the N^-1 factor
// doubled the I-cache footprint and pushed the 14-limb kernel past 256 VGPRs).  Requires
// q < 2^(64L - 1) (checked by the launcher), so a Montgomery product of canonical inputs is
// < 2q < 2^(64L).
#pragma once
#include <stdint.h>

#include "common.hpp"
#include "ntt64.hpp"

namespace rg {

constexpr int kWideThreads = 128;  // threads per workgroup
constexpr int kWideMaxL = 14;

struct WideArgs {
  const uint64_t* in;
  uint64_t* out;
  const uint64_t* tw;  // Montgomery [N][L]: tw (forward) or twInv / 2 (inverse)
  uint32_t q[2 * kWideMaxL];
  uint32_t q28[64 * kWideMaxL / 28];  // q in 28-bit digits (mont28)
  uint32_t qinv28;                    // -q^-1 mod 2^28
  int logN, G0, P, logS, cpt;  // pass: global stages [G0, G0 + P), points at stride 2^logS
  long long nsub;              // sub-transforms of the pass over the batch
};

#if defined(__HIPCC__)

// (static_for, common.hpp: the products are hundreds of partial products, past what the loop
// unroller fully unrolls, and a rolled loop indexes the digit arrays dynamically)
// z = x y 2^(-64 L) mod q, canonical, for canonical x, y and q < 2^(64 L - 1): Montgomery on
// 28-bit digits (K = 64 L / 28: 16 for L = 7, 32 for L = 14; R = 2^(28 K) = 2^(64 L), so the
// reference's Montgomery tables serve unchanged).  A 28-bit digit product is < 2^56,
// so a column of up to 2 K products plus the carry stays below 2^63 in one 64-bit accumulator:
// no carry-out per partial product (the 32-bit-digit form pays a v_addc for each), and the
// products are plain C that hipcc schedules and pads itself.  Digits are cut from and packed
// back into the 32-bit words around the product (~2 operations per word each way).
template <int L>
__device__ __forceinline__ void to28(uint32_t (&d)[64 * L / 28], const uint32_t (&w)[2 * L]) {
  constexpr int K = 64 * L / 28, D = 2 * L;
  static_for<K>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int j = (28 * k) >> 5, sh = (28 * k) & 31;
    if constexpr (sh <= 4 || j + 1 >= D)
      d[k] = (w[j] >> sh) & 0x0FFFFFFFu;
    else
      d[k] = __builtin_amdgcn_alignbit(w[j + 1], w[j], sh) & 0x0FFFFFFFu;
  });
}
template <int L>
__device__ __forceinline__ void from28(uint32_t (&w)[2 * L], const uint32_t (&d)[64 * L / 28]) {
  constexpr int K = 64 * L / 28, D = 2 * L;
  static_for<D>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    constexpr int k0 = (32 * j) / 28, off = 32 * j - 28 * k0;  // word j starts at bit off of digit k0
    uint32_t v = d[k0] >> off;
    if constexpr (k0 + 1 < K) v |= d[k0 + 1] << (28 - off);
    if constexpr (k0 + 2 < K && 56 - off < 32) v |= d[k0 + 2] << (56 - off);
    w[j] = v;
  });
}
template <int L>
__device__ __forceinline__ void mont28(uint32_t (&z)[2 * L], const uint32_t (&x)[2 * L], const uint32_t (&y)[2 * L],
                                       const uint32_t (&q)[2 * L], const uint32_t* q28, uint32_t qi28) {
  constexpr int K = 64 * L / 28, D = 2 * L;
  static_assert(64 * L % 28 == 0, "digit split");
  uint32_t xd[K], yd[K], m[K], zd[K];
  to28<L>(xd, x);
  to28<L>(yd, y);
  uint64_t C = 0;  // carry into the column: the previous column's sum >> 28
  static_for<2 * K - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int xlo = k < K ? 0 : k - K + 1, xhi = k < K ? k : K - 1;
    constexpr int mlo = k < K ? 0 : k - K + 1, mhi = k < K ? k - 1 : K - 1;  // m q, j = k - i >= 1
    // two chains (x y, m q) for the SIMD's latency at 2 waves
    uint64_t A = C, B = 0;
    static_for<xhi - xlo + 1>([&](auto ic) {
      constexpr int i = xlo + decltype(ic)::value;
      A = (uint64_t)xd[i] * yd[k - i] + A;
    });
    if constexpr (mhi >= mlo)
      static_for<mhi - mlo + 1>([&](auto ic) {
        constexpr int i = mlo + decltype(ic)::value;
        B = (uint64_t)m[i] * q28[k - i] + B;
      });
    uint64_t t = A + B;
    if constexpr (k < K) {  // quotient digit: clears the column's 28 low bits
      m[k] = ((uint32_t)t * qi28) & 0x0FFFFFFFu;
      t = (uint64_t)m[k] * q28[0] + t;
    } else {
      zd[k - K] = (uint32_t)t & 0x0FFFFFFFu;
    }
    C = t >> 28;
  });
  zd[K - 1] = (uint32_t)C;
  from28<L>(z, zd);
  // [0, 2q) -> [0, q)
  uint32_t u[D];
  lmask b;
  u[0] = sub_co(z[0], q[0], b);
#pragma unroll
  for (int i = 1; i < D; ++i) u[i] = subb_co(z[i], q[i], b, b);
#pragma unroll
  for (int i = 0; i < D; ++i) z[i] = sel(b, z[i], u[i]);
}

template <int D>
__device__ __forceinline__ void add_wide(uint32_t (&r)[D], const uint32_t (&x)[D], const uint32_t (&y)[D],
                                         const uint32_t (&q)[D]) {
  uint32_t s[D], u[D];
  lmask c, b;
  s[0] = add_co(x[0], y[0], c);
#pragma unroll
  for (int i = 1; i < D; ++i) s[i] = addc_co(x[i], y[i], c, c);
  u[0] = sub_co(s[0], q[0], b);
#pragma unroll
  for (int i = 1; i < D; ++i) u[i] = subb_co(s[i], q[i], b, b);
  const lmask m = c | ~b;
#pragma unroll
  for (int i = 0; i < D; ++i) r[i] = sel(m, u[i], s[i]);
}

template <int D>
__device__ __forceinline__ void sub_wide(uint32_t (&r)[D], const uint32_t (&x)[D], const uint32_t (&y)[D],
                                         const uint32_t (&q)[D]) {
  uint32_t d[D], f[D];
  lmask b, c;
  d[0] = sub_co(x[0], y[0], b);
#pragma unroll
  for (int i = 1; i < D; ++i) d[i] = subb_co(x[i], y[i], b, b);
  f[0] = add_co(d[0], q[0], c);
#pragma unroll
  for (int i = 1; i < D; ++i) f[i] = addc_co(d[i], q[i], c, c);
#pragma unroll
  for (int i = 0; i < D; ++i) r[i] = sel(b, f[i], d[i]);
}

// r = x / 2 mod q for canonical x: (x + (x odd ? q : 0)) >> 1, canonical (x + q < 2q < 2^(32 D))
template <int D>
__device__ __forceinline__ void half_wide(uint32_t (&r)[D], const uint32_t (&x)[D], const uint32_t (&q)[D]) {
  const uint32_t odd = 0u - (x[0] & 1u);
  uint32_t s[D];
  lmask c;
  s[0] = add_co(x[0], q[0] & odd, c);
#pragma unroll
  for (int i = 1; i < D; ++i) s[i] = addc_co(x[i], q[i] & odd, c, c);
#pragma unroll
  for (int i = 0; i + 1 < D; ++i) r[i] = __builtin_amdgcn_alignbit(s[i + 1], s[i], 1);
  r[D - 1] = s[D - 1] >> 1;
}

// One pass over `cpt` sub-transforms per workgroup.  LDS: limb planes of u64, plane l holds
// element (c, x) at c 2^P + x.  Stages are a runtime loop (the body is one butterfly), so P, the
// strides and the pass position are arguments, not template parameters.
template <int L, bool INV>
__global__ __launch_bounds__(kWideThreads, 2) void ntt_wide_pass(WideArgs a) {  // >= 2 waves/SIMD (<= 256 VGPRs)
  constexpr int D = 2 * L;
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  const int P = a.P, NP = 1 << P, cpt = a.cpt, logS = a.logS;
  const int plane = cpt * NP;
  const long long s0 = (long long)blockIdx.x * cpt;
  const int subs_log = a.logN - P;  // log2 sub-transforms per polynomial
  uint32_t q[D];
#pragma unroll
  for (int i = 0; i < D; ++i) q[i] = a.q[i];
  auto mont = [&](uint32_t(&z)[D], const uint32_t(&x)[D], const uint32_t(&y)[D]) {
    mont28<L>(z, x, y, q, a.q28, a.qinv28);
  };
  // global element index of point x of tile sub-transform c (or -1 past the batch)
  auto elem = [&](int c, int x) -> long long {
    const long long s = s0 + c;
    if (s >= a.nsub) return -1;
    const long long b = s >> subs_log, r = s & ((1LL << subs_log) - 1);
    const long long hi = r >> logS, lo = r & ((1LL << logS) - 1);
    return (b << a.logN) | (hi << (a.logN - a.G0)) | ((long long)x << logS) | lo;
  };
  // ---- HBM -> LDS: memory-friendly order (rows: c, x, l; columns: x, c, l)
  const int W = cpt * NP * L;
  for (int f = threadIdx.x; f < W; f += kWideThreads) {
    const int l = f % L, e = f / L;
    const int c = logS == 0 ? e / NP : e % cpt, x = logS == 0 ? e % NP : e / cpt;
    const long long g = elem(c, x);
    if (g >= 0) lds[l * plane + c * NP + x] = a.in[g * L + l];
  }
  __syncthreads();
  // ---- the P stages
  const int nbf = cpt * (NP >> 1);
  // twiddle index of butterfly bf at local stage g
  auto tw_idx = [&](int g, int bf) -> long long {
    const int c = bf >> (P - 1), p = bf & ((NP >> 1) - 1), bitpos = P - 1 - g;
    const int x0 = ((p >> bitpos) << (bitpos + 1)) | (p & ((1 << bitpos) - 1));
    const long long r = (s0 + c) & ((1LL << subs_log) - 1);
    const long long hi = (r >> logS) & ((1LL << a.G0) - 1);
    return (1LL << (a.G0 + g)) + (hi << g) + (x0 >> (bitpos + 1));
  };
  // L = 14: the next butterfly's twiddle is loaded one butterfly ahead (across the stage barrier),
  // so its L2 latency hides behind the current product, which 2 waves/SIMD do not (zp880 +1.3%);
  // L = 7 (4 waves/SIMD) loads it in place (the prefetch's extra VGPRs and index work cost 1%)
  constexpr bool PF = L >= 14;
  uint32_t wn[D];
  auto fetch = [&](long long idx) {
    const uint64_t* tp = a.tw + idx * L;
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const uint64_t t = tp[l];
      wn[2 * l] = lo32(t);
      wn[2 * l + 1] = hi32(t);
    }
  };
  if (PF && (int)threadIdx.x < nbf) fetch(tw_idx(INV ? P - 1 : 0, (int)threadIdx.x));
  for (int st = 0; st < P; ++st) {
    const int g = INV ? P - 1 - st : st;  // local stage (global G0 + g)
    const int bitpos = P - 1 - g;
    for (int bf = threadIdx.x; bf < nbf; bf += kWideThreads) {
      const int c = bf >> (P - 1), p = bf & ((NP >> 1) - 1);
      const int x0 = ((p >> bitpos) << (bitpos + 1)) | (p & ((1 << bitpos) - 1)), x1 = x0 | (1 << bitpos);
      uint32_t u[D], v[D], w[D];
#pragma unroll
      for (int l = 0; l < L; ++l) {
        const uint64_t uu = lds[l * plane + c * NP + x0], vv = lds[l * plane + c * NP + x1];
        u[2 * l] = lo32(uu);
        u[2 * l + 1] = hi32(uu);
        v[2 * l] = lo32(vv);
        v[2 * l + 1] = hi32(vv);
      }
      auto take_w = [&]() {
        if constexpr (!PF) fetch(tw_idx(g, bf));
#pragma unroll
        for (int i = 0; i < D; ++i) w[i] = wn[i];
        if constexpr (PF) {  // the next butterfly of this stage, else this thread's first of the next stage
          int nb = bf + kWideThreads, ns = st;
          if (nb >= nbf) {
            nb = (int)threadIdx.x;
            ++ns;
          }
          if (ns < P) fetch(tw_idx(INV ? P - 1 - ns : ns, nb));
        }
      };
      uint32_t nu[D], nv[D];
      if constexpr (!INV) {  // ntt.go:254-259
        take_w();
        uint32_t t[D];
        mont(t, v, w);
        add_wide<D>(nu, u, t, q);
        sub_wide<D>(nv, u, t, q);
      } else {  // ntt.go:365-370 with each stage's outputs halved: log N stages give N^-1 (242-243)
        uint32_t d[D], s[D];
        if constexpr (PF) take_w();  // the next twiddle's loads issue ahead of this butterfly's work
        add_wide<D>(s, u, v, q);
        half_wide<D>(nu, s, q);
        sub_wide<D>(d, u, v, q);
        // u and v are dead here: without the prefetch the twiddle load is held behind the add /
        // sub so the live set at the product is d, w and nu, as the forward's is u, v and w
        if constexpr (!PF) {
          __builtin_amdgcn_sched_barrier(0);
          take_w();
        }
        mont(nv, d, w);  // w = twInv / 2
      }
#pragma unroll
      for (int l = 0; l < L; ++l) {
        lds[l * plane + c * NP + x0] = pk(nu[2 * l], nu[2 * l + 1]);
        lds[l * plane + c * NP + x1] = pk(nv[2 * l], nv[2 * l + 1]);
      }
    }
    // LDS-only barrier: __syncthreads() would also wait for the twiddle prefetch (vmcnt(0)).  The
    // workgroup fences restricted to the local address space order the LDS stage exchange (they
    // compile to lgkmcnt(0) + s_barrier) and leave the global prefetch in flight; only LDS is
    // shared between stages, global memory is written once after the last one
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  }
  // ---- LDS -> HBM
  for (int f = threadIdx.x; f < W; f += kWideThreads) {
    const int l = f % L, e = f / L;
    const int c = logS == 0 ? e / NP : e % cpt, x = logS == 0 ? e % NP : e / cpt;
    const long long g = elem(c, x);
    if (g >= 0) a.out[g * L + l] = lds[l * plane + c * NP + x];
  }
}

#endif  // __HIPCC__

}  // namespace rg
