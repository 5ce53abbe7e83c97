// ntt_kernels.hpp -- bigpoly negacyclic / cyclic NTT kernels for gfx950 (math/bigpoly/ntt.go).
//
// What is computed (bit-exact vs the reference):
//   forward  = nttInPlace   (ntt.go:246-355): Cooley-Tukey DIT, natural in -> bit-reversed out,
//              butterfly (u, v) <- (u + w v, u - w v) with w = tw[m + i]        (ntt.go:254-259)
//   inverse  = inttInPlace + scalarMulVecTo(N^-1) (ntt.go:357-466, 242-243): Gentleman-Sande,
//              (u, v) <- (u + v, (u - v) w), w = twInv[m + i]; the N^-1 scaling is fused into
//              the last stage ((u+v) N^-1, (u-v)(twInv[1] N^-1)) -- same residues.
// The table layout tw[m + i] is shared by the cyclic and negacyclic transformers, so one
// kernel family serves both (only the tables differ).
//
// How (MI355X-first):
//   A transform of N = 2^logN points is split into passes; a pass covers P consecutive
//   global stages [G0, G0+P) and decomposes into independent 2^P-point sub-transforms whose
//   points sit at stride S = 2^(logN-G0-P) (G0 = 0: "column" pass, S = 1: "row" pass).
//   One 256-thread workgroup owns SW = 256 / 2^(P-R) sub-transforms:
//     1. the tile is read from HBM with 16-B coalesced loads into LDS (limb planes, one pad
//        slot per 16 points so every round's ds_read_b64/ds_write_b64 is conflict-free),
//     2. ceil(P/R) rounds: each thread pulls 2^R points into VGPRs, runs R radix-2 stages
//        in registers (twiddles from the L2-resident table), writes them back,
//     3. the tile is written back with coalesced 16-B stores (in place is allowed).
//   N = 2^16 at L = 1 is two passes of 8 stages (column then row; reversed for the inverse).
//   The batch of polynomials is processed in MALL-sized chunks (column pass, row pass per
//   chunk) so the pass-to-pass intermediate stays in the 256 MiB Infinity Cache and HBM
//   sees ~one read and one write per element per transform.
#pragma once
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "field.hpp"
#include "ntt_plan.hpp"

namespace rg {

constexpr int kWG = 256;

template <int L>
struct NttArgs {
  const uint64_t* in;
  uint64_t* out;
  const uint64_t* tw;  // L==1 && SHOUP: (w, w') pairs [N][2]; else Montgomery [N][L]
  FieldParams<L> F;
  uint64_t nsc[L];   // N^-1: Montgomery form (or plain value for SHOUP)
  uint64_t nsc_sh;   // Shoup companion of nsc
  uint64_t w1n[L];   // twInv[1] * N^-1
  uint64_t w1n_sh;
  int logN, G0;
  int qlo1;             // q mod 2^32 == 1 (L == 1 fast reduction)
  long long total_sub;  // batch * N / 2^P
};

// per-L register radix (points per thread = 2^R) keeps VGPR use near 128
template <int L>
struct RadixOf {
  static constexpr int value = (L == 1 || L == 2) ? 4 : (L <= 4 ? 3 : (L <= 7 ? 2 : 2));
};
template <int L>
constexpr int pmax_of() {
  return RadixOf<L>::value + 8;
}

template <int L, bool SHOUP>
struct Tw {
  uint64_t w[L];
  uint64_t wp;
};

template <int L, bool SHOUP>
__device__ __forceinline__ void load_tw(Tw<L, SHOUP>& w, const uint64_t* tw, long long idx) {
  if constexpr (SHOUP) {
    const ulonglong2 v = reinterpret_cast<const ulonglong2*>(tw)[idx];
    w.w[0] = v.x;
    w.wp = v.y;
  } else {
#pragma unroll
    for (int l = 0; l < L; ++l) w.w[l] = tw[idx * L + l];
  }
}

template <int L, bool SHOUP>
__device__ __forceinline__ void mul_tw(uint64_t* z, const uint64_t* x, const Tw<L, SHOUP>& w,
                                       const FieldParams<L>& F) {
  if constexpr (SHOUP) {
    z[0] = shoup_mul(x[0], w.w[0], w.wp, F.q[0]);
  } else {
    f_mul<L>(z, x, w.w, F);
  }
}

// forward CT butterfly (ntt.go:254-259)
template <int L, bool SHOUP>
__device__ __forceinline__ void bfly_fwd(uint64_t* u, uint64_t* v, const Tw<L, SHOUP>& w, const FieldParams<L>& F) {
  uint64_t t[L];
  mul_tw<L, SHOUP>(t, v, w, F);
  if constexpr (L == 1 && SHOUP) {  // q < 2^63: 2q fits a word
    uint64_t a = u[0];
    u[0] = mod_add(a, t[0], F.q[0]);
    v[0] = mod_sub(a, t[0], F.q[0]);
  } else {
    f_sub<L>(v, u, t, F);
    f_add<L>(u, u, t, F);
  }
}
// inverse GS butterfly (ntt.go:365-370)
template <int L, bool SHOUP>
__device__ __forceinline__ void bfly_inv(uint64_t* u, uint64_t* v, const Tw<L, SHOUP>& w, const FieldParams<L>& F) {
  uint64_t d[L];
  if constexpr (L == 1 && SHOUP) {
    uint64_t a = u[0], b = v[0];
    u[0] = mod_add(a, b, F.q[0]);
    d[0] = mod_sub(a, b, F.q[0]);
  } else {
    f_sub<L>(d, u, v, F);
    f_add<L>(u, u, v, F);
  }
  mul_tw<L, SHOUP>(v, d, w, F);
}

__device__ __forceinline__ int padx(int x) { return x + (x >> 4); }

// ----------------------------------------------------------------------------------------
// Lock-step single-word Shoup stages (L = 1).  One radix-2 stage of a radix-16 round is 8
// independent butterflies; writing each micro-step for all 8 before the next one exposes
// 8-way ILP in program order, which hides the dependent-issue latency and the carry/VCC
// hazards of 64-bit integer code at the low occupancy the register-resident tile allows.
// q < 2^63 (checked at plan creation) so every intermediate fits one word.
// ----------------------------------------------------------------------------------------
struct ShoupK {
  uint64_t q;
  uint32_t qlo1;  // q mod 2^32 == 1  ->  lo64(x*q) = x + ((x_lo*q_hi) << 32)
};

__device__ __forceinline__ uint64_t lo64_mul_q(uint64_t x, uint64_t q, bool qlo1) {
  if (qlo1) {
    const uint32_t m = (uint32_t)x * (uint32_t)(q >> 32);
    return x + ((uint64_t)m << 32);
  }
  return x * q;
}

// 32-bit-half arithmetic with explicit carry chains: the borrow out of the trial
// subtraction IS the select mask (no separate 64-bit compare), q < 2^63.
__device__ __forceinline__ uint64_t pack(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
__device__ __forceinline__ uint64_t addmod63(uint64_t a, uint64_t b, uint64_t q) {
  uint32_t c, br;
  const uint32_t s0 = __builtin_addc((uint32_t)a, (uint32_t)b, 0u, &c);
  const uint32_t s1 = __builtin_addc((uint32_t)(a >> 32), (uint32_t)(b >> 32), c, &c);
  const uint32_t t0 = __builtin_subc(s0, (uint32_t)q, 0u, &br);
  const uint32_t t1 = __builtin_subc(s1, (uint32_t)(q >> 32), br, &br);
  return br ? pack(s0, s1) : pack(t0, t1);
}
__device__ __forceinline__ uint64_t submod63(uint64_t a, uint64_t b, uint64_t q) {
  uint32_t br, c;
  const uint32_t d0 = __builtin_subc((uint32_t)a, (uint32_t)b, 0u, &br);
  const uint32_t d1 = __builtin_subc((uint32_t)(a >> 32), (uint32_t)(b >> 32), br, &br);
  const uint32_t e0 = __builtin_addc(d0, (uint32_t)q, 0u, &c);
  const uint32_t e1 = __builtin_addc(d1, (uint32_t)(q >> 32), c, &c);
  return br ? pack(e0, e1) : pack(d0, d1);
}
__device__ __forceinline__ uint64_t reduce2q(uint64_t r, uint64_t q) {  // [0, 2q) -> [0, q)
  uint32_t br;
  const uint32_t t0 = __builtin_subc((uint32_t)r, (uint32_t)q, 0u, &br);
  const uint32_t t1 = __builtin_subc((uint32_t)(r >> 32), (uint32_t)(q >> 32), br, &br);
  return br ? r : pack(t0, t1);
}
// y * w mod q (Shoup, w' = floor(w 2^64 / q)), result in [0, 2q)
template <bool QLO1>
__device__ __forceinline__ uint64_t shoup_lazy(uint64_t y, uint64_t w, uint64_t wp, uint64_t q) {
  const uint32_t y0 = (uint32_t)y, y1 = (uint32_t)(y >> 32);
  const uint32_t p0 = (uint32_t)wp, p1 = (uint32_t)(wp >> 32);
  const uint64_t t1 = mad64(y1, p0, __umulhi(y0, p0));
  const uint64_t t2 = mad64(y0, p1, (uint32_t)t1);
  const uint64_t qh = mad64(y1, p1, t1 >> 32) + (t2 >> 32);
  const uint32_t w0 = (uint32_t)w, w1 = (uint32_t)(w >> 32);
  const uint64_t pw = mad64(y0, w0, 0);
  const uint32_t yw1 = (uint32_t)(pw >> 32) + y0 * w1 + y1 * w0;
  const uint32_t yw0 = (uint32_t)pw;
  if constexpr (QLO1) {
    const uint32_t m = (uint32_t)qh * (uint32_t)(q >> 32);
    uint32_t br;
    const uint32_t r0 = __builtin_subc(yw0, (uint32_t)qh, 0u, &br);
    const uint32_t r1 = __builtin_subc(yw1, (uint32_t)(qh >> 32), br, &br) - m;
    return pack(r0, r1);
  } else {
    return pack(yw0, yw1) - qh * q;
  }
}

// fwd: for k in [0, 8): (u_k, v_k) <- (u_k + w_k v_k, u_k - w_k v_k); twiddle w_k = tw[k / HALF]
template <int HALF, bool QLO1>
__device__ __forceinline__ void stage8_fwd(uint64_t (&e)[16][1], const uint64_t* w, const uint64_t* wp, uint64_t q) {
  uint64_t r[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int blk = k / HALF, u = k % HALF, i1 = blk * 2 * HALF + u + HALF;
    r[k] = shoup_lazy<QLO1>(e[i1][0], w[blk], wp[blk], q);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = reduce2q(r[k], q);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int blk = k / HALF, u = k % HALF, i0 = blk * 2 * HALF + u, i1 = i0 + HALF;
    const uint64_t a = e[i0][0];
    e[i0][0] = addmod63(a, r[k], q);
    e[i1][0] = submod63(a, r[k], q);
  }
}

// inv: (u, v) <- (u + v, (u - v) w)
template <int HALF, bool QLO1>
__device__ __forceinline__ void stage8_inv(uint64_t (&e)[16][1], const uint64_t* w, const uint64_t* wp, uint64_t q) {
  uint64_t d[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int blk = k / HALF, u = k % HALF, i0 = blk * 2 * HALF + u, i1 = i0 + HALF;
    const uint64_t a = e[i0][0], b = e[i1][0];
    e[i0][0] = addmod63(a, b, q);
    d[k] = submod63(a, b, q);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int blk = k / HALF, u = k % HALF, i1 = blk * 2 * HALF + u + HALF;
    e[i1][0] = reduce2q(shoup_lazy<QLO1>(d[k], w[blk], wp[blk], q), q);
  }
}

// ----------------------------------------------------------------------------------------
// rounds
// ----------------------------------------------------------------------------------------
template <int L, int P, int R, bool INV, bool SHOUP, bool SCALE, int K>
__device__ __forceinline__ void do_rounds(const NttArgs<L>& a, uint64_t* lds, int s, int t, long long hi,
                                          int plane) {
  constexpr int NR = (P + R - 1) / R;
  constexpr int R0 = P - R * (NR - 1);
  constexpr int RK = (K == 0) ? R0 : R;
  constexpr int NG = 1 << (R - RK);  // groups per thread this round
  constexpr int NPK = 1 << RK;
  // bit window of this round
  constexpr int LO = INV ? ((K == 0) ? 0 : R0 + R * (K - 1)) : (P - ((K == 0) ? 0 : R0 + R * (K - 1)) - RK);
  constexpr int HI = LO + RK;
  const int PADN = (1 << P) + ((1 << P) >> 4);
  uint64_t* ls = lds + (long long)s * PADN;

#pragma unroll 1
  for (int g = 0; g < NG; ++g) {
    const int o = t * NG + g;                   // index over the bits outside [LO, HI)
    const int o_low = o & ((1 << LO) - 1);
    const int o_high = o >> LO;                 // bits above HI
    const int xbase = (o_high << HI) | o_low;
    uint64_t e[NPK][L];
#pragma unroll
    for (int y = 0; y < NPK; ++y) {
      const int x = xbase | (y << LO);
#pragma unroll
      for (int l = 0; l < L; ++l) e[y][l] = ls[(long long)l * plane + padx(x)];
    }
    if constexpr (!INV) {
#pragma unroll
      for (int sp = 0; sp < RK; ++sp) {
        const int gp = P - HI + sp;  // local stage index (0 = first stage of the pass)
        const int half = NPK >> (sp + 1);
#pragma unroll
        for (int blk = 0; blk < (1 << sp); ++blk) {
          const long long idx = (1LL << (a.G0 + gp)) + (hi << gp) + ((long long)o_high << sp) + blk;
          Tw<L, SHOUP> w;
          load_tw<L, SHOUP>(w, a.tw, idx);
#pragma unroll
          for (int u = 0; u < half; ++u) {
            const int i0 = blk * 2 * half + u;
            bfly_fwd<L, SHOUP>(e[i0], e[i0 + half], w, a.F);
          }
        }
      }
    } else {
#pragma unroll
      for (int sp = 0; sp < RK; ++sp) {
        const int gp = P - 1 - (LO + sp);
        const int half = 1 << sp;
        const bool last = SCALE && (a.G0 + gp == 0);
#pragma unroll
        for (int blk = 0; blk < (NPK >> (sp + 1)); ++blk) {
          const long long idx =
              (1LL << (a.G0 + gp)) + (hi << gp) + ((long long)o_high << (RK - sp - 1)) + blk;
          Tw<L, SHOUP> w;
          if (last) {
#pragma unroll
            for (int l = 0; l < L; ++l) w.w[l] = a.w1n[l];
            w.wp = a.w1n_sh;
          } else {
            load_tw<L, SHOUP>(w, a.tw, idx);
          }
#pragma unroll
          for (int u = 0; u < half; ++u) {
            const int i0 = blk * 2 * half + u;
            bfly_inv<L, SHOUP>(e[i0], e[i0 + half], w, a.F);
            if (last) {  // (u + v) * N^-1
              Tw<L, SHOUP> ns;
#pragma unroll
              for (int l = 0; l < L; ++l) ns.w[l] = a.nsc[l];
              ns.wp = a.nsc_sh;
              uint64_t z[L];
              mul_tw<L, SHOUP>(z, e[i0], ns, a.F);
#pragma unroll
              for (int l = 0; l < L; ++l) e[i0][l] = z[l];
            }
          }
        }
      }
    }
#pragma unroll
    for (int y = 0; y < NPK; ++y) {
      const int x = xbase | (y << LO);
#pragma unroll
      for (int l = 0; l < L; ++l) ls[(long long)l * plane + padx(x)] = e[y][l];
    }
  }
  __syncthreads();
  if constexpr (K + 1 < NR) do_rounds<L, P, R, INV, SHOUP, SCALE, K + 1>(a, lds, s, t, hi, plane);
}

// ----------------------------------------------------------------------------------------
// pass kernel
// ----------------------------------------------------------------------------------------
template <int L, int P, bool INV, bool SHOUP, bool SCALE>
__global__ __launch_bounds__(kWG) void ntt_pass_kernel(NttArgs<L> a) {
  constexpr int R = (RadixOf<L>::value < P) ? RadixOf<L>::value : P;
  constexpr int NP = 1 << P;
  constexpr int TS = 1 << (P - R);
  constexpr int SW = kWG / TS;
  constexpr int PADN = NP + (NP >> 4);
  constexpr int PLANE = SW * PADN;  // u64 per limb plane
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];

  const int logN = a.logN;
  const int logS = logN - a.G0 - P;
  const long long S = 1LL << logS;
  const int nlo = (int)(S < SW ? S : SW);
  const int nhi = SW / nlo;
  const long long sub0 = (long long)blockIdx.x * SW;
  const long long rowid0 = sub0 >> logS;
  const long long lo0 = sub0 & (S - 1);
  const int rowshift = logN - a.G0;  // log2 of the row pitch in elements
  const long long total = a.total_sub;

  // ---- 1. HBM -> LDS (coalesced) ----
  // flat element e = (sr * NP + x) * nlo + sl
  constexpr int NE = SW * NP;
  const bool pairs = (L % 2 == 0) || (nlo % 2 == 0) || (nlo == (int)S);
  if (pairs) {
    const int NU = NE * L / 2;  // u64 pairs in the tile
    for (int f2 = threadIdx.x; f2 < NU; f2 += kWG) {
      const int f = 2 * f2;
      const int e = f / L, l = f % L;
      const int sl = e % nlo, xr = e / nlo, x = xr % NP, sr = xr / NP;
      const int s = sr * nlo + sl;
      if (sub0 + s >= total) continue;
      const long long addr = (((rowid0 + sr) << rowshift) + (long long)x * S + lo0 + sl) * L + l;
      const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(a.in + addr);
      lds[(long long)l * PLANE + s * PADN + padx(x)] = v.x;
      // second word: next limb of the same element, or limb 0 of the next element
      const int f1 = f + 1;
      const int e1 = f1 / L, l1 = f1 % L;
      const int sl1 = e1 % nlo, xr1 = e1 / nlo, x1 = xr1 % NP, sr1 = xr1 / NP;
      const int s1 = sr1 * nlo + sl1;
      lds[(long long)l1 * PLANE + s1 * PADN + padx(x1)] = v.y;
    }
  } else {
    const int NU = NE * L;
    for (int f = threadIdx.x; f < NU; f += kWG) {
      const int e = f / L, l = f % L;
      const int sl = e % nlo, xr = e / nlo, x = xr % NP, sr = xr / NP;
      const int s = sr * nlo + sl;
      if (sub0 + s >= total) continue;
      const long long addr = (((rowid0 + sr) << rowshift) + (long long)x * S + lo0 + sl) * L + l;
      lds[(long long)l * PLANE + s * PADN + padx(x)] = a.in[addr];
    }
  }
  __syncthreads();

  // ---- 2. rounds ----
  const int s = threadIdx.x / TS;
  const int t = threadIdx.x % TS;
  const long long rowid = rowid0 + s / nlo;
  const long long hi = rowid & ((1LL << a.G0) - 1);  // row index within the polynomial
  do_rounds<L, P, R, INV, SHOUP, SCALE, 0>(a, lds, s, t, hi, PLANE);

  // ---- 3. LDS -> HBM ----
  if (pairs) {
    const int NU = NE * L / 2;
    for (int f2 = threadIdx.x; f2 < NU; f2 += kWG) {
      const int f = 2 * f2;
      const int e = f / L, l = f % L;
      const int sl = e % nlo, xr = e / nlo, x = xr % NP, sr = xr / NP;
      const int s0 = sr * nlo + sl;
      if (sub0 + s0 >= total) continue;
      const long long addr = (((rowid0 + sr) << rowshift) + (long long)x * S + lo0 + sl) * L + l;
      const int f1 = f + 1;
      const int e1 = f1 / L, l1 = f1 % L;
      const int sl1 = e1 % nlo, xr1 = e1 / nlo, x1 = xr1 % NP, sr1 = xr1 / NP;
      const int s1 = sr1 * nlo + sl1;
      ulonglong2 v;
      v.x = lds[(long long)l * PLANE + s0 * PADN + padx(x)];
      v.y = lds[(long long)l1 * PLANE + s1 * PADN + padx(x1)];
      *reinterpret_cast<ulonglong2*>(a.out + addr) = v;
    }
  } else {
    const int NU = NE * L;
    for (int f = threadIdx.x; f < NU; f += kWG) {
      const int e = f / L, l = f % L;
      const int sl = e % nlo, xr = e / nlo, x = xr % NP, sr = xr / NP;
      const int s0 = sr * nlo + sl;
      if (sub0 + s0 >= total) continue;
      const long long addr = (((rowid0 + sr) << rowshift) + (long long)x * S + lo0 + sl) * L + l;
      a.out[addr] = lds[(long long)l * PLANE + s0 * PADN + padx(x)];
    }
  }
}

template <int L, int P>
constexpr size_t lds_bytes() {
  constexpr int R = (RadixOf<L>::value < P) ? RadixOf<L>::value : P;
  constexpr int NP = 1 << P;
  constexpr int SW = kWG / (1 << (P - R));
  return (size_t)SW * (NP + (NP >> 4)) * L * 8;
}


// ----------------------------------------------------------------------------------------
// compact per-stage kernel: one thread per butterfly, one launch per stage.  Used for small
// ranks (logN < kMinTiledP) and for the wide buckler fields (L = 7, 14) where a register-
// tiled pass would be dominated by code size rather than bandwidth.
// ----------------------------------------------------------------------------------------
template <int L, bool INV, bool SHOUP>
__global__ __launch_bounds__(256) void ntt_stage_kernel(NttArgs<L> a, int lt, int scale) {
  const long long half_n = 1LL << (a.logN - 1);
  const long long total = a.total_sub * half_n;  // total_sub = batch here
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < total; k += stride) {
    const long long b = k >> (a.logN - 1);
    const long long r = k & (half_n - 1);
    const long long t = 1LL << lt;
    const long long m = 1LL << (a.logN - 1 - lt);
    const long long i = r >> lt;
    const long long j = (i << (lt + 1)) + (r & (t - 1));
    const uint64_t* src = a.in + (b << a.logN) * L;
    uint64_t* dst = a.out + (b << a.logN) * L;
    uint64_t u[L], v[L];
#pragma unroll
    for (int l = 0; l < L; ++l) {
      u[l] = src[j * L + l];
      v[l] = src[(j + t) * L + l];
    }
    Tw<L, SHOUP> w;
    if (INV && scale) {
#pragma unroll
      for (int l = 0; l < L; ++l) w.w[l] = a.w1n[l];
      w.wp = a.w1n_sh;
    } else {
      load_tw<L, SHOUP>(w, a.tw, m + i);
    }
    if constexpr (!INV) {
      bfly_fwd<L, SHOUP>(u, v, w, a.F);
    } else {
      bfly_inv<L, SHOUP>(u, v, w, a.F);
      if (scale) {
        Tw<L, SHOUP> ns;
#pragma unroll
        for (int l = 0; l < L; ++l) ns.w[l] = a.nsc[l];
        ns.wp = a.nsc_sh;
        uint64_t z[L];
        mul_tw<L, SHOUP>(z, u, ns, a.F);
#pragma unroll
        for (int l = 0; l < L; ++l) u[l] = z[l];
      }
    }
#pragma unroll
    for (int l = 0; l < L; ++l) {
      dst[j * L + l] = u[l];
      dst[(j + t) * L + l] = v[l];
    }
  }
}

// smallest P handled by the LDS-tiled pass kernel (smaller transforms use stage kernels)
constexpr int kMinTiledP = 6;

template <int L>
static void fill_args(NttArgs<L>& a, const NttLaunch& p) {
  memcpy(a.F.q, p.q, 8 * L);
  a.F.qinv = p.qinv;
  memcpy(a.nsc, p.nsc, 8 * L);
  a.nsc_sh = p.nsc_sh;
  memcpy(a.w1n, p.w1n, 8 * L);
  a.w1n_sh = p.w1n_sh;
  a.logN = p.logN;
  a.tw = p.tw;
  a.qlo1 = (uint32_t)p.q[0] == 1u;
}

template <int L, int P, bool INV, bool SHOUP, bool SCALE>
static rg_status launch_pass(const NttArgs<L>& a, hipStream_t st) {
  constexpr int R = (RadixOf<L>::value < P) ? RadixOf<L>::value : P;
  constexpr int SW = kWG / (1 << (P - R));
  const long long grid = (a.total_sub + SW - 1) / SW;
  constexpr size_t lds = lds_bytes<L, P>();
  static_assert(lds <= 160 * 1024, "tile exceeds LDS");
  auto k = ntt_pass_kernel<L, P, INV, SHOUP, SCALE>;
  static bool attr_set = false;
  if (!attr_set) {
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(kWG), lds, st, a);
  return check_launch("ntt_pass");
}

template <int L, bool INV, bool SHOUP, bool SCALE, int P = kMinTiledP>
static rg_status dispatch_P(int p, const NttArgs<L>& a, hipStream_t st) {
  if constexpr (P > pmax_of<L>()) {
    return RG_ERR_UNSUPPORTED;
  } else {
    if (p == P) return launch_pass<L, P, INV, SHOUP, SCALE>(a, st);
    return dispatch_P<L, INV, SHOUP, SCALE, P + 1>(p, a, st);
  }
}

}  // namespace rg

// ----------------------------------------------------------------------------------------
// 2-round pass specialisation (P = 8 = 2 x radix-16), the shape of every pass of the
// degree-2^16 transform.  Compared with ntt_pass_kernel:
//   * global <-> VGPR directly wherever the round's point pattern is coalesced (column
//     passes always; row passes on the side where lanes walk consecutive x), so LDS carries
//     only the one exchange between the rounds (plus one transpose on the row pass's other
//     side);
//   * persistent workgroups: the next tile's global loads are issued before the current
//     tile's butterflies, hiding HBM latency under VALU work (L = 1);
//   * twiddles that are uniform over the workgroup (column pass, the high-bit round) come
//     from scalar loads.
// Lane mapping: COL: s = tid & 15 (column, consecutive addresses), t = tid >> 4;
//               ROW: t = tid & 15 (consecutive addresses), s = tid >> 4.
// LDS layout lds[l][s * PADN + pad(x)]: COL uses pad(x) = x, PADN = 257; ROW uses
// pad(x) = x + x/16, PADN = 272 (see DESIGN.md for the bank analysis).
// ----------------------------------------------------------------------------------------
namespace rg {

template <bool COL>
struct R2Layout {
  static constexpr int PADN = COL ? 257 : 272;
  __device__ static __forceinline__ int pad(int x) { return COL ? x : x + (x >> 4); }
};

template <int L, bool SHOUP, bool UNIFORM>
__device__ __forceinline__ void load_tw2(Tw<L, SHOUP>& w, const uint64_t* tw, long long idx) {
  if constexpr (UNIFORM) {
    const int i = __builtin_amdgcn_readfirstlane((int)idx);
    load_tw<L, SHOUP>(w, tw, i);
  } else {
    load_tw<L, SHOUP>(w, tw, idx);
  }
}


template <int SP, bool INV, bool SCALE, bool QLO1>
__device__ __forceinline__ void lockstep_stage(const NttArgs<1>& a, uint64_t (&e)[16][1], bool high, long long hi,
                                               int o_high, bool uniform) {
  // forward stage SP of the round: HALF = 8 >> SP, 2^SP twiddles; inverse: HALF = 1 << SP
  constexpr int HALF = INV ? (1 << SP) : (8 >> SP);
  constexpr int NB = 8 / HALF;
  const int gp = INV ? (7 - ((high ? 4 : 0) + SP)) : ((high ? 0 : 4) + SP);
  const int shift = INV ? (3 - SP) : SP;
  uint64_t w[NB], wp[NB];
  const bool last = INV && SCALE && (a.G0 + gp == 0);
  if (last) {
    w[0] = a.w1n[0];
    wp[0] = a.w1n_sh;
  } else {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      long long idx = (1LL << (a.G0 + gp)) + (hi << gp) + ((long long)o_high << shift) + b;
      if (uniform) idx = __builtin_amdgcn_readfirstlane((int)idx);
      const ulonglong2 v = reinterpret_cast<const ulonglong2*>(a.tw)[idx];
      w[b] = v.x;
      wp[b] = v.y;
    }
  }
  const uint64_t q = a.F.q[0];
  if constexpr (!INV) {
    stage8_fwd<HALF, QLO1>(e, w, wp, q);
  } else {
    stage8_inv<HALF, QLO1>(e, w, wp, q);
    if (last) {  // (u + v) * N^-1 on the 8 upper outputs
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int i0 = (k / HALF) * 2 * HALF + (k % HALF);
        e[i0][0] = shoup_mul(e[i0][0], a.nsc[0], a.nsc_sh, q);
      }
    }
  }
}

template <bool INV, bool SCALE, bool QLO1>
__device__ __forceinline__ void lockstep_round(const NttArgs<1>& a, uint64_t (&e)[16][1], bool high, long long hi,
                                               int o_high, bool uniform) {
  lockstep_stage<0, INV, SCALE, QLO1>(a, e, high, hi, o_high, uniform);
  lockstep_stage<1, INV, SCALE, QLO1>(a, e, high, hi, o_high, uniform);
  lockstep_stage<2, INV, SCALE, QLO1>(a, e, high, hi, o_high, uniform);
  lockstep_stage<3, INV, SCALE, QLO1>(a, e, high, hi, o_high, uniform);
}

template <int L, bool INV, bool SHOUP, bool SCALE, bool COL, bool PREFETCH, bool QLO1>
__global__ __launch_bounds__(kWG) void ntt_r2_kernel(NttArgs<L> a) {
  constexpr int NP = 256, SW = 16;
  using LY = R2Layout<COL>;
  constexpr int PADN = LY::PADN;
  __shared__ uint64_t lds[L * SW * PADN];

  const int tid = threadIdx.x;
  const int s = COL ? (tid & 15) : (tid >> 4);
  const int t = COL ? (tid >> 4) : (tid & 15);
  const int logN = a.logN;
  const int logS = logN - a.G0 - 8;  // COL: logS >= 4; ROW: 0
  const long long ntiles = a.total_sub / SW;
  const int rowshift = logN - a.G0;

  // Addressing: a tile-uniform base (SGPRs) plus a 32-bit per-lane element offset, so the
  // loads/stores use saddr + voffset and no 64-bit address is kept per point.
  //   COL: elem = (rowid0 << rowshift) + lo0 + (x << logS) + s
  //   ROW: elem = (sub0 << rowshift) + (s << rowshift) + x
  auto tile_base = [&](long long tile) -> long long {
    const long long sub0 = tile * SW;
    if constexpr (COL)
      return ((sub0 >> logS) << rowshift) + (sub0 & ((1LL << logS) - 1));
    else
      return sub0 << rowshift;
  };
  const uint32_t lane_off = COL ? (uint32_t)s : ((uint32_t)s << rowshift);
  const int xshift = COL ? logS : 0;
  auto gload = [&](uint64_t (&r)[16][L], long long tile, bool low_pattern) {
    const uint64_t* base = a.in + tile_base(tile) * L;
#pragma unroll
    for (int y = 0; y < 16; ++y) {
      const uint32_t x = low_pattern ? (16 * t + y) : (t + 16 * y);
      const uint32_t off = ((x << xshift) + lane_off) * L;
#pragma unroll
      for (int l = 0; l < L; ++l) r[y][l] = base[off + l];
    }
  };
  auto gstore = [&](const uint64_t (&r)[16][L], long long tile, bool low_pattern) {
    uint64_t* base = a.out + tile_base(tile) * L;
#pragma unroll
    for (int y = 0; y < 16; ++y) {
      const uint32_t x = low_pattern ? (16 * t + y) : (t + 16 * y);
      const uint32_t off = ((x << xshift) + lane_off) * L;
#pragma unroll
      for (int l = 0; l < L; ++l) base[off + l] = r[y][l];
    }
  };
  auto lds_put = [&](const uint64_t (&r)[16][L], bool low_pattern) {
#pragma unroll
    for (int y = 0; y < 16; ++y) {
      const int x = low_pattern ? (16 * t + y) : (t + 16 * y);
#pragma unroll
      for (int l = 0; l < L; ++l) lds[l * SW * PADN + s * PADN + LY::pad(x)] = r[y][l];
    }
  };
  auto lds_get = [&](uint64_t (&r)[16][L], bool low_pattern) {
#pragma unroll
    for (int y = 0; y < 16; ++y) {
      const int x = low_pattern ? (16 * t + y) : (t + 16 * y);
#pragma unroll
      for (int l = 0; l < L; ++l) r[y][l] = lds[l * SW * PADN + s * PADN + LY::pad(x)];
    }
  };

  // radix-16 round on e[y] (y = the 4 bits being transformed), forward (DIT, top bit first)
  // or inverse (DIF, low bit first).  `high` selects the x-bit window [4,8) vs [0,4).
  auto round = [&](uint64_t (&e)[16][L], bool high, long long hi) {
    // o_high: bits of x above the window (t when the window is [0,4), none otherwise)
    const int o_high = high ? 0 : t;
    const bool uniform = COL && high;  // twiddle index depends on nothing per-lane
    if constexpr (L == 1 && SHOUP) {
      lockstep_round<INV, SCALE, QLO1>(a, e, high, hi, o_high, uniform);
      return;
    }
    if constexpr (!INV) {
#pragma unroll
      for (int sp = 0; sp < 4; ++sp) {
        const int gp = (high ? 0 : 4) + sp;
        const int half = 8 >> sp;
#pragma unroll
        for (int blk = 0; blk < (1 << sp); ++blk) {
          const long long idx = (1LL << (a.G0 + gp)) + (hi << gp) + ((long long)o_high << sp) + blk;
          Tw<L, SHOUP> w;
          if (uniform)
            load_tw2<L, SHOUP, true>(w, a.tw, idx);
          else
            load_tw2<L, SHOUP, false>(w, a.tw, idx);
#pragma unroll
          for (int u = 0; u < half; ++u) {
            const int i0 = blk * 2 * half + u;
            bfly_fwd<L, SHOUP>(e[i0], e[i0 + half], w, a.F);
          }
        }
      }
    } else {
#pragma unroll
      for (int sp = 0; sp < 4; ++sp) {
        const int lo = high ? 4 : 0;
        const int gp = 7 - (lo + sp);
        const int half = 1 << sp;
        const bool last = SCALE && (a.G0 + gp == 0);
#pragma unroll
        for (int blk = 0; blk < (16 >> (sp + 1)); ++blk) {
          const long long idx = (1LL << (a.G0 + gp)) + (hi << gp) + ((long long)o_high << (3 - sp)) + blk;
          Tw<L, SHOUP> w;
          if (last) {
#pragma unroll
            for (int l = 0; l < L; ++l) w.w[l] = a.w1n[l];
            w.wp = a.w1n_sh;
          } else if (uniform) {
            load_tw2<L, SHOUP, true>(w, a.tw, idx);
          } else {
            load_tw2<L, SHOUP, false>(w, a.tw, idx);
          }
#pragma unroll
          for (int u = 0; u < half; ++u) {
            const int i0 = blk * 2 * half + u;
            bfly_inv<L, SHOUP>(e[i0], e[i0 + half], w, a.F);
            if (last) {
              Tw<L, SHOUP> ns;
#pragma unroll
              for (int l = 0; l < L; ++l) ns.w[l] = a.nsc[l];
              ns.wp = a.nsc_sh;
              uint64_t z[L];
              mul_tw<L, SHOUP>(z, e[i0], ns, a.F);
#pragma unroll
              for (int l = 0; l < L; ++l) e[i0][l] = z[l];
            }
          }
        }
      }
    }
  };

  // forward: round A = high window (pattern x = t + 16y), round B = low window (x = 16t + y)
  // inverse: round A = low window, round B = high window
  const bool a_low = INV;
  uint64_t cur[16][L], nxt[16][L];
  long long tile = blockIdx.x;
  // ROW + first round on the low pattern: lanes walk x = 16t+y -> load coalesced (x = t+16y)
  // and transpose through LDS.
  constexpr bool LOAD_T = !COL && INV;
  constexpr bool STORE_T = !COL && !INV;
  if (tile < ntiles) gload(cur, tile, LOAD_T ? false : a_low);
  for (; tile < ntiles; tile += gridDim.x) {
    const long long nt = tile + gridDim.x;
    if (PREFETCH && nt < ntiles) gload(nxt, nt, LOAD_T ? false : a_low);
    const long long hi = COL ? 0 : ((tile * SW + s) & ((1LL << a.G0) - 1));
    if constexpr (LOAD_T) {
      lds_put(cur, false);
      __syncthreads();
      lds_get(cur, true);
      __syncthreads();
    }
    round(cur, !a_low, hi);
    lds_put(cur, a_low);
    __syncthreads();
    lds_get(cur, !a_low);
    __syncthreads();
    round(cur, a_low, hi);
    if constexpr (STORE_T) {
      lds_put(cur, true);
      __syncthreads();
      lds_get(cur, false);
      __syncthreads();
      gstore(cur, tile, false);
    } else {
      gstore(cur, tile, !a_low);
    }
    if (PREFETCH) {
#pragma unroll
      for (int y = 0; y < 16; ++y)
#pragma unroll
        for (int l = 0; l < L; ++l) cur[y][l] = nxt[y][l];
    } else if (nt < ntiles) {
      gload(cur, nt, LOAD_T ? false : a_low);
    }
  }
}

template <int L, bool INV, bool SHOUP, bool SCALE, bool COL, bool PF, bool QLO1>
static rg_status launch_r2_pf(const NttArgs<L>& a, hipStream_t st) {
  const long long ntiles = a.total_sub / 16;
  static int grid_cap = 0;
  if (!grid_cap) {
    int per_cu = 0, dev = 0, cus = 256;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ntt_r2_kernel<L, INV, SHOUP, SCALE, COL, PF, QLO1>, kWG, 0);
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    grid_cap = (per_cu > 0 ? per_cu : 1) * cus;
  }
  const long long grid = ntiles < grid_cap ? ntiles : grid_cap;
  hipLaunchKernelGGL((ntt_r2_kernel<L, INV, SHOUP, SCALE, COL, PF, QLO1>), dim3((unsigned)grid), dim3(kWG), 0, st, a);
  return check_launch("ntt_r2");
}

// the next-tile register prefetch at L = 1 (q >= 2^63: the CIOS single-word fields; Shoup fields
// take ntt_r8); none at L >= 2, where the tile's registers leave no room for it
template <int L, bool INV, bool SHOUP, bool SCALE, bool COL>
static rg_status launch_r2(const NttArgs<L>& a, hipStream_t st) {
  static_assert(!(L == 1 && SHOUP), "single-word Shoup fields run on ntt_r8 (run_tiled)");
  return launch_r2_pf<L, INV, SHOUP, SCALE, COL, L == 1, false>(a, st);
}

template <int L, bool INV, bool SHOUP, bool SCALE>
static rg_status dispatch_r2(bool col, const NttArgs<L>& a, hipStream_t st) {
  return col ? launch_r2<L, INV, SHOUP, SCALE, true>(a, st) : launch_r2<L, INV, SHOUP, SCALE, false>(a, st);
}

}  // namespace rg

namespace rg {

}  // namespace rg

// ----------------------------------------------------------------------------------------
// Radix-8 pass for single-word Shoup fields (P = 8 as rounds of 3 + 3 + 2 bits).
// 8 points per thread (16 VGPRs of data instead of 32) and 512-thread workgroups holding 16
// sub-transforms: the register file admits ~8 waves per SIMD, which is what hides the
// dependent-issue latency of 64-bit integer multiply chains (the radix-16 pass measured
// ~6 cycles per VALU instruction at 2 waves/SIMD).  Two LDS exchanges per pass instead of
// one.  Lane mapping as in ntt_r2_kernel: COL s fastest (16 columns -> 128 B runs),
// ROW t fastest (32 consecutive points).  LDS images per exchange: see ntt_r8_kernel.
// ----------------------------------------------------------------------------------------
namespace rg {

template <int RK, bool INV, bool SCALE, bool QLO1>
__device__ __forceinline__ void r8_round(const NttArgs<1>& a, uint64_t (&e)[8], int LO, long long hi, int t,
                                         bool uniform) {
  // window [LO, LO+RK) of x; the thread's 8 registers hold NG = 8 >> RK groups of 2^RK
  // points: register r = g * 2^RK + y, group index g extends the thread's other bits.
  constexpr int NG = 8 >> RK;
  constexpr int NPK = 1 << RK;
  const int HI = LO + RK;
  const uint64_t q = a.F.q[0];
#pragma unroll
  for (int sp = 0; sp < RK; ++sp) {
    const int gp = INV ? (7 - (LO + sp)) : ((8 - HI) + sp);
    const bool last = INV && SCALE && (a.G0 + gp == 0);
    const int half = INV ? (1 << sp) : (NPK >> (sp + 1));
    const int nblk = NPK / (2 * half);
    uint64_t w[4], wp[4];
    // twiddles for the 4 butterflies of this stage (k = g * (NPK/2) + blk * half + u)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int g = k / (NPK / 2), kk = k % (NPK / 2), blk = kk / half;
      if (k % half) {
        w[k] = w[k - 1];
        wp[k] = wp[k - 1];
        continue;
      }
      // bits of x above the window: o = t * NG + g, o_high = o >> LO
      const int o = t * NG + g;
      const long long ohigh = o >> LO;
      long long idx = INV ? ((1LL << (a.G0 + gp)) + (hi << gp) + (ohigh << (RK - sp - 1)) + blk)
                          : ((1LL << (a.G0 + gp)) + (hi << gp) + (ohigh << sp) + blk);
      if (last) {
        w[k] = a.w1n[0];
        wp[k] = a.w1n_sh;
      } else {
        if (uniform) idx = __builtin_amdgcn_readfirstlane((int)idx);
        const ulonglong2 v = reinterpret_cast<const ulonglong2*>(a.tw)[idx];
        w[k] = v.x;
        wp[k] = v.y;
      }
      (void)nblk;
    }
    uint64_t r[4];
    if constexpr (!INV) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int g = k / (NPK / 2), kk = k % (NPK / 2), blk = kk / half, u = kk % half;
        const int i1 = g * NPK + blk * 2 * half + u + half;
        r[k] = reduce2q(shoup_lazy<QLO1>(e[i1], w[k], wp[k], q), q);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int g = k / (NPK / 2), kk = k % (NPK / 2), blk = kk / half, u = kk % half;
        const int i0 = g * NPK + blk * 2 * half + u, i1 = i0 + half;
        const uint64_t x0 = e[i0];
        e[i0] = addmod63(x0, r[k], q);
        e[i1] = submod63(x0, r[k], q);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int g = k / (NPK / 2), kk = k % (NPK / 2), blk = kk / half, u = kk % half;
        const int i0 = g * NPK + blk * 2 * half + u, i1 = i0 + half;
        const uint64_t x0 = e[i0], x1 = e[i1];
        e[i0] = addmod63(x0, x1, q);
        r[k] = submod63(x0, x1, q);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int g = k / (NPK / 2), kk = k % (NPK / 2), blk = kk / half, u = kk % half;
        const int i0 = g * NPK + blk * 2 * half + u, i1 = i0 + half;
        e[i1] = reduce2q(shoup_lazy<QLO1>(r[k], w[k], wp[k], q), q);
        if (last) e[i0] = shoup_mul(e[i0], a.nsc[0], a.nsc_sh, q);
      }
    }
  }
}

template <bool INV, bool SCALE, bool COL, bool QLO1, bool PF>
__global__ __launch_bounds__(512) void ntt_r8_kernel(NttArgs<1> a) {
  constexpr int SW = 16, PADN = 288;
  __shared__ uint64_t lds[SW * PADN];
  const int tid = threadIdx.x;
  const int s = COL ? (tid & 15) : (tid >> 5);
  const int t = COL ? (tid >> 4) : (tid & 31);
  const int logN = a.logN;
  const int logS = logN - a.G0 - 8;
  const int rowshift = logN - a.G0;
  const long long ntiles = a.total_sub / SW;
  const uint32_t lane_off = COL ? (uint32_t)s : ((uint32_t)s << rowshift);
  const int xshift = COL ? logS : 0;
  auto tile_base = [&](long long tile) -> long long {
    const long long sub0 = tile * SW;
    return COL ? (((sub0 >> logS) << rowshift) + (sub0 & ((1LL << logS) - 1))) : (sub0 << rowshift);
  };
  // LDS image per exchange (bank-conflict-free for both patterns of the exchange, checked
  // against the ds_read_b64 / ds_write_b64 lane-group model):
  //   COL: transposed [x][s] image, 16 x + s + 16 (x >> 3) -- every pattern
  //   ROW: [s][x] image; {H,M}: x + 4 (x >> 5); {M,L}: x + (x >> 3); {L,H}: x + (x >> 5)
  enum { HM, ML, LH };
  auto lpos = [&](int x, int ph) {
    if (COL) return 16 * x + s + 16 * (x >> 3);
    return s * PADN + x + (ph == HM ? 4 * (x >> 5) : ph == ML ? (x >> 3) : (x >> 5));
  };
  // point patterns: H = top window x = t + 32 y;  M = x = (t>>2)<<5 | y<<2 | (t&3);
  //                 L = bottom window, 2 groups: x = 8t + 4g + y   (register r = 4g + y)
  auto xH = [&](int y) { return t + 32 * y; };
  auto xM = [&](int y) { return ((t >> 2) << 5) | (y << 2) | (t & 3); };
  auto xL = [&](int r) { return 8 * t + r; };
  // the first round's raw global loads (coalesced pattern): forward H; inverse COL L, ROW H
  constexpr bool LOAD_L = INV && COL;
  auto gload = [&](uint64_t (&r)[8], long long tile) {
    const uint64_t* gin = a.in + tile_base(tile);
#pragma unroll
    for (int y = 0; y < 8; ++y) r[y] = gin[((uint32_t)(LOAD_L ? xL(y) : xH(y)) << xshift) + lane_off];
  };
  const bool uni = COL;
  uint64_t e[8], nx[8];
  long long tile = blockIdx.x;
  if (PF && tile < ntiles) gload(e, tile);
  for (; tile < ntiles; tile += gridDim.x) {
    const long long nt = tile + gridDim.x;
    if (!PF) gload(e, tile);
    if (PF && nt < ntiles) gload(nx, nt);  // next tile's HBM reads overlap this tile's butterflies
    const long long hi = COL ? 0 : ((tile * SW + s) & ((1LL << a.G0) - 1));
    uint64_t* gout = a.out + tile_base(tile);
    if (INV && !COL) {  // ROW inverse: loaded in H pattern, transpose to L through LDS
#pragma unroll
      for (int y = 0; y < 8; ++y) lds[lpos(xH(y), LH)] = e[y];
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 8; ++r) e[r] = lds[lpos(xL(r), LH)];
      __syncthreads();
    }
    if (!INV) {
      r8_round<3, false, SCALE, QLO1>(a, e, 5, hi, t, uni);
#pragma unroll
      for (int y = 0; y < 8; ++y) lds[lpos(xH(y), HM)] = e[y];
      __syncthreads();
#pragma unroll
      for (int y = 0; y < 8; ++y) e[y] = lds[lpos(xM(y), HM)];
      r8_round<3, false, SCALE, QLO1>(a, e, 2, hi, t, false);
      __syncthreads();
#pragma unroll
      for (int y = 0; y < 8; ++y) lds[lpos(xM(y), ML)] = e[y];
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 8; ++r) e[r] = lds[lpos(xL(r), ML)];
      r8_round<2, false, SCALE, QLO1>(a, e, 0, hi, t, false);
      if (COL) {
#pragma unroll
        for (int r = 0; r < 8; ++r) gout[((uint32_t)xL(r) << xshift) + lane_off] = e[r];
      } else {
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 8; ++r) lds[lpos(xL(r), LH)] = e[r];
        __syncthreads();
#pragma unroll
        for (int y = 0; y < 8; ++y) gout[(uint32_t)xH(y) + lane_off] = lds[lpos(xH(y), LH)];
      }
    } else {
      r8_round<2, true, SCALE, QLO1>(a, e, 0, hi, t, false);
#pragma unroll
      for (int r = 0; r < 8; ++r) lds[lpos(xL(r), ML)] = e[r];
      __syncthreads();
#pragma unroll
      for (int y = 0; y < 8; ++y) e[y] = lds[lpos(xM(y), ML)];
      r8_round<3, true, SCALE, QLO1>(a, e, 2, hi, t, false);
      __syncthreads();
#pragma unroll
      for (int y = 0; y < 8; ++y) lds[lpos(xM(y), HM)] = e[y];
      __syncthreads();
#pragma unroll
      for (int y = 0; y < 8; ++y) e[y] = lds[lpos(xH(y), HM)];
      r8_round<3, true, SCALE, QLO1>(a, e, 5, hi, t, uni);
#pragma unroll
      for (int y = 0; y < 8; ++y) gout[((uint32_t)xH(y) << xshift) + lane_off] = e[y];
    }
    __syncthreads();  // LDS reuse by the next tile
    if (PF) {
#pragma unroll
      for (int y = 0; y < 8; ++y) e[y] = nx[y];
    }
  }
}

// one tile per workgroup (the persistent prefetching grid, PF = true, measured slower in round 2
// and is no longer instantiated: tools/experiments/ntt_knob_kernels.patch)
template <bool INV, bool SCALE, bool COL, bool QLO1>
static rg_status launch_r8_q(const NttArgs<1>& a, hipStream_t st) {
  const long long ntiles = a.total_sub / 16;
  hipLaunchKernelGGL((ntt_r8_kernel<INV, SCALE, COL, QLO1, false>), dim3((unsigned)ntiles), dim3(512), 0, st, a);
  return check_launch("ntt_r8");
}

template <bool INV, bool SCALE, bool COL>
static rg_status launch_r8(const NttArgs<1>& a, hipStream_t st) {
  return a.qlo1 ? launch_r8_q<INV, SCALE, COL, true>(a, st) : launch_r8_q<INV, SCALE, COL, false>(a, st);
}


}  // namespace rg

namespace rg {

template <int L, bool SHOUP>
static rg_status run_tiled(const NttLaunch& p, hipStream_t st) {
  const size_t N = (size_t)1 << p.logN;
  const size_t poly_u64 = N * L;
  // chunk the batch so the pass-to-pass intermediate stays in the 256 MiB Infinity Cache
  static size_t chunk_bytes = 0;
  if (!chunk_bytes) {  // RINGO_NTT_CHUNK_MB overrides the Infinity-Cache-sized chunk (tuning)
    const char* e = knob(Knob::NttChunkMb);
    chunk_bytes = (size_t)(e ? atoi(e) : 192) << 20;
  }
  size_t chunk = std::max<size_t>(1, chunk_bytes / (poly_u64 * 8));
  if (p.npasses == 1) chunk = p.batch;
  NttArgs<L> a;
  fill_args<L>(a, p);
  for (size_t b0 = 0; b0 < p.batch; b0 += chunk) {
    const size_t nb = std::min(chunk, p.batch - b0);
    for (int k = 0; k < p.npasses; ++k) {
      const PassDesc& ps = p.inv ? p.passes[p.npasses - 1 - k] : p.passes[k];
      a.in = (k == 0 ? p.in : p.out) + b0 * poly_u64;
      a.out = p.out + b0 * poly_u64;
      a.G0 = ps.G0;
      a.total_sub = (long long)nb * (long long)(N >> ps.P);
      rg_status s;
      // 2-round specialisation: P = 8 with radix 16, column pass (stride >= 16) or row pass
      const int logS = p.logN - ps.G0 - ps.P;
      if (RadixOf<L>::value == 4 && ps.P == 8 && (logS == 0 || logS >= 4) && (a.total_sub % 16) == 0) {
        const bool col = logS >= 4;
        if constexpr (L == 1 && SHOUP) {  // radix-8 rounds (the radix-16 form measured slower)
          if (!p.inv)
            s = col ? launch_r8<false, false, true>(a, st) : launch_r8<false, false, false>(a, st);
          else if (ps.G0 == 0)
            s = col ? launch_r8<true, true, true>(a, st) : launch_r8<true, true, false>(a, st);
          else
            s = col ? launch_r8<true, false, true>(a, st) : launch_r8<true, false, false>(a, st);
        } else {
          if (!p.inv)
            s = dispatch_r2<L, false, SHOUP, false>(col, a, st);
          else if (ps.G0 == 0)
            s = dispatch_r2<L, true, SHOUP, true>(col, a, st);
          else
            s = dispatch_r2<L, true, SHOUP, false>(col, a, st);
        }
        RG_TRY(s);
        continue;
      }
      if (!p.inv)
        s = dispatch_P<L, false, SHOUP, false>(ps.P, a, st);
      else if (ps.G0 == 0)
        s = dispatch_P<L, true, SHOUP, true>(ps.P, a, st);
      else
        s = dispatch_P<L, true, SHOUP, false>(ps.P, a, st);
      RG_TRY(s);
    }
  }
  return RG_OK;
}

template <int L, bool SHOUP>
static rg_status run_stages(const NttLaunch& p, hipStream_t st) {
  NttArgs<L> a;
  fill_args<L>(a, p);
  a.G0 = 0;
  a.total_sub = (long long)p.batch;
  const long long nbfly = (long long)p.batch << (p.logN - 1);
  long long blocks = (nbfly + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  for (int s = 0; s < p.logN; ++s) {
    // forward: t = N/2 .. 1 (lt = logN-1 .. 0); inverse: t = 1 .. N/2
    const int lt = p.inv ? s : p.logN - 1 - s;
    a.in = (s == 0) ? p.in : p.out;
    a.out = p.out;
    const int scale = (p.inv && lt == p.logN - 1) ? 1 : 0;
    if (p.inv)
      hipLaunchKernelGGL((ntt_stage_kernel<L, true, SHOUP>), dim3((unsigned)blocks), dim3(256), 0, st, a, lt, scale);
    else
      hipLaunchKernelGGL((ntt_stage_kernel<L, false, SHOUP>), dim3((unsigned)blocks), dim3(256), 0, st, a, lt, scale);
    RG_TRY(check_launch("ntt_stage"));
  }
  return RG_OK;
}

}  // namespace rg


