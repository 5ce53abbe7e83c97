// ntt64.hpp -- single-word (q < 2^64/3, L = 1) NTT arithmetic for gfx950: lazy butterflies.
//
// Values between butterfly stages live in [0, 2q) ("Harvey" lazy form); only the last stage of
// a transform maps them to the canonical residues the reference produces (gnark fully reduces,
// jindo/internal/zp/element.go:397-466), so every output limb is bit-identical to ntt.go.
// The twiddle product is Shoup's precomputed-quotient multiply, exact for any 64-bit input:
//   wp = floor(w 2^64 / q),  qh = floor(y wp / 2^64),  y w - qh q  in [0, 2q).
// q mod 2^32 == 1 (every jindo-modulus prime: p - 1 = b^(2^e) with b even) turns lo64(qh q)
// into qh + ((qh_lo q_hi) << 32): one 32-bit multiply instead of three.
// Cost model (tools/ubench, MI355X): 32-bit multiplies, 64-bit shifts/adds and carry ops issue
// at ~4.4 cycles per wave64 instruction, plain v_add/v_sub/v_and/v_mov at ~2.4; a butterfly is
// 8 multiplies + ~13 adds/selects.
#pragma once
#include <stdint.h>

#include <algorithm>

#include "field.hpp"

namespace rg {

struct Q64 {
  uint64_t q, q2;  // q, 2q (2q < 2^64 needs q < 2^63; the lazy add below needs q < 2^64/3)
  uint32_t qhi;    // q >> 32
  uint32_t qlo1;   // q mod 2^32 == 1
};

RG_HD Q64 make_q64(uint64_t q) {
  Q64 Q;
  Q.q = q;
  Q.q2 = 2 * q;
  Q.qhi = (uint32_t)(q >> 32);
  Q.qlo1 = (uint32_t)q == 1u;
  return Q;
}

#if defined(__HIPCC__)

// y * w mod q in [0, 2q), exact Shoup for any y < 2^64
template <bool QLO1>
__device__ __forceinline__ uint64_t shoup2(uint64_t y, uint64_t w, uint64_t wp, const Q64& Q) {
  const uint32_t y0 = (uint32_t)y, y1 = (uint32_t)(y >> 32);
  const uint32_t p0 = (uint32_t)wp, p1 = (uint32_t)(wp >> 32);
  // qh = hi64(y * wp): mid = y0 p1 + y1 p0 + hi(y0 p0) < 2^65 carries at most once
  unsigned long long c1, c2;
  const uint64_t mid0 = __builtin_addcll((uint64_t)y0 * p1, (uint64_t)y1 * p0, 0ull, &c1);
  const uint64_t mid = __builtin_addcll(mid0, (uint64_t)__umulhi(y0, p0), 0ull, &c2);
  const uint64_t qh = (uint64_t)y1 * p1 + ((mid >> 32) | ((uint64_t)(c1 | c2) << 32));
  const uint32_t w0 = (uint32_t)w, w1 = (uint32_t)(w >> 32);
  if constexpr (QLO1) {
    const uint64_t l = (uint64_t)y0 * w0;
    const uint32_t hi = (uint32_t)(l >> 32) + y0 * w1 + y1 * w0 - (uint32_t)qh * Q.qhi;
    return (((uint64_t)hi << 32) | (uint32_t)l) - qh;
  } else {
    return y * w - qh * Q.q;
  }
}

// [0, 4q) sum as (value mod 2^64, carry) -> [0, 2q)
__device__ __forceinline__ uint64_t lazy_add(uint64_t x, uint64_t y, const Q64& Q) {
  unsigned long long c, b;
  const uint64_t s = __builtin_addcll(x, y, 0ull, &c);
  const uint64_t t = __builtin_subcll(s, Q.q2, 0ull, &b);
  return (c | (b ^ 1ull)) ? t : s;
}
// x - y + 2q (x, y in [0, 2q)) -> [0, 2q)
__device__ __forceinline__ uint64_t lazy_sub(uint64_t x, uint64_t y, const Q64& Q) {
  unsigned long long b;
  const uint64_t d = __builtin_subcll(x, y, 0ull, &b);
  return b ? d + Q.q2 : d;
}
// [0, 2q) -> [0, q)
__device__ __forceinline__ uint64_t canon(uint64_t x, const Q64& Q) {
  unsigned long long b;
  const uint64_t t = __builtin_subcll(x, Q.q, 0ull, &b);
  return b ? x : t;
}

// Cooley-Tukey (ntt.go:254-259): (x, y) <- (x + w y, x - w y), lazy in and out
template <bool QLO1 = true>
__device__ __forceinline__ void fwd_bfly_lazy(uint64_t& x, uint64_t& y, uint64_t w, uint64_t wp, const Q64& Q) {
  const uint64_t t = shoup2<QLO1>(y, w, wp, Q);
  const uint64_t a = x;
  x = lazy_add(a, t, Q);
  y = lazy_sub(a, t, Q);
}
// Gentleman-Sande (ntt.go:365-370): (x, y) <- (x + y, (x - y) w), lazy in and out
template <bool QLO1 = true>
__device__ __forceinline__ void inv_bfly_lazy(uint64_t& x, uint64_t& y, uint64_t w, uint64_t wp, const Q64& Q) {
  const uint64_t a = x, b = y;
  x = lazy_add(a, b, Q);
  y = shoup2<QLO1>(lazy_sub(a, b, Q), w, wp, Q);
}


// ---- explicit-carry forms (VOP3b carry outputs in SGPR lane masks; the compiler keeps the
// 32-bit halves of 64-bit values as sub-registers, so no pair is ever rebuilt) ----
typedef unsigned long long lmask;  // wave64 lane mask (SGPR pair)

__device__ __forceinline__ uint64_t mad_co(uint32_t a, uint32_t b, uint64_t c, lmask& co) {
  uint64_t d;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(co) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ uint32_t add_co(uint32_t a, uint32_t b, lmask& co) {
  uint32_t d;
  asm("v_add_co_u32 %0, %1, %2, %3" : "=v"(d), "=s"(co) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ uint32_t addc_co(uint32_t a, uint32_t b, lmask ci, lmask& co) {
  uint32_t d;
  asm("v_addc_co_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(co) : "v"(a), "v"(b), "s"(ci));
  return d;
}
__device__ __forceinline__ uint32_t sub_co(uint32_t a, uint32_t b, lmask& bo) {
  uint32_t d;
  asm("v_sub_co_u32 %0, %1, %2, %3" : "=v"(d), "=s"(bo) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ uint32_t subb_co(uint32_t a, uint32_t b, lmask bi, lmask& bo) {
  uint32_t d;
  asm("v_subb_co_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(bo) : "v"(a), "v"(b), "s"(bi));
  return d;
}
__device__ __forceinline__ uint32_t sel(lmask m, uint32_t if1, uint32_t if0) {
  uint32_t d;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(d) : "v"(if0), "v"(if1), "s"(m));
  return d;
}
__device__ __forceinline__ uint64_t pk(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
__device__ __forceinline__ uint32_t lo32(uint64_t v) { return (uint32_t)v; }
__device__ __forceinline__ uint32_t hi32(uint64_t v) { return (uint32_t)(v >> 32); }

// Shoup y * w mod q in [0, 2q), q mod 2^32 == 1; nqhi = -(q >> 32) mod 2^32
__device__ __forceinline__ uint64_t shoup_x(uint64_t y, uint64_t w, uint64_t wp, uint32_t nqhi) {
  const uint32_t y0 = lo32(y), y1 = hi32(y), p0 = lo32(wp), p1 = hi32(wp);
  lmask cb, k;
  const uint64_t a = (uint64_t)y0 * p1 + __umulhi(y0, p0);   // < 2^64
  const uint64_t b = mad_co(y1, p0, a, cb);                  // y1 p0 + a, carry into 2^96
  const uint64_t c = (uint64_t)y1 * p1 + hi32(b);            // < 2^64 (qh fits)
  const uint32_t qh0 = lo32(c);
  const uint32_t qh1 = addc_co(hi32(c), 0u, cb, k);
  const uint64_t l = (uint64_t)y0 * lo32(w);
  const uint32_t hi = hi32(l) + y0 * hi32(w) + y1 * lo32(w) + qh0 * nqhi;
  lmask br;
  const uint32_t r0 = sub_co(lo32(l), qh0, br);
  const uint32_t r1 = subb_co(hi, qh1, br, k);
  return pk(r0, r1);
}
// (x, y) <- (x + w y, x - w y), lazy [0, 2q) in and out; q2 = 2q
__device__ __forceinline__ void fwd_bfly_x(uint64_t& x, uint64_t& y, uint64_t w, uint64_t wp, uint64_t q2,
                                           uint32_t nqhi) {
  const uint64_t t = shoup_x(y, w, wp, nqhi);
  lmask c, c2, b, b2, e, e2;
  const uint32_t s0 = add_co(lo32(x), lo32(t), c);
  const uint32_t s1 = addc_co(hi32(x), hi32(t), c, c2);
  const uint32_t u0 = sub_co(s0, lo32(q2), b);
  const uint32_t u1 = subb_co(s1, hi32(q2), b, b2);
  const lmask m = c2 | ~b2;  // s >= 2q (65-bit)
  const uint32_t d0 = sub_co(lo32(x), lo32(t), e);
  const uint32_t d1 = subb_co(hi32(x), hi32(t), e, e2);
  const uint64_t d = pk(d0, d1);
  const uint64_t f = d + q2;
  x = pk(sel(m, u0, s0), sel(m, u1, s1));
  y = pk(sel(e2, lo32(f), d0), sel(e2, hi32(f), d1));
}


// (x, y) <- (x + y, (x - y) w), lazy [0, 2q) in and out
__device__ __forceinline__ void inv_bfly_x(uint64_t& x, uint64_t& y, uint64_t w, uint64_t wp, uint64_t q2,
                                           uint32_t nqhi) {
  lmask c, c2, b, b2, e, e2;
  const uint32_t s0 = add_co(lo32(x), lo32(y), c);
  const uint32_t s1 = addc_co(hi32(x), hi32(y), c, c2);
  const uint32_t u0 = sub_co(s0, lo32(q2), b);
  const uint32_t u1 = subb_co(s1, hi32(q2), b, b2);
  const lmask m = c2 | ~b2;
  const uint32_t d0 = sub_co(lo32(x), lo32(y), e);
  const uint32_t d1 = subb_co(hi32(x), hi32(y), e, e2);
  const uint64_t d = pk(d0, d1);
  const uint64_t f = d + q2;
  x = pk(sel(m, u0, s0), sel(m, u1, s1));
  y = shoup_x(pk(sel(e2, lo32(f), d0), sel(e2, hi32(f), d1)), w, wp, nqhi);
}
// [0, 2q) -> [0, q)
__device__ __forceinline__ uint64_t canon_x(uint64_t x, uint64_t q) {
  lmask b, b2;
  const uint32_t t0 = sub_co(lo32(x), lo32(q), b);
  const uint32_t t1 = subb_co(hi32(x), hi32(q), b, b2);
  return pk(sel(b2, lo32(x), t0), sel(b2, hi32(x), t1));
}

// ----------------------------------------------------------------------------------------
// Pass kernel: 8 consecutive radix-2 stages [G0, G0+8) of a 2^logN-point transform, as 2^(logN-8)
// independent 256-point sub-transforms per polynomial whose points sit at stride S =
// 2^(logN-G0-8): COL (S >= 16, G0 = 0) or ROW (S = 1).  A 512-thread workgroup owns a tile of
// 16 sub-transforms x 256 points = 32 KiB; each thread holds 8 points in registers and runs
// three rounds of 3 + 3 + 2 stages with two LDS exchanges (plus one transpose for coalesced
// ROW stores/loads).  Index algebra (ntt.go:98-115 forward, :357-466 inverse): local stage k
// combines bit b = 7-k of the in-sub-transform index x and uses
//     tw[2^(G0+k) + (hi << k) + (x >> (b+1))],   hi = sub-transform prefix (ROW: row index).
// Register patterns per round (t = lane's slot, y / r = register):
//     H: x = t + 32 y   (window bits [5,8))       M: x = (t>>2)<<5 | y<<2 | (t&3)   (bits [2,5))
//     L: x = 8 t + r    (window bits [0,2), r>>2 = x bit 2)
// ----------------------------------------------------------------------------------------
struct Ntt64Args {
  const uint64_t* in;
  uint64_t* out;
  // (w, floor(w 2^64 / q)) pairs, forward or inverse: [N] in the reference order tw[m + i]
  // (ntt.go:153-203), then for N = 2^16 a lane-ordered copy of the ROW pass's last two stages:
  // row r, stage 14: [r*192 + 32 g + t] = tw[2^14 + 64 r + 2 t + g]       (g < 2,  t < 32)
  //        stage 15: [r*192 + 64 + 32 j + t] = tw[2^15 + 128 r + 4 t + j] (j < 4)
  const uint64_t* tw;
  uint64_t q, q2;
  uint32_t nqhi, pad_;
  uint64_t ninv, ninv_p;  // N^-1 and its Shoup quotient (inverse, last stage)
  uint64_t w1n, w1n_p;    // twInv[1] N^-1
  long long total_sub;    // batch * 2^(logN - 8)
  int logN, G0;
  int rev;  // 1: tiles in reverse order (a transform's second pass: Infinity Cache reuse, rg_bstore)
};

// ----------------------------------------------------------------------------------------
// N = 2^16 pass kernel: compile-time strides, buffer addressing (one VGPR offset per access
// pattern, per-access constants in SGPR soffsets / immediates) and one tile per workgroup, so
// no address is held in registers across the tile.  COL = global stages [0, 8) on the 256
// columns (stride 256), ROW = [8, 16) on the 256 rows.
// Tiles: COL = 16 adjacent columns of one polynomial.  ROW = 16 rows; with RP ("row-major over
// polynomials", batch % 16 == 0) the 16 rows are the SAME row of 16 consecutive polynomials,
// so every twiddle of the tile is shared by all 16 sub-transforms (as in COL): the first
// round's twiddles come from scalar loads and the others are loaded once per lane slot t,
// shared by both half-waves.  Without RP the 16 rows are 16 consecutive rows of one poly.
// ----------------------------------------------------------------------------------------
typedef unsigned int rg_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int rg_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rg_buf(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
// cache policy of the transform's data: loads nt, stores default.  A transform's second pass
// runs its tiles in reverse order (Ntt64Args::rev), so it starts on the polynomials its first pass
// wrote last, which the default-policy stores left in the 256 MiB Infinity Cache; the next call's
// first pass (forward order) likewise starts where this second pass ended.  Round 5: 0.902 ->
// 0.889 ms per step against nt stores in forward order (nt on both, in forward order, had been
// -3% against the default in round 2; the default alone without the reversal is +5%).  The
// M- and L-round twiddles are staged in LDS per tile for COL and RP
// tiles (L round -0.6% per step, M round a further -2.3%, against per-lane global loads that
// queue behind the tile's HBM traffic); s_setprio on the tile loads (+6%) or on the
// butterflies (+5%) measured slower.
constexpr int kNttAux = 2, kNttAuxSt = 0;
__device__ __forceinline__ uint64_t rg_bload(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  const rg_u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, kNttAux);
  return pk(v.x, v.y);
}
__device__ __forceinline__ void rg_bstore(uint64_t x, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  rg_u32x2 v;
  v.x = lo32(x);
  v.y = hi32(x);
  __builtin_amdgcn_raw_buffer_store_b64(v, r, voff, soff, kNttAuxSt);
}

// PROBE (tuning only; production = 0): 1 = twiddles from registers (no table loads),
// 2 = butterflies replaced by one add (memory / LDS / twiddle-load floor), 3 = both,
// 4 = no global data loads / stores (the tile is synthesised from the thread index and its
// result kept live by a store that never fires): the compute floor (butterflies, twiddle loads,
// LDS exchanges) of the same launch, timed by bench.py through rg_set_probe
// LTW / MTW: the L round (PAT 2) and the M round (PAT 1) read their twiddles from the tile's LDS
// copy `ltw` (248 entries staged by ntt16_tile: COL tw[8, 256); RP the row's lane-ordered L-round
// copy, then its 56 stage 3-5 entries) instead of per-lane global loads
template <int RK, int LO, int PAT, bool INV, bool SCALE, bool COL, bool RP, int PROBE>
__device__ __forceinline__ void ntt16_round(const Ntt64Args& a, __amdgpu_buffer_rsrc_t twr, uint64_t (&e)[8],
                                            uint32_t hi, uint32_t t, const ulonglong2* ltw = nullptr) {
  constexpr bool LTW = PAT == 2 && (COL || RP);
  constexpr int G0 = COL ? 0 : 8;
  // twiddle index independent of the lane: the H round of COL / RP tiles.  (The M round of COL
  // tiles is wave-uniform too, x >> (b + 1) depending on t >> 2 = tid >> 6 only, but scalar loads
  // there measured no faster: their lgkmcnt waits also wait for the exchange's LDS traffic.)
  constexpr bool UNIFORM = (COL || RP) && PAT == 0;
  constexpr bool MTW = PAT == 1 && (COL || RP) && (PROBE & 1) == 0;
  auto xof = [&](int rho) -> uint32_t {
    if (PAT == 0) return t + 32u * rho;
    if (PAT == 1) return ((t >> 2) << 5) | ((uint32_t)rho << 2) | (t & 3u);
    return 8u * t + rho;
  };
  constexpr int NPK = 1 << RK;
#pragma unroll
  for (int sp = 0; sp < RK; ++sp) {
    const int bw = INV ? sp : (RK - 1 - sp);
    const int b = LO + bw;
    const int k = 7 - b;
    const int half = 1 << bw;
    const bool last = INV && SCALE && k == 0;  // SCALE: this pass holds global stage 0
    uint64_t w[4], wp[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int grp = j / (NPK / 2), jj = j % (NPK / 2);
      const int rho0 = grp * NPK + ((jj >> bw) << (bw + 1)) + (jj & (half - 1));
      if ((jj & (half - 1)) != 0) {  // same x >> (b+1) as the previous pair
        w[j] = w[j - 1];
        wp[j] = wp[j - 1];
        continue;
      }
      if (last) {
        w[j] = a.w1n;
        wp[j] = a.w1n_p;
        continue;
      }
      if constexpr ((PROBE & 1) != 0) {
        w[j] = a.w1n + (xof(rho0) >> (b + 1)) + hi;
        wp[j] = a.w1n_p;
      } else if constexpr (UNIFORM) {
        const uint32_t idx = (1u << (G0 + k)) + (hi << k) + (xof(rho0) >> (b + 1));
        const uint32_t iu = __builtin_amdgcn_readfirstlane(idx);
        const ulonglong2 v = reinterpret_cast<const ulonglong2*>(a.tw)[iu];
        w[j] = v.x;
        wp[j] = v.y;
      } else if constexpr (LTW && COL) {
        const ulonglong2 v = ltw[(1u << k) + (xof(rho0) >> (b + 1)) - 8u];
        w[j] = v.x;
        wp[j] = v.y;
      } else if constexpr (LTW) {
        const ulonglong2 v = ltw[(k == 6 ? 32u * grp : 64u + 32u * (rho0 >> 1)) + t];
        w[j] = v.x;
        wp[j] = v.y;
      } else if constexpr (MTW) {  // M round: COL tw[8, 64) ahead of the L round's; RP the row's stage 3-5 entries after them
        const ulonglong2 v = COL ? ltw[(1u << k) + (xof(rho0) >> (b + 1)) - 8u]
                                 : ltw[192u + (k == 3 ? 0u : k == 4 ? 8u : 24u) + (xof(rho0) >> (b + 1))];
        w[j] = v.x;
        wp[j] = v.y;
      } else if constexpr (!COL && PAT == 2) {
        // ROW last round (stages 14, 15): lane-ordered copy after the natural table, lane t's
        // j-th twiddle at t + 32 j, so every load is one coalesced 512-B run
        const uint32_t pos = (65536u + hi * 192u) + (k == 6 ? 32u * grp : 64u + 32u * (rho0 >> 1)) + t;
        const rg_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(twr, pos * 16u, 0, 0);
        w[j] = pk(v.x, v.y);
        wp[j] = pk(v.z, v.w);
      } else {
        const uint32_t idx = (1u << (G0 + k)) + (hi << k) + (xof(rho0) >> (b + 1));
        const rg_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(twr, idx * 16u, 0, 0);
        w[j] = pk(v.x, v.y);
        wp[j] = pk(v.z, v.w);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int grp = j / (NPK / 2), jj = j % (NPK / 2);
      const int rho0 = grp * NPK + ((jj >> bw) << (bw + 1)) + (jj & (half - 1));
      const int rho1 = rho0 + half;
      if constexpr ((PROBE & 2) != 0) {
        e[rho0] += e[rho1] ^ w[j] ^ wp[j];
      } else if constexpr (!INV) {
        fwd_bfly_x(e[rho0], e[rho1], w[j], wp[j], a.q2, a.nqhi);
      } else {
        inv_bfly_x(e[rho0], e[rho1], w[j], wp[j], a.q2, a.nqhi);
        if (last) e[rho0] = shoup_x(e[rho0], a.ninv, a.ninv_p, a.nqhi);
      }
    }
  }
}

// One 16 x 256 tile.  LDS images (u64 index):
//   COL: transposed [x][s] image 16 x + s + 16 (x >> 3) for every exchange; per pattern this is
//        a lane base plus compile-time offsets: H (x = t + 32 y): 16t + s + 16(t>>3) + 576 y;
//        M (x = 32(t>>2) + 4y + (t&3)): s + 16(t&3) + 576(t>>2) + 64 y + 16(y>>1);
//        L (x = 8t + r): 144 t + s + 16 r.
//   ROW: [s][x] rows of 288 with a per-exchange pad: H<->M pad 4(x>>5), M<->L pad (x>>3),
//        L<->H pad (x>>5).
// Every pattern pair was checked conflict-free for ds_*_b64 half-wave groups
// (SQ_LDS_BANK_CONFLICT = 0 for COL in profiles/r01_ntt16_pmc_summary.txt).
template <bool INV, bool COL, bool SCALE, bool CANON, bool RP, int PROBE = 0>
__device__ __forceinline__ void ntt16_tile(const Ntt64Args& a, uint32_t tile, uint64_t* lds, ulonglong2* ltw) {
  const uint32_t tid = threadIdx.x;
  const uint32_t s = COL ? (tid & 15u) : (tid >> 5);
  const uint32_t t = COL ? (tid >> 4) : (tid & 31u);
  // tile base (elements) and the stride between the tile's ROW sub-transforms
  //   COL: poly * 2^16 + column block * 16
  //   ROW: 16 consecutive rows (tile * 4096), or RP: row (tile & 255) of polys 16 (tile >> 8) + s
  const size_t tbase = COL  ? (((size_t)(tile >> 4) << 16) + ((tile & 15u) << 4))
                       : RP ? (((size_t)(tile >> 8) << 20) + ((tile & 255u) << 8))
                            : ((size_t)tile << 12);
  constexpr uint32_t RSH = RP ? 16 : 8;  // log2 of the ROW sub-transform stride (elements)
  const __amdgpu_buffer_rsrc_t rin = rg_buf(a.in + tbase);
  const __amdgpu_buffer_rsrc_t rout = rg_buf(a.out + tbase);
  const __amdgpu_buffer_rsrc_t twr = rg_buf(a.tw);
  const uint32_t hi = COL ? 0u : RP ? (uint32_t)__builtin_amdgcn_readfirstlane(tile & 255u) : (((tile << 4) + s) & 255u);
  uint64_t e[8];
  constexpr bool LTW = (COL || RP) && (PROBE & 1) == 0;
  // The M and L rounds' 248 twiddle pairs, one 8-B word per thread (496 threads): the word is
  // loaded after the tile's data loads and written to LDS just before the first barrier, so no
  // wave waits for it before issuing its data loads (the first load's latency would otherwise
  // open every tile).  COL: tw[8, 256); RP: the row's lane-ordered L-round copy, then its 56
  // stage 3-5 entries.
  const bool stv_on = LTW && tid < 496u;
  uint32_t st_src = 0, st_dst = tid;
  if constexpr (COL) {
    st_src = 16u + tid;
  } else if (tid < 384u) {
    st_src = 2u * (65536u + hi * 192u) + tid;
  } else {
    const uint32_t wd = tid - 384u, ent = wd >> 1;
    const uint32_t kk = ent < 8u ? 3u : ent < 24u ? 4u : 5u, j = ent - (kk == 3u ? 0u : kk == 4u ? 8u : 24u);
    st_src = 2u * ((1u << (8u + kk)) + (hi << kk) + j) + (wd & 1u);
    st_dst = 2u * (192u + ent) + (wd & 1u);
  }
  uint64_t stv = 0;
  auto stage_write = [&]() {
    if (stv_on) reinterpret_cast<uint64_t*>(ltw)[st_dst] = stv;
  };
  // ---- global load
  if constexpr ((PROBE & 4) != 0) {
#pragma unroll
    for (int y = 0; y < 8; ++y) e[y] = (uint64_t)(tid * 0x9E3779B9u + tile * 8u + (uint32_t)y);
  } else if constexpr (COL) {
    if constexpr (!INV) {
      const uint32_t vo = ((t << 8) + s) * 8u;
#pragma unroll
      for (int y = 0; y < 8; ++y) e[y] = rg_bload(rin, vo, (uint32_t)y << 16);
    } else {
      const uint32_t vo = ((t << 11) + s) * 8u;
#pragma unroll
      for (int r = 0; r < 8; ++r) e[r] = rg_bload(rin, vo, (uint32_t)r << 11);
    }
  } else {
    const uint32_t vo = ((s << RSH) + t) * 8u;
#pragma unroll
    for (int y = 0; y < 8; ++y) e[y] = rg_bload(rin, vo + 256u * y, 0);
  }
  if (stv_on) stv = reinterpret_cast<const uint64_t*>(a.tw)[st_src];
  // PROBE & 4: the result stays live through a store that never fires (values are < 2q < 2^64 - 1)
  auto st64 = [&](uint64_t x, uint32_t voff, uint32_t soff) {
    if constexpr ((PROBE & 4) != 0) {
      if (x == ~0ull) rg_bstore(x, rout, voff, soff);
    } else {
      rg_bstore(x, rout, voff, soff);
    }
  };
  const uint32_t bH = 16 * t + s + 16 * (t >> 3), bM = s + 16 * (t & 3) + 576 * (t >> 2), bL = 144 * t + s;
  auto offM = [](int y) { return 64 * y + 16 * (y >> 1); };
  const uint32_t rH = 288 * s + t, rM = 288 * s + 36 * (t >> 2) + (t & 3), rL9 = 288 * s + 9 * t,
                 rL8 = 288 * s + 8 * t + (t >> 2);
  if constexpr (!INV) {
    ntt16_round<3, 5, 0, false, false, COL, RP, PROBE>(a, twr, e, hi, t);
    stage_write();
    // exchange H -> M
#pragma unroll
    for (int y = 0; y < 8; ++y) lds[COL ? bH + 576 * y : rH + 36 * y] = e[y];
    __syncthreads();
#pragma unroll
    for (int y = 0; y < 8; ++y) e[y] = lds[COL ? bM + offM(y) : rM + 4 * y];
    ntt16_round<3, 2, 1, false, false, COL, RP, PROBE>(a, twr, e, hi, t, ltw);
    __syncthreads();
    // exchange M -> L
#pragma unroll
    for (int y = 0; y < 8; ++y) lds[COL ? bM + offM(y) : rM + 4 * y + (y >> 1)] = e[y];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; ++r) e[r] = lds[COL ? bL + 16 * r : rL9 + r];
    ntt16_round<2, 0, 2, false, false, COL, RP, PROBE>(a, twr, e, hi, t, ltw);
    if (CANON) {
#pragma unroll
      for (int r = 0; r < 8; ++r) e[r] = canon_x(e[r], a.q);
    }
    if constexpr (COL) {
      const uint32_t vo = ((t << 11) + s) * 8u;
#pragma unroll
      for (int r = 0; r < 8; ++r) st64(e[r], vo, (uint32_t)r << 11);
    } else {  // L -> H through LDS (pad x >> 5), then coalesced rows
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 8; ++r) lds[rL8 + r] = e[r];
      __syncthreads();
      const uint32_t vo = ((s << RSH) + t) * 8u;
#pragma unroll
      for (int y = 0; y < 8; ++y) st64(lds[rH + 33 * y], vo + 256u * y, 0);
    }
  } else {
    stage_write();
    if constexpr (!COL) {  // ROW inverse: loaded in H, transpose to L (pad x >> 5)
#pragma unroll
      for (int y = 0; y < 8; ++y) lds[rH + 33 * y] = e[y];
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 8; ++r) e[r] = lds[rL8 + r];
      __syncthreads();
    }
    if constexpr (COL && LTW) __syncthreads();  // the staged twiddles (ROW's transpose has its barrier)
    ntt16_round<2, 0, 2, true, SCALE, COL, RP, PROBE>(a, twr, e, hi, t, ltw);
    // exchange L -> M
#pragma unroll
    for (int r = 0; r < 8; ++r) lds[COL ? bL + 16 * r : rL9 + r] = e[r];
    __syncthreads();
#pragma unroll
    for (int y = 0; y < 8; ++y) e[y] = lds[COL ? bM + offM(y) : rM + 4 * y + (y >> 1)];
    ntt16_round<3, 2, 1, true, SCALE, COL, RP, PROBE>(a, twr, e, hi, t, ltw);
    __syncthreads();
    // exchange M -> H
#pragma unroll
    for (int y = 0; y < 8; ++y) lds[COL ? bM + offM(y) : rM + 4 * y] = e[y];
    __syncthreads();
#pragma unroll
    for (int y = 0; y < 8; ++y) e[y] = lds[COL ? bH + 576 * y : rH + 36 * y];
    ntt16_round<3, 5, 0, true, SCALE, COL, RP, PROBE>(a, twr, e, hi, t);
    if (CANON) {
#pragma unroll
      for (int y = 0; y < 8; ++y) e[y] = canon_x(e[y], a.q);
    }
    if constexpr (COL) {
      const uint32_t vo = ((t << 8) + s) * 8u;
#pragma unroll
      for (int y = 0; y < 8; ++y) st64(e[y], vo, (uint32_t)y << 16);
    } else {
      const uint32_t vo = ((s << RSH) + t) * 8u;
#pragma unroll
      for (int y = 0; y < 8; ++y) st64(e[y], vo + 256u * y, 0);
    }
  }
}

template <bool INV, bool COL, bool SCALE, bool CANON, bool RP = false, int MINW = 1, int PROBE = 0>
__global__ __launch_bounds__(512, MINW) void ntt16_pass(Ntt64Args a) {
  __shared__ uint64_t lds[16 * 288];
  __shared__ ulonglong2 ltw[COL || RP ? 248 : 1];  // 39.9 KiB per workgroup with lds: 4 per CU
  const uint32_t tile = a.rev ? gridDim.x - 1u - blockIdx.x : blockIdx.x;
  ntt16_tile<INV, COL, SCALE, CANON, RP, PROBE>(a, tile, lds, ltw);
}

#endif  // __HIPCC__

}  // namespace rg
