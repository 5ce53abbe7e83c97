// ntt256.hpp -- degree-2^16 NTT for 4-limb fields with q = 1 mod 2^64 and q < 2^255: the Jindo
// default prime q255 = 60272^16 + 1 = 3767^16 * 2^64 + 1 (jindo/internal/zp/element.go:32,47-50),
// the "multi-limb jindo-modulus prime" of BASELINE configs[3].
//
// Elements are gnark Montgomery residues (R = 2^256, little-endian u64 limbs); twiddles are
// the reference's Montgomery tables tw[m + i] (math/bigpoly/ntt.go:153-203) so
// mont(v, tw) = v * w exactly as ntt.go's butterfly (ntt.go:254-259).  Values between stages
// are lazy in [0, 2q) (2q < 2^256), the last pass maps to [0, q): outputs are bit-identical.
//
// Montgomery product on 32-bit digits, product scanning with a 96-bit column accumulator: per
// partial product one v_mad_u64_u32 with carry-out plus one v_addc.  q = 1 mod 2^64 makes the
// quotient digit m_k = -t_k mod 2^32 (no multiply) and q's digits 0, 1 are (1, 0), so the
// reduction needs 6 x 8 products instead of 8 x 8: 112 products per modmul.
// Structure as ntt16_pass (ntt64.hpp): two 8-stage passes (COL, ROW), one tile per workgroup,
// here 4 sub-transforms x 256 points (32 KiB) per 128-thread workgroup, 8 points per thread,
// rounds of 3 + 3 + 2 stages through limb-planar LDS images.
#pragma once
#include <stdint.h>

#include "ntt64.hpp"

namespace rg {

struct Ntt256Args {
  const uint64_t* in;
  uint64_t* out;
  const uint64_t* tw;  // Montgomery twiddles [N][4]
  uint32_t q[8], q2[8];
  uint32_t w1n[8];           // twInv[1] N^-1, Montgomery
  long long total_sub;       // batch * 256
};

#if defined(__HIPCC__)

// z = x y 2^-256 mod q, z < 2q, for x < 2q, y < q
__device__ __forceinline__ void mont256(uint32_t (&z)[8], const uint32_t (&x)[8], const uint32_t (&y)[8],
                                        const uint32_t (&q)[8]) {
  uint32_t m[8];
  uint64_t A = 0;
  uint32_t H = 0;
#pragma unroll
  for (int k = 0; k < 15; ++k) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      lmask c, c2;
      A = mad_co(x[i], y[j], A, c);
      H = addc_co(H, 0u, c, c2);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int j = k - i;
      if (i >= k || j < 2 || j > 7) continue;
      lmask c, c2;
      A = mad_co(m[i], q[j], A, c);
      H = addc_co(H, 0u, c, c2);
    }
    if (k < 8) {
      // m_k = -A mod 2^32: A + m_k * q_0 clears the digit and carries (A_lo != 0) into the next
      lmask br, c2, c3;
      m[k] = sub_co(0u, lo32(A), br);  // borrow = (A_lo != 0) = the carry out of A_lo + m_k
      const uint32_t lo = addc_co(hi32(A), 0u, br, c2);
      A = pk(lo, addc_co(H, 0u, c2, c3));
    } else {
      z[k - 8] = lo32(A);
      A = pk(hi32(A), H);
    }
    H = 0;
  }
  z[7] = lo32(A);
}

// x * 2^-SH mod q for q = 1 mod 2^SH (the N^-1 of N = 2^SH, ntt.go:242-243): with
// k = -x mod 2^SH, x + k q is divisible by 2^SH and (x + k q) / 2^SH < 2q for x < 2q.
// q's digits 0, 1 are (1, 0): k q = k + sum_{j>=2} k q_j 2^(32 j).
template <int SH>
__device__ __forceinline__ void div2p_256(uint32_t (&x)[8], const uint32_t (&q)[8]) {
  static_assert(SH >= 1 && SH <= 31, "shift");
  const uint32_t k = (0u - x[0]) & ((1u << SH) - 1u);
  uint32_t y[9];
  uint64_t acc = (uint64_t)x[0] + k;
  y[0] = lo32(acc);
  acc = (uint64_t)x[1] + hi32(acc);
  y[1] = lo32(acc);
#pragma unroll
  for (int j = 2; j < 8; ++j) {
    acc = (uint64_t)k * q[j] + x[j] + hi32(acc);
    y[j] = lo32(acc);
  }
  y[8] = hi32(acc);
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = __builtin_amdgcn_alignbit(y[j + 1], y[j], SH);
}

// x + y (x, y < 2q, sum < 4q < 2^257) -> [0, 2q)
__device__ __forceinline__ void lazy_add256(uint32_t (&r)[8], const uint32_t (&x)[8], const uint32_t (&y)[8],
                                            const uint32_t (&q2)[8]) {
  uint32_t s[8], u[8];
  lmask c, b;
  s[0] = add_co(x[0], y[0], c);
#pragma unroll
  for (int i = 1; i < 8; ++i) s[i] = addc_co(x[i], y[i], c, c);
  u[0] = sub_co(s[0], q2[0], b);
#pragma unroll
  for (int i = 1; i < 8; ++i) u[i] = subb_co(s[i], q2[i], b, b);
  const lmask m = c | ~b;
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = sel(m, u[i], s[i]);
}
// x - y + 2q if negative -> [0, 2q)
__device__ __forceinline__ void lazy_sub256(uint32_t (&r)[8], const uint32_t (&x)[8], const uint32_t (&y)[8],
                                            const uint32_t (&q2)[8]) {
  uint32_t d[8], f[8];
  lmask b, c;
  d[0] = sub_co(x[0], y[0], b);
#pragma unroll
  for (int i = 1; i < 8; ++i) d[i] = subb_co(x[i], y[i], b, b);
  f[0] = add_co(d[0], q2[0], c);
#pragma unroll
  for (int i = 1; i < 8; ++i) f[i] = addc_co(d[i], q2[i], c, c);
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = sel(b, f[i], d[i]);
}
__device__ __forceinline__ void canon256(uint32_t (&x)[8], const uint32_t (&q)[8]) {
  uint32_t u[8];
  lmask b;
  u[0] = sub_co(x[0], q[0], b);
#pragma unroll
  for (int i = 1; i < 8; ++i) u[i] = subb_co(x[i], q[i], b, b);
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = sel(b, x[i], u[i]);
}

// Butterfly bodies.  Inlined: the tile is ~18K instructions, but the four independent
// butterflies of a stage interleave; out of line (__noinline__, 2.2K-instruction kernels) they
// measured 1.5x slower (the calls serialise the butterflies).
struct D8 {
  uint32_t d[8];
};
struct D16 {
  D8 x, y;
};
#define RG_NTT256_BFLY __device__ __forceinline__
RG_NTT256_BFLY D16 bfly_fwd256(D8 x, D8 y, D8 w, const Ntt256Args* a) {
  uint32_t tt[8];
  D16 r;
  mont256(tt, y.d, w.d, a->q);
  lazy_sub256(r.y.d, x.d, tt, a->q2);
  lazy_add256(r.x.d, x.d, tt, a->q2);
  return r;
}
RG_NTT256_BFLY D16 bfly_inv256(D8 x, D8 y, D8 w, const Ntt256Args* a) {
  uint32_t d[8];
  D16 r;
  lazy_sub256(d, x.d, y.d, a->q2);
  lazy_add256(r.x.d, x.d, y.d, a->q2);
  mont256(r.y.d, d, w.d, a->q);
  return r;
}

// LOGC: bits of the pass's sub-transform (8: 256 points; 7: the 128-point COL pass of N = 2^15,
// whose patterns are H x = t + 16 y, M x = (y>>2) 64 + (t>>2) 16 + (y&3) 4 + (t&3), L x = 8 t + r)
template <int RK, int LO, int PAT, bool INV, bool SCALE, bool COL, int LOGN = 16, int LOGC = 8>
__device__ __forceinline__ void ntt256_round(const Ntt256Args& a, __amdgpu_buffer_rsrc_t twr, uint32_t (&e)[8][8],
                                             uint32_t hi, uint32_t t, bool rowuni) {
  constexpr int G0 = COL ? 0 : LOGN - 8;
  auto xof = [&](int rho) -> uint32_t {
    if (PAT == 0) return t + (1u << (LOGC - 3)) * rho;
    if (PAT == 1) {
      if (LOGC == 8) return ((t >> 2) << 5) | ((uint32_t)rho << 2) | (t & 3u);
      return ((uint32_t)(rho >> 2) << 6) | ((t >> 2) << 4) | ((uint32_t)(rho & 3) << 2) | (t & 3u);
    }
    return 8u * t + rho;
  };
  constexpr int NPK = 1 << RK;
#pragma unroll
  for (int sp = 0; sp < RK; ++sp) {
    const int bw = INV ? sp : (RK - 1 - sp);
    const int b = LO + bw;
    const int k = LOGC - 1 - b;
    const int half = 1 << bw;
    const bool last = INV && SCALE && k == 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int grp = j / (NPK / 2), jj = j % (NPK / 2);
      const int rho0 = grp * NPK + ((jj >> bw) << (bw + 1)) + (jj & (half - 1));
      const int rho1 = rho0 + half;
      uint32_t w[8];
      if (last) {
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = a.w1n[i];
      } else {
        const uint32_t idx = (1u << (G0 + k)) + (hi << k) + (xof(rho0) >> (b + 1));
        if ((COL || rowuni) && PAT == 0) {  // wave-uniform index: scalar loads
          const uint32_t iu = __builtin_amdgcn_readfirstlane(idx);
          const uint32_t* p = reinterpret_cast<const uint32_t*>(a.tw) + 8u * iu;
#pragma unroll
          for (int i = 0; i < 8; ++i) w[i] = p[i];
        } else {
          const rg_u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(twr, idx * 32u, 0, 0);
          const rg_u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(twr, idx * 32u + 16u, 0, 0);
          w[0] = v0.x; w[1] = v0.y; w[2] = v0.z; w[3] = v0.w;
          w[4] = v1.x; w[5] = v1.y; w[6] = v1.z; w[7] = v1.w;
        }
      }
      D8 X, Y, W;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        X.d[i] = e[rho0][i];
        Y.d[i] = e[rho1][i];
        W.d[i] = w[i];
      }
      const D16 R = INV ? bfly_inv256(X, Y, W, &a) : bfly_fwd256(X, Y, W, &a);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        e[rho0][i] = R.x.d[i];
        e[rho1][i] = R.y.d[i];
      }
      if constexpr (INV) {
        if (last) div2p_256<LOGN>(e[rho0], a.q);  // (u + v) N^-1, N = 2^LOGN
      }
    }
  }
}

// One tile of 4 sub-transforms x 256 points.  LDS: limb planes (u64) of [s][x] rows:
//   COL: pitch 296, pad (x >> 3) for every exchange; ROW: pitch 288, pads 4(x>>5) (H<->M),
//   (x>>3) (M<->L), (x>>5) (L<->H) -- conflict-free for ds_*_b64 half-wave groups (checked by
//   enumeration, tools/nttlab/banks.py).
// An exchange moves the 4 limb planes through an LDS image of kNtt256Planes planes: with 2,
// two rounds of (put, barrier, get) of 2 planes each, so a 128-thread workgroup holds 18.9 KiB
// instead of 37.9 KiB and occupancy is set by VGPRs (3-4 waves/SIMD), not LDS (2 waves/SIMD).
// (amdgpu_waves_per_eu(4), a 128-VGPR cap, spilled 1-26 VGPRs and measured 3% slower: round 2)
constexpr int kNtt256Planes = 2;
// LOGN = 16 (COL and ROW both 8-stage passes) or 15 (COL: 7 stages on 256 columns of 128 points,
// 8 of them per tile; ROW: 8 stages on 128 rows of 256 points), as ntt.hip plans them.
// PROBE (experiments build only, rg_set_probe(5); production = 0): 1 = no HBM data movement,
// the tile synthesised in registers and the result kept live by a store that never fires, so the
// same launch times the butterflies, twiddle loads and LDS exchanges alone.
template <bool INV, bool COL, bool SCALE, bool CANON, bool RP, int LOGN = 16, int PROBE = 0>
__global__ __launch_bounds__(128) void ntt256_pass(Ntt256Args a) {
  static_assert(LOGN == 15 || LOGN == 16, "ntt256_pass: N = 2^15 or 2^16");
  constexpr int LOGC = COL ? LOGN - 8 : 8;        // bits of a sub-transform
  constexpr uint32_t CPT = COL ? (1024u >> LOGC) : 4u;  // sub-transforms per tile
  constexpr int PITCH = COL ? (LOGC == 8 ? 296 : 148) : 288, PLANE = (int)CPT * PITCH;
  constexpr int NPL = kNtt256Planes;  // limb planes per LDS round (4 or 2)
  static_assert(NPL == 4 || NPL == 2, "kNtt256Planes");
  constexpr uint32_t R = 1u << (LOGN - 8);  // ROW: rows per polynomial; COL: tiles per polynomial x CPT / 256
  __shared__ uint64_t lds[NPL * PLANE];
  const uint32_t tid = threadIdx.x;
  const uint32_t s = COL ? (tid % CPT) : (tid >> 5);
  const uint32_t t = COL ? (tid / CPT) : (tid & 31u);
  const uint32_t tile = blockIdx.x;
  // element (32 B) offsets: COL: poly * 2^LOGN + CPT * column block;  ROW: RP: row (tile % R) of
  // polys 4 (tile / R) + s, else 4 consecutive rows
  constexpr uint32_t TPP = 256u / CPT;  // COL tiles per polynomial
  const size_t tbase = COL  ? (((size_t)(tile / TPP) << LOGN) + (tile % TPP) * CPT)
                       : RP ? (((size_t)(tile / R) << (LOGN + 2)) + ((tile % R) << 8))
                            : ((size_t)tile << 10);
  constexpr uint32_t SSH = COL ? 0 : (RP ? LOGN : 8);  // log2 sub-transform stride (elements)
  constexpr uint32_t XSH = COL ? 8 : 0;                // log2 point stride (elements)
  const __amdgpu_buffer_rsrc_t rin = rg_buf(a.in + 4 * tbase);
  const __amdgpu_buffer_rsrc_t rout = rg_buf(a.out + 4 * tbase);
  const __amdgpu_buffer_rsrc_t twr = rg_buf(a.tw);
  const uint32_t hi = COL ? 0u : RP ? (uint32_t)__builtin_amdgcn_readfirstlane(tile % R) : (((tile << 2) + s) & (R - 1u));
  uint32_t e[8][8];
  auto gload = [&](int reg, uint32_t x) {
    const uint32_t off = ((s << SSH) + (x << XSH)) * 32u;
    if constexpr (PROBE != 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) e[reg][i] = (off + (uint32_t)i) * 0x9E3779B9u + tile;
      e[reg][7] &= 0x3fffffffu;
      return;
    }
    const rg_u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, 0);
    const rg_u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(rin, off + 16u, 0, 0);
    e[reg][0] = v0.x; e[reg][1] = v0.y; e[reg][2] = v0.z; e[reg][3] = v0.w;
    e[reg][4] = v1.x; e[reg][5] = v1.y; e[reg][6] = v1.z; e[reg][7] = v1.w;
  };
  auto gstore = [&](int reg, uint32_t x) {
    const uint32_t off = ((s << SSH) + (x << XSH)) * 32u;
    rg_u32x4 v0, v1;
    v0.x = e[reg][0]; v0.y = e[reg][1]; v0.z = e[reg][2]; v0.w = e[reg][3];
    v1.x = e[reg][4]; v1.y = e[reg][5]; v1.z = e[reg][6]; v1.w = e[reg][7];
    if constexpr (PROBE != 0) {  // canonical values never have a top word of ~0
      if (v1.w != ~0u) return;
    }
    __builtin_amdgcn_raw_buffer_store_b128(v0, rout, off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(v1, rout, off + 16u, 0, 0);
  };
  auto xH = [&](int y) { return t + (1u << (LOGC - 3)) * y; };
  auto xM = [&](int y) -> uint32_t {
    if (LOGC == 8) return ((t >> 2) << 5) | ((uint32_t)y << 2) | (t & 3u);
    return ((uint32_t)(y >> 2) << 6) | ((t >> 2) << 4) | ((uint32_t)(y & 3) << 2) | (t & 3u);
  };
  auto xL = [&](int r) { return 8u * t + r; };
  enum { HM, ML, LH };
  auto lpos = [&](uint32_t x, int ph) -> uint32_t {
    if (COL) return s * PITCH + x + (x >> 3);
    return s * PITCH + x + (ph == HM ? 4 * (x >> 5) : ph == ML ? (x >> 3) : (x >> 5));
  };
  // limbs [l0, l0 + NPL) of register `reg` to / from LDS planes 0..NPL-1
  auto put = [&](int reg, uint32_t x, int ph, int l0) {
    const uint32_t p = lpos(x, ph);
#pragma unroll
    for (int l = 0; l < NPL; ++l) lds[l * PLANE + p] = pk(e[reg][2 * (l0 + l)], e[reg][2 * (l0 + l) + 1]);
  };
  auto get = [&](int reg, uint32_t x, int ph, int l0) {
    const uint32_t p = lpos(x, ph);
#pragma unroll
    for (int l = 0; l < NPL; ++l) {
      const uint64_t v = lds[l * PLANE + p];
      e[reg][2 * (l0 + l)] = lo32(v);
      e[reg][2 * (l0 + l) + 1] = hi32(v);
    }
  };
  // registers written at positions px(i) (phase pp) are read back at positions gx(i) (phase gp);
  // pre: the LDS image may still be read by an earlier exchange (barrier first)
  auto xchg = [&](auto px, int pp, auto gx, int gp, bool pre) {
#pragma unroll
    for (int l0 = 0; l0 < 4; l0 += NPL) {
      if (pre || l0 > 0) __syncthreads();
#pragma unroll
      for (int i = 0; i < 8; ++i) put(i, px(i), pp, l0);
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 8; ++i) get(i, gx(i), gp, l0);
    }
  };
  const bool rowuni = RP;
  if constexpr (!INV) {
#pragma unroll
    for (int y = 0; y < 8; ++y) gload(y, xH(y));
    ntt256_round<3, LOGC - 3, 0, false, false, COL, LOGN, LOGC>(a, twr, e, hi, t, rowuni);
    xchg(xH, HM, xM, HM, false);
    ntt256_round<LOGC - 5, 2, 1, false, false, COL, LOGN, LOGC>(a, twr, e, hi, t, rowuni);
    xchg(xM, ML, xL, ML, true);
    ntt256_round<2, 0, 2, false, false, COL, LOGN, LOGC>(a, twr, e, hi, t, rowuni);
    if (CANON) {
#pragma unroll
      for (int r = 0; r < 8; ++r) canon256(e[r], a.q);
    }
    if constexpr (COL) {
#pragma unroll
      for (int r = 0; r < 8; ++r) gstore(r, xL(r));
    } else {  // L -> H for coalesced rows
      xchg(xL, LH, xH, LH, true);
#pragma unroll
      for (int y = 0; y < 8; ++y) gstore(y, xH(y));
    }
  } else {
    if constexpr (COL) {
#pragma unroll
      for (int r = 0; r < 8; ++r) gload(r, xL(r));
    } else {  // rows arrive coalesced in H, transpose to L
#pragma unroll
      for (int y = 0; y < 8; ++y) gload(y, xH(y));
      xchg(xH, LH, xL, LH, false);
    }
    ntt256_round<2, 0, 2, true, SCALE, COL, LOGN, LOGC>(a, twr, e, hi, t, rowuni);
    xchg(xL, ML, xM, ML, !COL);
    ntt256_round<LOGC - 5, 2, 1, true, SCALE, COL, LOGN, LOGC>(a, twr, e, hi, t, rowuni);
    xchg(xM, HM, xH, HM, true);
    ntt256_round<3, LOGC - 3, 0, true, SCALE, COL, LOGN, LOGC>(a, twr, e, hi, t, rowuni);
    if (CANON) {
#pragma unroll
      for (int y = 0; y < 8; ++y) canon256(e[y], a.q);
    }
#pragma unroll
    for (int y = 0; y < 8; ++y) gstore(y, xH(y));
  }
}

#endif  // __HIPCC__

}  // namespace rg
