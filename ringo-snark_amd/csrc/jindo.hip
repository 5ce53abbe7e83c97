// jindo.hip -- the Jindo commitment (jindo/prover.go:45-202) and the device work of
// Prover.Evaluate (prover.go:205-324) on gfx950, batched over independent commits, with the
// prover's randomness and the Fiat-Shamir challenges injected (include/ringo.h).
//
// Commit pipeline per batch of B commits (all device-resident, one stream):
//   1. digits_kernel   thread per (commit, column, row, slot): source element (v, firstRow =
//                      v - lastRow shifted, lastRow, mask; prover.go:65-128) -> fromMont ->
//                      base-b digits (encoder.go:120-146, utils.go:12-19), two per long
//                      division by b^2, into the encode's coefficient slots j*slots+i.
//   2. prep256_kernel  wave per ring polynomial (d = 256; prep_kernel, a workgroup per
//                      polynomial, covers other d): the randEncode tail (encoder.go:166-200:
//                      MForm(noise), X^slots negacyclic shift, - b*s, + MForm(digits)) or the
//                      MLWE finalize (prover.go:130-141), then the 256-point negacyclic NTT per
//                      RNS limb in registers (Lattigo ordering/roots).
//   3. the inner Ajtai product, a per-(limb, coeff) modular GEMM
//                      sum_k In[j][k]*Enc[k] + sum_k CK.MLWE[j][k]*MLWE[k] + MLWE[mlwe+j]
//                      (prover.go:149-157): exact sums reduced once (MulCoeffsMontgomeryThenAdd
//                      summed == (sum a*b) * 2^-64 mod q).  mac_mfma_kernel (mac_mfma.hip, the
//                      matrix cores) where its digit bound holds (every configs shape); else
//                      mac_kernel (exact 128/160-bit sums, any prime and J).  Round 2-5's VALU
//                      Karatsuba MAC (mac3h) is tools/experiments/jindo_knob_kernels.patch.
//   4. round_kernel    workgroup per polynomial: IMForm, INTT, centred CRT (Garner, up to 4
//                      primes), floor shift by the cut, Euclidean mod q', MForm, NTT in the
//                      destination ring (prover.go:164-176, rns.go:76-114).
//   5. the MAC + round_kernel again for the outer commitment (prover.go:180-202).
// Evaluate: every MulCoeffsMontgomeryThenAdd loop is a J = 1 dot product on mac_kernel
// (rg_jindo_eval_*), plus rns_reduce_kernel after a cross-GPU sum of partial openBatches.
// All residues are canonical, so results are bit-exact against the reference's Lattigo
// calls given the same primes (Lattigo conventions restated: see DESIGN.md, "parity").
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "ck_crs.hpp"
#include "common.hpp"
#include "csprng.hpp"
#include "digits_dc.hpp"
#include "csprng_host.hpp"
#include "field.hpp"
#include "host_field.hpp"
#include "mac_mfma.hpp"
#include "ntt64.hpp"

namespace rg {

constexpr int kMaxQ = 4;     // RNS limbs per ring
constexpr int kMaxD = 1024;  // ring degree supported by the LDS kernels
constexpr int kMaxJ = 32;    // MSIS rank accumulated per thread

struct RnsPrime {
  uint64_t q;
  uint64_t rinv, rinv_sh;    // 2^-64 mod q (IMForm)
  uint64_t r64, r64_sh;      // 2^64 mod q (MForm)
  uint64_t one_sh;           // floor(2^64 / q): x mod q = shoup(x, 1)
  uint64_t ninv, ninv_sh;    // d^-1 mod q
  uint64_t bmod, bmod_sh;    // base mod q
  uint64_t rw1, rw1_sh;      // 2^64 w1 mod q, w1 = the forward table's first-stage root (prep256 stage 0)
};

struct RingDev {
  int n;                    // limbs
  RnsPrime p[kMaxQ];
  const ulonglong2* fwd;    // [n][d] (w, w') psi^brv
  const ulonglong2* bwd;    // [n][d] psi^-brv
};

// CRT (Garner) constants for a source ring
struct CrtDev {
  int n;
  uint64_t q[kMaxQ];
  uint64_t inv[kMaxQ][kMaxQ], inv_sh[kMaxQ][kMaxQ];  // inv[j][k] = q_k^-1 mod q_j (k < j)
  uint64_t Q[4], Qhalf[4];                            // product (4 words) and floor(Q/2)
};

// destination mod constants: 2^(64k) mod q' for multiword reduction
struct DstDev {
  int n;
  uint64_t pw[kMaxQ][4], pw_sh[kMaxQ][4];
};

// ------------------------------------------------------------------------------------------
// device helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t sh_mul(uint64_t y, uint64_t w, uint64_t wp, uint64_t q) {
  return shoup_mul(y, w, wp, q);
}
__device__ __forceinline__ uint64_t signed_residue(long long c, uint64_t q) {
  // setCoeffSigned (utils.go:49-61): c >= 0 -> c ; else Go's c%q + q (== q when q | c; the
  // following MForm maps that to 0 either way)
  if (c >= 0) return (uint64_t)c < q ? (uint64_t)c : (uint64_t)c % q;
  const uint64_t a = (uint64_t)(-(c + 1)) + 1;
  return a < q ? q - a : q - a % q;
}

// d-point negacyclic NTT (Lattigo ordering: natural -> bit-reversed) of one limb held in LDS,
// by `nt` threads (thread index `ti`); synchronises the whole workgroup between stages.
__device__ void ntt_lds(uint64_t* p, int d, const ulonglong2* roots, uint64_t q, int ti, int nt, bool active) {
  int lt = 0;
  while ((2 << lt) < d) ++lt;  // log2(d/2)
  for (int m = 1, t = d >> 1; m < d; m <<= 1, t >>= 1, --lt) {
    if (active) {
      for (int k = ti; k < (d >> 1); k += nt) {
        const int i = k >> lt, j = (i << (lt + 1)) + (k & (t - 1));
        const ulonglong2 w = roots[m + i];
        const uint64_t u = p[j], v = sh_mul(p[j + t], w.x, w.y, q);
        p[j] = mod_add(u, v, q);
        p[j + t] = mod_sub(u, v, q);
      }
    }
    __syncthreads();
  }
}
// inverse (GS, bit-reversed -> natural), times d^-1
__device__ void intt_lds(uint64_t* p, int d, const ulonglong2* roots, const RnsPrime& P, int ti, int nt, bool active) {
  const uint64_t q = P.q;
  for (int m = d >> 1, t = 1, lt = 0; m >= 1; m >>= 1, t <<= 1, ++lt) {
    if (active) {
      for (int k = ti; k < (d >> 1); k += nt) {
        const int i = k >> lt, j = (i << (lt + 1)) + (k & (t - 1));
        const ulonglong2 w = roots[m + i];
        const uint64_t u = p[j], v = p[j + t];
        p[j] = mod_add(u, v, q);
        p[j + t] = sh_mul(mod_sub(u, v, q), w.x, w.y, q);
      }
    }
    __syncthreads();
  }
  if (active)
    for (int k = ti; k < d; k += nt) p[k] = sh_mul(p[k], P.ninv, P.ninv_sh, q);
  __syncthreads();
}

// ------------------------------------------------------------------------------------------
// 1. digits
// ------------------------------------------------------------------------------------------
struct JShape {
  int rank, rows, cols, slots, exp, d, in_msis, out_msis, mlwe, dcmp, log_in_cut, log_out_cut;
  int nq, nqo;
  uint64_t base;
  long long nv;
};

template <int L>
struct DigitArgs {
  JShape s;
  FieldParams<L> F;
  uint64_t base_inv;  // floor(2^64 / base)
  uint64_t b2, b2_inv;  // base^2 and floor(2^64 / base^2) when base^2 < 2^32, else 0
  DigitDc dc;           // divide-and-conquer constants (digits_dc.hpp); dc.exp = 0: the loop below
  const uint64_t* v;         // [B][nv][L]
  const uint64_t* last_row;  // [B][cols*slots][L]
  const uint64_t* mask;      // [B][rows][slots][L]
  uint32_t* digits;          // [B][cols+1][rows][d]
  long long total;           // B * (cols+1) * rows * slots
  IdxDiv d_slots, d_rows, d_cols1;  // total < 2^32: the index split by idx_div (else 64-bit division)
};

// (num = r * 2^32 + chunk) / b with the precomputed reciprocal, r < b < 2^32
__device__ __forceinline__ uint32_t divstep(uint64_t num, uint64_t b, uint64_t binv, uint64_t& r) {
  uint64_t qt = mul_hi(num, binv);
  uint64_t rem = num - qt * b;
  if (rem >= b) {
    rem -= b;
    ++qt;
  }
  r = rem;
  return (uint32_t)qt;
}

// the same step for a divisor d in (2^31, 2^32) (b^2 of every configs field: 60272^2, 60256^2),
// whose reciprocal is 2^32 + B0: hi64(num (2^32 + B0)) = r + hi32(r B0 + n0 + hi32(n0 B0)) for
// num = r 2^32 + n0 -- three 32-bit multiplies instead of a 64 x 64 high product and a 64-bit
// product
__device__ __forceinline__ uint32_t divstep_b2(uint32_t r, uint32_t n0, uint32_t d, uint32_t B0, uint32_t& rem) {
  const uint64_t t = mad64(r, B0, (uint64_t)n0 + __umulhi(n0, B0));
  uint32_t qt = r + (uint32_t)(t >> 32);
  uint64_t rm = (((uint64_t)r << 32) | n0) - (uint64_t)qt * d;
  if (rm >= d) {
    rm -= d;
    ++qt;
  }
  rem = (uint32_t)rm;
  return qt;
}

// x R^-1 mod q (Slice = fromMont, element.go): Montgomery reduction alone, L^2 word products
// instead of the 2 L^2 of f_mul(x, 1).  For any x < R, (x + m q) / R < q + 1, so one conditional
// subtraction of q leaves the canonical residue (a non-canonical word such as x = q gives 0, as
// f_mul(x, 1) did).
template <int L>
__device__ __forceinline__ void f_redc(uint64_t* z, const uint64_t* x, const FieldParams<L>& F) {
  uint64_t t[L];
#pragma unroll
  for (int i = 0; i < L; ++i) t[i] = x[i];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const uint64_t m = t[0] * F.qinv;
    uint64_t lo, hi;
    mul_wide(m, F.q[0], lo, hi);
    uint32_t c0 = 0;
    addc(lo, t[0], c0);  // == 0 mod 2^64; only the carry is kept
    uint64_t carry = hi + c0;
#pragma unroll
    for (int j = 1; j < L; ++j) {
      mul_wide(m, F.q[j], lo, hi);
      uint32_t c = 0;
      lo = addc(lo, t[j], c);
      hi += c;
      c = 0;
      lo = addc(lo, carry, c);
      t[j - 1] = lo;
      carry = hi + c;
    }
    t[L - 1] = carry;
  }
  uint64_t d[L];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) d[i] = subb(t[i], F.q[i], br);
#pragma unroll
  for (int i = 0; i < L; ++i) z[i] = br ? t[i] : d[i];
}

template <int L>
__global__ __launch_bounds__(256) void digits_kernel(DigitArgs<L> a) {
  const JShape& S = a.s;
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= a.total) return;
  int slot, row, col;
  long long b;
  if (a.total <= 0xffffffffLL) {  // (slot, row, col, b) without 64-bit divisions
    const uint32_t g = (uint32_t)gid, q1 = idx_div(g, a.d_slots), q2 = idx_div(q1, a.d_rows),
                   q3 = idx_div(q2, a.d_cols1);
    slot = (int)(g - q1 * a.d_slots.d);
    row = (int)(q1 - q2 * a.d_rows.d);
    col = (int)(q2 - q3 * a.d_cols1.d);
    b = q3;
  } else {
    slot = (int)(gid % S.slots);
    long long r = gid / S.slots;
    row = (int)(r % S.rows);
    r /= S.rows;
    col = (int)(r % (S.cols + 1));
    b = r / (S.cols + 1);
  }
  const long long cs = (long long)S.cols * S.slots;
  const uint64_t* vb = a.v + b * S.nv * L;
  uint32_t* out = a.digits + (((b * (S.cols + 1) + col) * S.rows + row) * (long long)S.d);

  // which element feeds this slot (prover.go:89-128); `have` = false -> zero slot
  uint64_t x[L];
  bool have = true;
  if (col == S.cols) {  // mask column: every slot present
    const uint64_t* m = a.mask + ((b * S.rows + row) * S.slots + slot) * L;
#pragma unroll
    for (int l = 0; l < L; ++l) x[l] = m[l];
  } else if (row == S.rows - 1) {  // last row
    const uint64_t* m = a.last_row + (b * cs + (long long)col * S.slots + slot) * L;
#pragma unroll
    for (int l = 0; l < L; ++l) x[l] = m[l];
  } else if (row == 0) {  // first row: v[i] - lastRow[i-1] (genFirstLastRow :74-83)
    const long long i = (long long)col * S.slots + slot;
    uint64_t vi[L], lr[L];
#pragma unroll
    for (int l = 0; l < L; ++l) vi[l] = (i < S.nv) ? vb[i * L + l] : 0;
    if (i == 0) {
#pragma unroll
      for (int l = 0; l < L; ++l) x[l] = vi[l];
    } else {
      const uint64_t* m = a.last_row + (b * cs + i - 1) * L;
#pragma unroll
      for (int l = 0; l < L; ++l) lr[l] = m[l];
      f_sub<L>(x, vi, lr, a.F);
    }
  } else {  // data row: v[row*cs + col*slots + slot] when < nv
    const long long i = row * cs + (long long)col * S.slots + slot;
    have = i < S.nv;
#pragma unroll
    for (int l = 0; l < L; ++l) x[l] = have ? vb[i * L + l] : 0;
  }
  // canonical limbs (Slice = fromMont)
  uint64_t c[L];
  f_redc<L>(c, x, a.F);
  if (!have) {
#pragma unroll
    for (int l = 0; l < L; ++l) c[l] = 0;
  }
  // base-b digits: exp-1 remainders then the final quotient (encoder.go:125-136)
  if constexpr (L == 4 || L == 2) {
    if (a.dc.exp == S.exp) {  // every configs field: by divide and conquer (digits_dc.hpp)
      dc_digits<L>(c, a.dc, [&](int j, uint32_t dg) { out[j * S.slots + slot] = dg; });
      return;
    }
  }
  uint32_t w[2 * L];
#pragma unroll
  for (int l = 0; l < L; ++l) {
    w[2 * l] = (uint32_t)c[l];
    w[2 * l + 1] = (uint32_t)(c[l] >> 32);
  }
  int jd = 0;
  if (a.b2) {  // two digits per long division: divide by b^2 (< 2^32), split the remainder
    // words above `top` are zero (the value shrinks ~2 log2(b) bits a pass); the word loop stays
    // unrolled with a predicate so w[] is never indexed dynamically (registers, not scratch)
    auto top_of = [&]() {
      int tp = 0;
#pragma unroll
      for (int k = 1; k < 2 * L; ++k) tp = w[k] ? k : tp;
      return tp;
    };
    int top = top_of();
    const bool b2fast = (a.b2_inv >> 32) == 1;  // uniform: d in (2^31, 2^32)
    for (; jd + 1 < S.exp - 1; jd += 2) {
      uint64_t rem = 0;
      if (b2fast) {
        uint32_t r32 = 0;
#pragma unroll
        for (int k = 2 * L - 1; k >= 0; --k)
          if (k <= top) w[k] = divstep_b2(r32, w[k], (uint32_t)a.b2, (uint32_t)a.b2_inv, r32);
        rem = r32;
      } else {
#pragma unroll
        for (int k = 2 * L - 1; k >= 0; --k)
          if (k <= top) w[k] = divstep((rem << 32) | w[k], a.b2, a.b2_inv, rem);
      }
      top = top_of();
      uint64_t lo;
      const uint32_t hi = divstep(rem, S.base, a.base_inv, lo);
      out[jd * S.slots + slot] = (uint32_t)lo;
      out[(jd + 1) * S.slots + slot] = hi;
    }
  }
  for (; jd < S.exp - 1; ++jd) {
    uint64_t rem = 0;
#pragma unroll
    for (int k = 2 * L - 1; k >= 0; --k) w[k] = divstep((rem << 32) | w[k], S.base, a.base_inv, rem);
    out[jd * S.slots + slot] = (uint32_t)rem;
  }
  out[(S.exp - 1) * S.slots + slot] = w[0];
}

// zero-fill digit slots not covered (d > exp*slots never happens for jindo; kept for safety)

// ------------------------------------------------------------------------------------------
// 2. prep: encode tail / MLWE finalize + NTT
// ------------------------------------------------------------------------------------------
struct PrepArgs {
  JShape s;
  RingDev R;
  const uint32_t* digits;     // [B][cols+1][rows][d]
  const long long* enc_noise;  // [B][cols+1][rows][d]
  const long long* mlwe_noise; // [B][cols+1][nm][d]
  uint64_t* enc;               // [B][cols+1][rows][nq][d]
  uint64_t* mlwe;              // [B][cols+1][nm][nq][d]
  long long n_enc;             // B * (cols+1) * rows
  long long n_ml;              // B * (cols+1) * (inMSIS + mlwe)
  long long clim;              // |noise| bound for the one-integer encode form: 2^61 / base
};

// Encodes the reference does not perform (prover.go:101-105, 118-123): data rows j in
// [1, rows-2] of column i whose first index j*cols*slots (+ i*slots) is past len(v); their
// Opening.Encode stays zero.  The start index grows with j, so the reference's `break`
// is the same as testing each row.
__device__ __forceinline__ bool enc_skipped(const JShape& S, int col, int row) {
  if (row < 1 || row > S.rows - 2) return false;
  const long long cs = (long long)S.cols * S.slots;
  const long long start = row * cs + (col == S.cols ? 0 : (long long)col * S.slots);
  return start > S.nv;
}

__global__ __launch_bounds__(256) void prep_kernel(PrepArgs a) {
  __shared__ uint64_t poly[kMaxQ][kMaxD];
  const JShape& S = a.s;
  const int d = S.d, nq = S.nq, tid = threadIdx.x;
  const int nm = S.in_msis + S.mlwe;
  const long long job = blockIdx.x;
  const bool is_enc = job < a.n_enc;
  uint64_t* dst;
  if (is_enc) {
    const long long pj = job;
    const int cr = (int)(pj % ((long long)(S.cols + 1) * S.rows));
    dst = a.enc + pj * nq * d;
    if (enc_skipped(S, cr / S.rows, cr % S.rows)) {  // Opening.Encode[i][j] stays zero
      for (int k = tid; k < nq * d; k += blockDim.x) dst[k] = 0;
      return;
    }
    const uint32_t* dg = a.digits + pj * d;
    const long long* nz = a.enc_noise + pj * d;
    for (int k = tid; k < d; k += blockDim.x) {
      const long long c = nz[k];
      // the X^slots shift: coefficient k receives s[k - slots] (k >= slots) or -s[k + d - slots]
      const int ks = k - S.slots;
      const long long cs = ks >= 0 ? nz[ks] : nz[ks + d];
      const uint64_t dgk = dg[k];
      for (int l = 0; l < nq; ++l) {
        const RnsPrime& P = a.R.p[l];
        const uint64_t q = P.q;
        const uint64_t sm = sh_mul(signed_residue(c, q), P.r64, P.r64_sh, q);    // MForm(s) :184
        uint64_t sh = sh_mul(signed_residue(cs, q), P.r64, P.r64_sh, q);
        if (ks < 0) sh = mod_neg(sh, q);  // wrapped coefficients negate (:191-195)
        sh = mod_sub(sh, sh_mul(sm, P.bmod, P.bmod_sh, q), q);                   // :196
        const uint64_t dm = sh_mul(dgk, P.r64, P.r64_sh, q);  // MForm(digits) :198 (digit <= b < q)
        poly[l][k] = mod_add(dm, sh, q);                                          // :199
      }
    }
  } else {
    const long long mj = job - a.n_enc;  // (b, col, j) flattened
    dst = a.mlwe + mj * nq * d;
    const long long* nz = a.mlwe_noise + mj * d;
    for (int k = tid; k < d; k += blockDim.x) {
      const long long c = nz[k];
      for (int l = 0; l < nq; ++l) {
        const RnsPrime& P = a.R.p[l];
        poly[l][k] = sh_mul(signed_residue(c, P.q), P.r64, P.r64_sh, P.q);  // MForm (prover.go:140)
      }
    }
    (void)nm;
  }
  __syncthreads();
  // NTT per limb: two limbs at a time on the two halves of the workgroup
  const int half = blockDim.x >> 1;
  for (int l0 = 0; l0 < nq; l0 += 2) {
    const int l = l0 + (tid >= half ? 1 : 0);
    const bool active = l < nq;
    const int lc = active ? l : l0;
    ntt_lds(poly[lc], d, a.R.fwd + (long long)lc * d, a.R.p[lc].q, tid % half, half, active);
  }
  for (int k = tid; k < nq * d; k += blockDim.x) dst[k] = poly[k / d][k % d];
}

// Wave-per-polynomial prep for d = 256 (every Jindo parameter set): one wave owns one job and two
// RNS limbs at a time (lanes 0-31 limb l0, 32-63 limb l0+1), 8 coefficients per lane; the
// 256-point negacyclic NTT runs as rounds of 3 + 3 + 2 radix-2 stages in registers with
// wave-local LDS exchanges (no workgroup barrier; ntt64.hpp's ROW index algebra with hi = 0),
// lazy [0, 2q) Shoup arithmetic, canonical output.  Same results as prep_kernel.
constexpr int kPrepWaves = 4;
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}
template <int RK, int LO, int PAT, int SP0 = 0, bool LAZY = false>
__device__ __forceinline__ void prep_round(uint64_t (&e)[8], const ulonglong2* roots, uint64_t q, uint64_t q2,
                                           uint32_t t) {
  auto xof = [&](int rho) -> uint32_t {
    if (PAT == 0) return t + 32u * rho;
    if (PAT == 1) return ((t >> 2) << 5) | ((uint32_t)rho << 2) | (t & 3u);
    return 8u * t + rho;
  };
  constexpr int NPK = 1 << RK;
#pragma unroll
  for (int sp = SP0; sp < RK; ++sp) {
    const int bw = RK - 1 - sp, b = LO + bw, k = 7 - b, half = 1 << bw;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int grp = j / (NPK / 2), jj = j % (NPK / 2);
      const int rho0 = grp * NPK + ((jj >> bw) << (bw + 1)) + (jj & (half - 1));
      const ulonglong2 w = roots[(1u << k) + (xof(rho0) >> (b + 1))];  // the limb's table, staged in LDS
      // Harvey with a 4q-wide twiddle product: values in [0, 8q) (ring primes < 2^61), x
      // reduced to [0, 4q), t = y w - Q' q in [0, 4q) with Q' the Shoup quotient less the low
      // cross products (Q - 2 <= Q' <= Q): three 32-bit multiplies for the quotient, not four
      // x >= 4q ? x - 4q : x, on the borrow (q2 = 4q here); LAZY (36 q < 2^64): x unreduced, each
      // stage widens the bound by 4q, [0, 8q) after stage 0 -> [0, 36q) after stage 7
      const uint64_t x = LAZY ? e[rho0] : canon_x(e[rho0], q2);
      const uint64_t y = e[rho0 + half];
      const uint32_t y0 = (uint32_t)y, y1 = (uint32_t)(y >> 32), p0 = (uint32_t)w.y, p1 = (uint32_t)(w.y >> 32);
      const uint64_t qa = mad64(y1, p1, __umulhi(y1, p0)) + __umulhi(y0, p1);
      const uint64_t tt = y * w.x - qa * q;
      e[rho0] = x + tt;
      e[rho0 + half] = x + q2 - tt;
    }
  }
}

// y w mod q in [0, 3q) for any 64-bit y: prep_round's Shoup product with the 3-multiply quotient
__device__ __forceinline__ uint64_t shoup3(uint64_t y, uint64_t w, uint64_t wp, uint64_t q) {
  const uint32_t y0 = (uint32_t)y, y1 = (uint32_t)(y >> 32), p0 = (uint32_t)wp, p1 = (uint32_t)(wp >> 32);
  const uint64_t qa = mad64(y1, p1, __umulhi(y1, p0)) + __umulhi(y0, p1);
  return y * w - qa * q;
}

// signed integer -> residue in [0, q) without division (Shoup by 1 reduces any 64-bit value)
__device__ __forceinline__ uint64_t red_signed(long long c, const RnsPrime& P) {
  const uint64_t ac = c < 0 ? (uint64_t)(-(c + 1)) + 1 : (uint64_t)c;
  const uint64_t m = sh_mul(ac, 1, P.one_sh, P.q);
  return c < 0 ? mod_neg(m, P.q) : m;
}

template <int MINW, bool PAIR1, int WAVES = kPrepWaves, bool LAZY = false>
__global__ __launch_bounds__(64 * WAVES, MINW) void prep256_kernel(PrepArgs a) {
  __shared__ uint64_t lds_all[WAVES][2 * 288];
  extern __shared__ ulonglong2 tw_lds[];  // the nq limbs' forward tables (w, w'), [nq][256]: dynamic LDS
  const JShape& S = a.s;
  const int nq = S.nq;
  const uint32_t lane = threadIdx.x & 63u, t = lane & 31u, hs = lane >> 5;
  const int wv = threadIdx.x >> 6;
  uint64_t* lds = lds_all[wv];
  const long long job = (long long)blockIdx.x * WAVES + wv;
  const bool has = job < a.n_enc + a.n_ml;
  const bool is_enc = job < a.n_enc;
  uint64_t* dst = nullptr;
  const uint32_t* dg = nullptr;
  const long long* nz = nullptr;
  bool skip = false;
  if (has && is_enc) {
    const long long pj = job;
    const int cr = (int)(pj % ((long long)(S.cols + 1) * S.rows));
    dst = a.enc + pj * nq * 256;
    skip = enc_skipped(S, cr / S.rows, cr % S.rows);  // Opening.Encode[i][j] stays zero
    dg = a.digits + pj * 256;
    nz = a.enc_noise + pj * 256;
  } else if (has) {
    const long long mj = job - a.n_enc;
    dst = a.mlwe + mj * nq * 256;
    nz = a.mlwe_noise + mj * 256;
  }
  // the job's inputs (noise, shifted noise, digits).  PAIR1 (nq <= 2, every configs ring): loaded
  // ahead of the table staging so the two loads' latencies overlap (configs[2] +1.4%); otherwise
  // read per limb pair after it, rather than held across the NTT
  long long cv[8], csv[8];
  uint32_t dv[8];
  auto load_in = [&]() {
#pragma unroll
    for (int y = 0; y < 8; ++y) {
      const int k = (int)t + 32 * y;
      cv[y] = nz[k];
      if (is_enc) {
        const int ks = k - S.slots;
        csv[y] = ks >= 0 ? nz[ks] : nz[ks + 256];
        dv[y] = dg[k];
      } else {
        csv[y] = 0;
        dv[y] = 0;
      }
    }
  };
  if (PAIR1 && has && !skip) load_in();
  // slot 0 of each limb's table (unused by the transform) holds (2^64 w1, Shoup) for stage 0
  for (int i = threadIdx.x; i < nq * 256; i += blockDim.x)
    tw_lds[i] = (i & 255) ? a.R.fwd[i] : make_ulonglong2(a.R.p[i >> 8].rw1, a.R.p[i >> 8].rw1_sh);
  __syncthreads();
  if (!has) return;
  if (skip) {
    for (int k = (int)lane; k < nq * 256; k += 64) dst[k] = 0;
    return;
  }
  const uint32_t rH = 288 * hs + t, rM = 288 * hs + 36 * (t >> 2) + (t & 3), rL9 = 288 * hs + 9 * t,
                 rL8 = 288 * hs + 8 * t + (t >> 2);
  auto pair = [&](const int l0) {
    const int limb = l0 + (int)hs;
    const bool active = limb < nq;
    const int lc = active ? limb : l0;
    const RnsPrime& P = a.R.p[lc];
    const uint64_t q = P.q, q2 = 4 * q;  // prep_round's lazy bound: values in [0, 2 q2)
    const ulonglong2* roots = tw_lds + lc * 256;
    // The encode tail MForm(dg) + MForm(+-s') - MForm(s) b (encoder.go:184-199) is MForm of ONE
    // signed integer v = dg +- s' - s b when that fits (|s| <= 2^61 / b, |s'| < 2^61); the MLWE
    // finalize is MForm(setCoeffSigned(s)) (prover.go:130-141): v = s.  MForm is a factor 2^64 on
    // every coefficient, so it rides on NTT stage 0: e holds v mod q (one add when |v| < q), and
    // stage 0 multiplies by 2^64 and 2^64 w1 instead of w1.
    uint64_t e[8];
    uint32_t big = 0;  // bit y: coefficient t + 32 y takes the term-by-term reduction
#pragma unroll
    for (int y = 0; y < 8; ++y) {
      const int k = (int)t + 32 * y;
      const long long c = cv[y];
      long long v = c;
      bool ok = true;
      if (is_enc) {
        const long long cs = csv[y];
        const uint64_t s2 = k < S.slots ? 0ull - (uint64_t)cs : (uint64_t)cs;  // wrapped coefficients negate
        ok = c >= -a.clim && c <= a.clim && cs > -(1LL << 61) && cs < (1LL << 61);
        v = (long long)((uint64_t)dv[y] + s2 - (uint64_t)c * S.base);
      }
      const uint64_t r = v < 0 ? (uint64_t)v + q : (uint64_t)v;  // v mod q when -q <= v < q
      ok = ok && r < q;
      big |= ok ? 0u : (1u << y);
      e[y] = r;
    }
    if (big) {  // rare (huge injected noise): every term reduced separately, same residue
      for (int y = 0; y < 8; ++y) {
        if (!((big >> y) & 1u)) continue;
        const int k = (int)t + 32 * y;
        if (is_enc) {
          const int ks = k - S.slots;
          const uint64_t cm = red_signed(nz[k], P);
          uint64_t s2 = red_signed(ks >= 0 ? nz[ks] : nz[ks + 256], P);
          if (k < S.slots) s2 = mod_neg(s2, q);
          const uint64_t val = mod_add(sh_mul(dg[k], 1, P.one_sh, q), s2, q);
          e[y] = mod_sub(val, sh_mul(cm, P.bmod, P.bmod_sh, q), q);
        } else {
          e[y] = red_signed(nz[k], P);
        }
      }
    }
    {  // stage 0 (pairs y, y + 4 of the H pattern, root w1) times 2^64: inputs in [0, q), outputs
       // in [0, 8q) like every later stage's
      const ulonglong2 rw = roots[0];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint64_t xr = shoup3(e[j], P.r64, P.r64_sh, q), yr = shoup3(e[j + 4], rw.x, rw.y, q);
        e[j] = xr + yr;
        e[j + 4] = xr + q2 - yr;
      }
    }
    // NTT: H round (stages 1-2; 0 above), H->M, M round (3-5), M->L, L round (6-7), L->H, store
    prep_round<3, 5, 0, 1, LAZY>(e, roots, q, q2, t);
#pragma unroll
    for (int y = 0; y < 8; ++y) lds[rH + 36 * y] = e[y];
    wave_lds_fence();
#pragma unroll
    for (int y = 0; y < 8; ++y) e[y] = lds[rM + 4 * y];
    prep_round<3, 2, 1, 0, LAZY>(e, roots, q, q2, t);
    wave_lds_fence();
#pragma unroll
    for (int y = 0; y < 8; ++y) lds[rM + 4 * y + (y >> 1)] = e[y];
    wave_lds_fence();
#pragma unroll
    for (int r = 0; r < 8; ++r) e[r] = lds[rL9 + r];
    prep_round<2, 0, 2, 0, LAZY>(e, roots, q, q2, t);
    wave_lds_fence();
#pragma unroll
    for (int r = 0; r < 8; ++r)  // [0, 8q) (LAZY: [0, 36q), Shoup by 1) -> [0, q)
      lds[rL8 + r] = LAZY ? shoup_mul(e[r], 1, P.one_sh, q) : canon_x(canon_x(canon_x(e[r], q2), 2 * q), q);
    wave_lds_fence();
    if (active) {
      uint64_t* o = dst + (long long)limb * 256;
#pragma unroll
      for (int y = 0; y < 8; ++y) o[t + 32 * y] = lds[rH + 33 * y];
    }
    wave_lds_fence();
  };
  if constexpr (PAIR1) {
    pair(0);
  } else {
    for (int l0 = 0; l0 < nq; l0 += 2) {
      load_in();
      pair(l0);
    }
  }
}

// ------------------------------------------------------------------------------------------
// 3. multiply-accumulate (inner / outer Ajtai products)
// ------------------------------------------------------------------------------------------
struct MacArgs {
  int d, nl, J;            // degree, limbs, outputs per column
  long long ncols;         // B * columns
  int T1, T2;              // terms from operand set 1 / 2
  const uint64_t* A1;      // [J][T1][nl][d]   commit key
  const uint64_t* B1;      // [ncols][T1][nl][d] (stride b1_col per column, b1_term per term)
  long long b1_col, b1_term;
  const uint64_t* A2;      // [J][T2][nl][d]
  const uint64_t* B2;
  long long b2_col, b2_term;
  const uint64_t* C;       // added after reduction: [ncols][...] + j * c_j  (nullable)
  long long c_col, c_j;
  uint64_t* out;           // [ncols][J][nl][d]
  RnsPrime P[kMaxQ];
};

// acc += a * b as an exact multiword sum; WIDE keeps a third word (needed only when
// (q-1)^2 * terms could reach 2^128: decided per launch on the host).
template <bool WIDE>
struct Acc {
  uint64_t lo, hi;
  uint32_t top;
  __device__ __forceinline__ void zero() {
    lo = hi = 0;
    top = 0;
  }
  __device__ __forceinline__ void mac(uint64_t a, uint64_t b) {
    uint64_t pl, ph;
    mul_wide(a, b, pl, ph);
    uint32_t c = 0;
    lo = addc(lo, pl, c);
    if constexpr (WIDE) {
      uint32_t c2 = 0;
      hi = addc(hi, ph, c2);
      uint32_t c3 = 0;
      hi = addc(hi, (uint64_t)c, c3);
      top += c2 + c3;
    } else {
      hi += ph + c;
    }
  }
  // (lo + hi 2^64 + top 2^128) * 2^-64 mod q = lo 2^-64 + hi + top 2^64
  __device__ __forceinline__ uint64_t reduce(const RnsPrime& P) const {
    const uint64_t q = P.q;
    uint64_t r = sh_mul(lo, P.rinv, P.rinv_sh, q);
    r = mod_add(r, sh_mul(hi, 1, P.one_sh, q), q);
    if constexpr (WIDE) r = mod_add(r, sh_mul((uint64_t)top, P.r64, P.r64_sh, q), q);
    return r;
  }
};

// Thread = (column group of NC columns, limb*coeff).  Per term: JB commit-key words are loaded
// once and reused for NC columns, NC data words reused for JB outputs (register tiling of the
// per-(limb, coeff) modular GEMM  out[j][col] = sum_t A[j][t] B[t][col]).
template <int JB, int NC, bool WIDE>
__global__ __launch_bounds__(256) void mac_kernel(MacArgs a, int j0) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long per_col = (long long)a.nl * a.d;
  const long long ngroups = (a.ncols + NC - 1) / NC;
  if (gid >= ngroups * per_col) return;
  const long long cg = gid / per_col;
  const int lk = (int)(gid % per_col);  // limb * d + coeff
  const int l = lk / a.d;
  const int J = min(JB, a.J - j0);
  const long long col0 = cg * NC;
  const int nc = (int)min((long long)NC, a.ncols - col0);
  Acc<WIDE> acc[NC][JB];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int j = 0; j < JB; ++j) acc[c][j].zero();
  for (int set = 0; set < 2; ++set) {
    const int T = set ? a.T2 : a.T1;
    if (!T) continue;
    const uint64_t* A = (set ? a.A2 : a.A1) + lk;
    const uint64_t* Bp = (set ? a.B2 : a.B1) + lk;
    const long long bcol = set ? a.b2_col : a.b1_col, bterm = set ? a.b2_term : a.b1_term;
    // J = 1 (Prover.Evaluate's dot products): unrolled so each thread keeps 4 terms' loads in
    // flight -- one term's 1 + NC loads per iteration left the opening stream latency-bound
    constexpr int kUnr = JB == 1 ? 4 : 1;
#pragma unroll kUnr
    for (int t = 0; t < T; ++t) {
      uint64_t av[JB], bv[NC];
#pragma unroll
      for (int j = 0; j < JB; ++j) av[j] = (j < J) ? A[((long long)(j0 + j) * T + t) * per_col] : 0;
#pragma unroll
      for (int c = 0; c < NC; ++c) bv[c] = (c < nc) ? Bp[(col0 + c) * bcol + t * bterm] : 0;
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int j = 0; j < JB; ++j) acc[c][j].mac(av[j], bv[c]);
    }
  }
  const RnsPrime& P = a.P[l];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (c >= nc) continue;
    const long long col = col0 + c;
#pragma unroll
    for (int j = 0; j < JB; ++j) {
      if (j >= J) continue;
      uint64_t r = acc[c][j].reduce(P);
      if (a.C) r = mod_add(a.C[col * a.c_col + (long long)(j0 + j) * a.c_j + lk], r, P.q);
      a.out[(col * a.J + j0 + j) * per_col + lk] = r;
    }
  }
}

constexpr int kMacNC = 4;

template <int JB, bool WIDE>
static rg_status launch_mac_jb(const MacArgs& m, int j0, hipStream_t st) {
  const long long groups = (m.ncols + kMacNC - 1) / kMacNC;
  const long long threads = groups * m.nl * m.d;
  hipLaunchKernelGGL((mac_kernel<JB, kMacNC, WIDE>), dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, m, j0);
  return check_launch("jindo mac");
}

template <bool WIDE>
static rg_status launch_mac_w(const MacArgs& m, int jb, int j0, hipStream_t st) {
  switch (jb) {
    case 1: return launch_mac_jb<1, WIDE>(m, j0, st);
    case 2: return launch_mac_jb<2, WIDE>(m, j0, st);
    case 3: return launch_mac_jb<3, WIDE>(m, j0, st);
    case 4: return launch_mac_jb<4, WIDE>(m, j0, st);
    case 5: return launch_mac_jb<5, WIDE>(m, j0, st);
    case 6: return launch_mac_jb<6, WIDE>(m, j0, st);
    case 7: return launch_mac_jb<7, WIDE>(m, j0, st);
    default: return launch_mac_jb<8, WIDE>(m, j0, st);
  }
}

// J outputs split into ceil(J/8) launches of equal width
static rg_status launch_mac(const MacArgs& m, hipStream_t st) {
  uint64_t qmax = 0;
  for (int l = 0; l < m.nl; ++l) qmax = std::max(qmax, m.P[l].q);
  const double bits = 2.0 * log2((double)(qmax - 1)) + log2((double)(m.T1 + m.T2) + 1.0);
  const bool wide = bits >= 127.5;
  const int passes = (m.J + 7) / 8;
  const int jb = (m.J + passes - 1) / passes;
  for (int j0 = 0; j0 < m.J; j0 += jb) RG_TRY(wide ? launch_mac_w<true>(m, jb, j0, st) : launch_mac_w<false>(m, jb, j0, st));
  return RG_OK;
}


// ------------------------------------------------------------------------------------------
// 4. round: IMForm -> INTT -> centred CRT -> floor shift -> mod q' -> MForm -> NTT
// ------------------------------------------------------------------------------------------
struct RoundArgs {
  int d, cut;
  RingDev src, dst;
  CrtDev crt;
  DstDev dm;
  const uint64_t* in;  // [npoly][src.n][d]
  uint64_t* out;       // [npoly] at stride out_stride, dst.n limbs (+ zero rows up to out_rows)
  long long out_stride;
  int out_rows;
  long long npoly;     // round256_kernel's polynomials (round_kernel: the grid)
};

__device__ __forceinline__ void mw_muladd(uint64_t* v, int nw, uint64_t m, uint64_t add) {
  uint64_t carry = add;
  for (int i = 0; i < nw; ++i) {
    uint64_t lo, hi;
    mul_wide(v[i], m, lo, hi);
    uint32_t c = 0;
    lo = addc(lo, carry, c);
    v[i] = lo;
    carry = hi + c;
  }
}

// reconstructTo (rns.go:76-105) of one coefficient's residues r[ns] (coefficient domain): the
// centred value as sign (returned) and 4-word magnitude
__device__ __forceinline__ bool crt_centred(const CrtDev& crt, int ns, const uint64_t* r, uint64_t mag[4]) {
  bool neg;
  mag[0] = mag[1] = mag[2] = mag[3] = 0;
  if (ns == 1) {  // reconstructTo fast path: toBalanced (rns.go:68-73,78-91)
    const uint64_t q = crt.q[0];
    neg = r[0] > (q >> 1);
    mag[0] = neg ? q - r[0] : r[0];
  } else {  // Garner: V = x0 + q0 (x1 + q1 (x2 + ...)) in [0, Q)  (rns.go:93-99)
    uint64_t x[kMaxQ];
    for (int j = 0; j < ns; ++j) {
      const uint64_t qj = crt.q[j];
      uint64_t v = r[j];
      for (int kk = 0; kk < j; ++kk) {
        uint64_t xk = x[kk];
        if (xk >= qj) xk = (xk - qj >= qj) ? xk % qj : xk - qj;  // ring primes share a bit size
        v = mod_sub(v, xk, qj);
        v = sh_mul(v, crt.inv[j][kk], crt.inv_sh[j][kk], qj);
      }
      x[j] = v;
    }
    uint64_t V[4] = {x[ns - 1], 0, 0, 0};
    for (int j = ns - 2; j >= 0; --j) mw_muladd(V, 4, crt.q[j], x[j]);
    // V >= floor(Q/2) -> V - Q (rns.go:100-102)
    bool ge = true;
    for (int i = 3; i >= 0; --i) {
      if (V[i] != crt.Qhalf[i]) {
        ge = V[i] > crt.Qhalf[i];
        break;
      }
    }
    neg = ge;
    if (neg) {
      uint32_t br = 0;
      for (int i = 0; i < 4; ++i) mag[i] = subb(crt.Q[i], V[i], br);
    } else {
      for (int i = 0; i < 4; ++i) mag[i] = V[i];
    }
  }
  return neg;
}

__global__ __launch_bounds__(256) void round_kernel(RoundArgs a) {
  // LDS sized per launch (max(ns, nd) limbs x d words), not for kMaxQ x kMaxD: occupancy is then
  // register-limited (7 waves/SIMD) instead of LDS-limited (5)
  extern __shared__ uint64_t poly_lds[];
  const int d = a.d, tid = threadIdx.x, ns = a.src.n, nd = a.dst.n;
  auto poly = [&](int l) { return poly_lds + (long long)l * d; };
  const long long pid = blockIdx.x;
  const uint64_t* in = a.in + pid * ns * d;
  for (int k = tid; k < ns * d; k += blockDim.x) {
    const int l = k / d;
    const RnsPrime& P = a.src.p[l];
    poly(l)[k % d] = sh_mul(in[k], P.rinv, P.rinv_sh, P.q);  // IMForm
  }
  __syncthreads();
  const int half = blockDim.x >> 1;
  for (int l0 = 0; l0 < ns; l0 += 2) {
    const int l = l0 + (tid >= half ? 1 : 0);
    const bool active = l < ns;
    const int lc = active ? l : l0;
    intt_lds(poly(lc), d, a.src.bwd + (long long)lc * d, a.src.p[lc], tid % half, half, active);
  }
  // CRT per coefficient
  for (int k = tid; k < d; k += blockDim.x) {
    uint64_t r[kMaxQ];
    for (int l = 0; l < ns; ++l) r[l] = poly(l)[k];
    uint64_t mag[4];
    bool neg = crt_centred(a.crt, ns, r, mag);
    // floor(value / 2^cut) (big.Int.Rsh on a signed value rounds toward -inf)
    bool lost = false;
    int cut = a.cut;
    while (cut > 0) {
      const int sft = cut > 63 ? 63 : cut;
      lost |= (mag[0] & ((1ull << sft) - 1)) != 0;
      for (int i = 0; i < 4; ++i) mag[i] = (mag[i] >> sft) | (i + 1 < 4 ? mag[i + 1] << (64 - sft) : 0);
      cut -= sft;
    }
    if (neg && lost) {
      for (int i = 0; i < 4; ++i)
        if (++mag[i]) break;
    }
    const bool zero = !(mag[0] | mag[1] | mag[2] | mag[3]);
    // setBigCoeffTo: Euclidean mod each destination prime (rns.go:108-114), then MForm
    for (int l = 0; l < nd; ++l) {
      const RnsPrime& P = a.dst.p[l];
      const uint64_t q = P.q;
      uint64_t m = 0;
      for (int i = 0; i < 4; ++i) m = mod_add(m, sh_mul(mag[i], a.dm.pw[l][i], a.dm.pw_sh[l][i], q), q);
      if (neg && !zero) m = mod_neg(m, q);
      r[l] = sh_mul(m, P.r64, P.r64_sh, q);
    }
    for (int l = 0; l < nd; ++l) poly(l)[k] = r[l];  // each thread owns coefficient k
  }
  __syncthreads();
  for (int l0 = 0; l0 < nd; l0 += 2) {
    const int l = l0 + (tid >= half ? 1 : 0);
    const bool active = l < nd;
    const int lc = active ? l : l0;
    ntt_lds(poly(lc), d, a.dst.fwd + (long long)lc * d, a.dst.p[lc].q, tid % half, half, active);
  }
  uint64_t* out = a.out + pid * a.out_stride;
  for (int k = tid; k < a.out_rows * d; k += blockDim.x) out[k] = (k / d < nd) ? poly(k / d)[k % d] : 0;
}


// Wave-per-polynomial round for d = 256 (every Jindo shape): one wave owns one polynomial, a
// limb pair at a time in its two half-waves (lanes 0-31 limb l0, 32-63 limb l0 + 1), 8 points per
// lane in registers.  The inverse and forward 256-point transforms run as rounds of 3 + 3 + 2
// radix-2 stages (ntt64.hpp's ROW index algebra, lazy [0, 2q) Shoup butterflies) with wave-private
// LDS exchanges and no workgroup barrier; the CRT step reads each coefficient's residues from the
// wave's limb rows.  round_kernel (a workgroup per polynomial, a barrier per stage) does the same
// arithmetic; results are the same canonical residues.
constexpr int kRoundWaves = 4;
template <int RK, int LO, int PAT, bool INV>
__device__ __forceinline__ void wround(uint64_t (&e)[8], const ulonglong2* roots, const Q64& Q, uint32_t t) {
  auto xof = [&](int rho) -> uint32_t {
    if (PAT == 0) return t + 32u * rho;
    if (PAT == 1) return ((t >> 2) << 5) | ((uint32_t)rho << 2) | (t & 3u);
    return 8u * t + rho;
  };
  constexpr int NPK = 1 << RK;
#pragma unroll
  for (int sp = 0; sp < RK; ++sp) {
    const int bw = INV ? sp : RK - 1 - sp, b = LO + bw, k = 7 - b, half = 1 << bw;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int grp = j / (NPK / 2), jj = j % (NPK / 2);
      const int rho0 = grp * NPK + ((jj >> bw) << (bw + 1)) + (jj & (half - 1)), rho1 = rho0 + half;
      const ulonglong2 w = roots[(1u << k) + (xof(rho0) >> (b + 1))];
      if constexpr (INV)
        inv_bfly_lazy<false>(e[rho0], e[rho1], w.x, w.y, Q);
      else
        fwd_bfly_lazy<false>(e[rho0], e[rho1], w.x, w.y, Q);
    }
  }
}

__global__ __launch_bounds__(64 * kRoundWaves) void round256_kernel(RoundArgs a) {
  // dynamic LDS: the limbs' tables (ns inverse, then nd forward; [l][256]), then per wave `rows`
  // rows of 288 words: limb l's exchanges and its natural-order coefficients in row l
  extern __shared__ ulonglong2 rtab[];
  const int ns = a.src.n, nd = a.dst.n, rows = (std::max(ns, nd) + 1) & ~1;
  for (int i = threadIdx.x; i < (ns + nd) * 256; i += blockDim.x)
    rtab[i] = i < ns * 256 ? a.src.bwd[i] : a.dst.fwd[i - ns * 256];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, t = lane & 31u, hs = lane >> 5;
  const int wv = threadIdx.x >> 6;
  uint64_t* wl = reinterpret_cast<uint64_t*>(rtab + (ns + nd) * 256) + (size_t)wv * rows * 288;
  const long long pid = (long long)blockIdx.x * kRoundWaves + wv;
  if (pid >= a.npoly) return;
  const uint64_t* in = a.in + pid * ns * 256;
  // 1. IMForm, inverse NTT (Gentleman-Sande, bit-reversed -> natural), times 256^-1, per limb pair
  for (int l0 = 0; l0 < ns; l0 += 2) {
    const int limb = l0 + (int)hs, lc = limb < ns ? limb : l0;
    const RnsPrime& P = a.src.p[lc];
    const Q64 Q = make_q64(P.q);
    const ulonglong2* roots = rtab + lc * 256;
    const uint32_t row = 288u * (uint32_t)(l0 + (int)hs);
    const uint32_t rH = row + t, rM = row + 36 * (t >> 2) + (t & 3), rL9 = row + 9 * t, rL8 = row + 8 * t + (t >> 2);
    uint64_t e[8];
#pragma unroll
    for (int y = 0; y < 8; ++y) e[y] = sh_mul(in[lc * 256 + t + 32 * y], P.rinv, P.rinv_sh, P.q);
#pragma unroll
    for (int y = 0; y < 8; ++y) wl[rH + 33 * y] = e[y];  // H -> L (pad x >> 5)
    wave_lds_fence();
#pragma unroll
    for (int r = 0; r < 8; ++r) e[r] = wl[rL8 + r];
    wround<2, 0, 2, true>(e, roots, Q, t);
    wave_lds_fence();
#pragma unroll
    for (int r = 0; r < 8; ++r) wl[rL9 + r] = e[r];  // L -> M
    wave_lds_fence();
#pragma unroll
    for (int y = 0; y < 8; ++y) e[y] = wl[rM + 4 * y + (y >> 1)];
    wround<3, 2, 1, true>(e, roots, Q, t);
    wave_lds_fence();
#pragma unroll
    for (int y = 0; y < 8; ++y) wl[rM + 4 * y] = e[y];  // M -> H
    wave_lds_fence();
#pragma unroll
    for (int y = 0; y < 8; ++y) e[y] = wl[rH + 36 * y];
    wround<3, 5, 0, true>(e, roots, Q, t);
    wave_lds_fence();
#pragma unroll
    for (int y = 0; y < 8; ++y) wl[row + t + 32 * y] = sh_mul(e[y], P.ninv, P.ninv_sh, P.q);  // natural order
    wave_lds_fence();
  }
  // 2. CRT per coefficient (4 per lane), floor shift, the destination residues in MForm
  for (int i = 0; i < 4; ++i) {
    const int k = (int)lane + 64 * i;
    uint64_t r[kMaxQ];
    for (int l = 0; l < ns; ++l) r[l] = wl[288 * l + k];
    uint64_t mag[4];
    const bool neg = crt_centred(a.crt, ns, r, mag);
    bool lost = false;
    int cut = a.cut;
    while (cut > 0) {
      const int sft = cut > 63 ? 63 : cut;
      lost |= (mag[0] & ((1ull << sft) - 1)) != 0;
      for (int w = 0; w < 4; ++w) mag[w] = (mag[w] >> sft) | (w + 1 < 4 ? mag[w + 1] << (64 - sft) : 0);
      cut -= sft;
    }
    if (neg && lost) {
      for (int w = 0; w < 4; ++w)
        if (++mag[w]) break;
    }
    const bool zero = !(mag[0] | mag[1] | mag[2] | mag[3]);
    for (int l = 0; l < nd; ++l) {
      const RnsPrime& P = a.dst.p[l];
      const uint64_t q = P.q;
      uint64_t m = 0;
      for (int w = 0; w < 4; ++w) m = mod_add(m, sh_mul(mag[w], a.dm.pw[l][w], a.dm.pw_sh[l][w], q), q);
      if (neg && !zero) m = mod_neg(m, q);
      r[l] = sh_mul(m, P.r64, P.r64_sh, q);
    }
    for (int l = 0; l < nd; ++l) wl[288 * l + k] = r[l];
  }
  wave_lds_fence();
  // 3. forward NTT (Cooley-Tukey, natural -> bit-reversed) per destination limb pair, stored in H
  uint64_t* out = a.out + pid * a.out_stride;
  for (int l0 = 0; l0 < nd; l0 += 2) {
    const int limb = l0 + (int)hs, lc = limb < nd ? limb : l0;
    const Q64 Q = make_q64(a.dst.p[lc].q);
    const ulonglong2* roots = rtab + (ns + lc) * 256;
    const uint32_t row = 288u * (uint32_t)(l0 + (int)hs);
    const uint32_t rH = row + t, rM = row + 36 * (t >> 2) + (t & 3), rL9 = row + 9 * t, rL8 = row + 8 * t + (t >> 2);
    uint64_t e[8];
#pragma unroll
    for (int y = 0; y < 8; ++y) e[y] = wl[288 * lc + t + 32 * y];
    wave_lds_fence();
    wround<3, 5, 0, false>(e, roots, Q, t);
#pragma unroll
    for (int y = 0; y < 8; ++y) wl[rH + 36 * y] = e[y];  // H -> M
    wave_lds_fence();
#pragma unroll
    for (int y = 0; y < 8; ++y) e[y] = wl[rM + 4 * y];
    wround<3, 2, 1, false>(e, roots, Q, t);
    wave_lds_fence();
#pragma unroll
    for (int y = 0; y < 8; ++y) wl[rM + 4 * y + (y >> 1)] = e[y];  // M -> L
    wave_lds_fence();
#pragma unroll
    for (int r = 0; r < 8; ++r) e[r] = wl[rL9 + r];
    wround<2, 0, 2, false>(e, roots, Q, t);
    wave_lds_fence();
#pragma unroll
    for (int r = 0; r < 8; ++r) wl[rL8 + r] = canon(e[r], Q);  // L -> H, canonical
    wave_lds_fence();
    if (limb < nd) {
#pragma unroll
      for (int y = 0; y < 8; ++y) out[limb * 256 + t + 32 * y] = wl[rH + 33 * y];
    }
    wave_lds_fence();
  }
  for (int k = nd * 256 + (int)lane; k < a.out_rows * 256; k += 64) out[k] = 0;
}

// ------------------------------------------------------------------------------------------
// 6. sampling: the randomness Prover.Commit draws (prover.go:65-139, encoder.go:149-183) on the
// device, from six sampler domains (csprng.hpp: one AES-256-CTR key per domain, a window of
// the domain's counter space per sampler instance):
//   kDomEncCdt    Encoder.twinCDT      one instance per encode polynomial (256 words)
//   kDomCosac     Encoder.cosac        one instance per group of kCosGroup samples (in order) ...
//   kDomCosacRnd  ... and its RoundedGaussianSampler, the same groups
//   kDomMlweCdt   Prover.mlweSampler   one instance per MLWE polynomial
//   kDomMlweRnd   Prover.roundedSampler one instance per sample
//   kDomUniform   crypto/rand (MustSetRandom), one instance per field element
// Instances are numbered from `first_commit`, the index of the batch's first commit in the
// prover's sequence, so batches and ranks never share keystream.
// ------------------------------------------------------------------------------------------
enum { kDomEncCdt = 0, kDomCosac, kDomCosacRnd, kDomMlweCdt, kDomMlweRnd, kDomUniform, kNumDom };
// COSAC samples per sampler-instance pair.  8, not 16 (round 4): a wave's 64 lanes then fill from
// 2 polynomials, so cosac2's queue hands out work in half the size and its end-of-launch tail halves
// (configs[2] 61.3 K -> 62.4 K commits/s with the stream DAG, profiles/r05h_dag_ab.txt)
constexpr int kCosGroup = 8;

struct SampleArgs {
  JShape s;
  IdxDiv d_half, d_nm, d_cols;  // mlwe_noise_kernel's index split (pairs < 2^32)
  AesKey key[kNumDom];
  const uint32_t* te0;
  unsigned long long first_commit;
  // encode noise
  const uint32_t* digits;  // [B][cols+1][rows][d]
  const double* delta;     // deltaInv[exp] (encoder.go:50-67)
  CdtDev cdt_enc, cdt_mlwe;
  ZigDev zig;
  double sd_ecd, sd_ecd_blind, sd_mask, sd_mask_blind, sd_mask_mlwe;
  long long* enc_noise;   // [B][cols+1][rows][d]
  long long* mlwe_noise;  // [B][cols+1][nm][d]
  long long n_enc_pairs, n_ml_pairs;
  long long batch;
  // cdt2_noise_kernel's tail bounds: [129][size + 2], row c, entry j + 1 = the reference's tail
  // cdf sum_{x = tailLo}^{j} rho(x - c/128) / norm for j = -1 .. size (host, Go's order)
  const double* cdt_sbound;
  const int* cdt_jmax;  // [128]: v0 <= jmax[c0] decides the sample as v0 (cdt2_noise_kernel)
  int* wq;              // [0] cdt2_noise_kernel's chunk counter, [2..3] cosac2's job counter (zeroed)
};

#pragma clang fp contract(off)
// centre of coefficient k of one encode: -fpSample[k] (encoder.go:153-165), the deltaInv
// convolution of the digit polynomial, summed term by term in Go's order
__device__ __forceinline__ double enc_centre(const SampleArgs& a, const uint32_t* dg, int k) {
  const JShape& S = a.s;
  double fp = 0.0;
  for (int i = 0; i < S.exp; ++i) {
    const double di = a.delta[i];
    if (di == 0.0) continue;
    const int dd = S.d - (i + 1) * S.slots;
    if (k >= dd)
      fp = fp + di * (double)dg[k - dd];
    else
      fp = fp - di * (double)dg[k + S.d - dd];
  }
  return -fp;
}
#pragma clang fp contract(on)

// ---- d = 256 encode noise, split by sampler -----------------------------------------------
// One kernel per sampler, so a wave never waits on the other sampler's slow path:
//   cdt2_noise_kernel   wave per TwinCDT polynomial, 4 coefficients per lane (2 AES blocks);
//                       digits staged in LDS for the deltaInv centres; one guide-table lookup
//                       per sample; tails decided inline;
//   cosac2_noise_kernel COSAC groups as a work queue through one state machine.
// The sampling entry points refuse shapes these kernels do not cover (d != 256, slots % 4 != 0,
// TwinCDT tables above kCdtLdsMaxSize entries: fields with exp >= 128, or caller stddevs far above
// NewParameters').  The round-2 kernels that covered them (enc_noise_kernel, cdt_noise_kernel +
// cdt_tail_kernel) are tools/experiments/legacy_samplers.patch.
#pragma clang fp contract(off)
constexpr int kCdtLdsMaxSize = 96;  // tables' high words + guide in LDS when size <= 96 (<= 145 KiB
                                    // per workgroup with the 64 KiB AES table)
constexpr int kCdtChunk = 8;        // consecutive polynomials per chunk (queue granularity; 32 / 16 / 8 A/B: profiles/r04q_queue_chunks_ab.txt)

__device__ __forceinline__ double rl_f64(double x, int lane) {
  const uint64_t b = __double_as_longlong(x);
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)b, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), lane);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// lower_bound of u in one table: the high words from LDS, the full word from global on a tie;
// found -> index - 1 (slices.BinarySearch, twin_cdt.go:86-93)
__device__ __forceinline__ int cdt_search_hi(const uint32_t* hi, const uint64_t* full, int n, uint64_t u) {
  const uint32_t uh = (uint32_t)(u >> 32);
  int lo = 0, len = n;
  while (len > 0) {
    const int half = len >> 1, mid = lo + half;
    const uint32_t th = hi[mid];
    const bool less = th != uh ? th < uh : full[mid] < u;
    if (less) {
      lo = mid + 1;
      len -= half + 1;
    } else {
      len = half;
    }
  }
  const bool eq = lo < n && hi[lo] == uh && full[lo] == u;
  return eq ? lo - 1 : lo;
}

// dynamic LDS of cdt2_noise_kernel: high words [128][size] u32, guide [128][257] u8, key, then
// the waves' digit slots and jmax
__host__ __device__ constexpr int cdt_guide_off(int size) { return 128 * size * 4; }
__host__ __device__ constexpr int cdt_key_off(int size) { return cdt_guide_off(size) + ((128 * 257 + 3) & ~3); }

// ---- cdt2: TwinCDT for every encode polynomial, tails decided inline ----------------------
// Each wave owns a contiguous range of the batch's (commit, column, row) polynomials: TwinCDT
// polynomials are sampled; COSAC ones get their deltaInv centres (as doubles, in enc_noise)
// for cosac2_noise_kernel; skipped ones are zeroed.
// The round-2 form (cdt_noise_kernel) spent its time on (profiling variants) the deltaInv centres,
// 16 dependent global loads per polynomial, and eight table searches per lane; its v0 != v1
// tails go to a second kernel that sums up to 2 tailHi + 1 exp terms each.  Here:
//  * the polynomial's 256 digits are staged in a wave-private 1 KiB LDS slot (one 16-B store per
//    lane), the next polynomial's digits already in flight, and the 16 shifted digit quadruples a
//    lane needs are 16 independent ds_read_b128;
//  * one search per sample (table c0: guide by top byte, bisection on the high words); table c1
//    gives the same lower bound unless u lies between the two tables' entries around it (two
//    word compares; ~0.1% of samples search c1 in full);
//  * a v0 != v1 tail compares p = u / 2^64 with the reference's cdf = sum_{x <= v0} rho(x - cFrac)
//    / norm through bounds: that sum decreases with the centre, cFrac lies in [c0, c0 + 1] / 128,
//    so S[c0 + 1][v0] (1 - 2^-40) <= cdf <= S[c0][v0] (1 + 2^-40) (S summed on the host in the same
//    order; 2^-40 covers both libms and the float sums).  Outside that band the comparison is
//    decided; inside it (p within 1e-12 of the sum: p ~ 1, unseen in practice) the wave sums the
//    terms in the reference's order.  Results equal the reference's draw for draw.
// deltaInv centres of coefficients 4 lane + h (encoder.go:153-165, Go's summation order) from the
// polynomial's 256 digits in the wave's LDS slot dl: coefficient k reads digit (k + (i+1) slots)
// mod 256, added when that index wrapped; fp = the negated centres.  Leading zero deltas (12 of 16
// at the configs' shapes: b^i / p underflows the double grid) are skipped (i0); later zeros are
// added: fp starts at +0 and never becomes -0, so adding 0 * g changes nothing, and four digits'
// loads are in flight at once.  One definition for both kernels that need centres, so TwinCDT
// and COSAC polynomials see the same arithmetic (fp contract off).
typedef const __attribute__((address_space(4))) double* dconst_ptr;
__device__ __forceinline__ void enc_centres(const uint4* dl, int lane, const JShape& S, dconst_ptr dlt, int i0,
                                            double (&fp)[4]) {
  fp[0] = fp[1] = fp[2] = fp[3] = 0.0;
  auto cstep = [&](double di, int i, const uint4& q) {
    // slots % 4 == 0 (the launch condition) makes base a multiple of 4: base + h >= 256 for
    // all four coefficients or for none, so one sign per digit; fp + (-di) g == fp - di g
    const double sdi = 4 * lane + (i + 1) * S.slots >= 256 ? di : -di;
    fp[0] = fp[0] + sdi * (double)q.x;
    fp[1] = fp[1] + sdi * (double)q.y;
    fp[2] = fp[2] + sdi * (double)q.z;
    fp[3] = fp[3] + sdi * (double)q.w;
  };
  auto dslot = [&](int i) { return dl[((4 * lane + (i + 1) * S.slots) & 255) >> 2]; };
  int i = i0;
  for (; i + 4 <= S.exp; i += 4) {
    const uint4 q0 = dslot(i), q1 = dslot(i + 1), q2 = dslot(i + 2), q3 = dslot(i + 3);
    const double d0 = dlt[i], d1 = dlt[i + 1], d2 = dlt[i + 2], d3 = dlt[i + 3];
    cstep(d0, i, q0);
    cstep(d1, i + 1, q1);
    cstep(d2, i + 2, q2);
    cstep(d3, i + 3, q3);
  }
  for (; i < S.exp; ++i) cstep(dlt[i], i, dslot(i));
}

// The COSAC polynomials' centres (row 0 of the data columns, every row of the mask column: the
// stddevs other than ecdStdDev, prover.go:93-123), written as doubles into enc_noise for
// cosac2_noise_kernel: one wave per polynomial, jobs in cosac2's order.  A launch of its own
// (not part of cdt2_noise_kernel) so that the TwinCDT and COSAC samplers are independent and
// can run on two streams, each filling the other's tail.
constexpr int kCentreWaves = 4;
__global__ __launch_bounds__(64 * kCentreWaves) void cos_centre_kernel(SampleArgs a) {
  __shared__ uint4 dls[kCentreWaves][64];
  const int wl = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const JShape& S = a.s;
  const int per = S.cols + S.rows;
  const long long job = (long long)blockIdx.x * kCentreWaves + wl;
  if (job >= a.batch * per) return;
  const long long b = job / per;
  const int j = (int)(job % per);
  const int col = j < S.cols ? j : S.cols, row = j < S.cols ? 0 : j - S.cols;
  const double sd = col == S.cols ? (row == 0 ? a.sd_mask_blind : a.sd_mask) : (row == 0 ? a.sd_ecd_blind : a.sd_ecd);
  if (enc_skipped(S, col, row) || sd == a.sd_ecd) return;  // cdt2_noise_kernel's polynomials
  const long long poly = (b * (S.cols + 1) + col) * S.rows + row;
  const dconst_ptr dlt = (dconst_ptr)a.delta;
  int i0 = 0;
  while (i0 < S.exp && dlt[i0] == 0.0) ++i0;
  uint4* dl = dls[wl];
  dl[lane] = reinterpret_cast<const uint4*>(a.digits + poly * 256)[lane];
  wave_lds_fence();
  double fp[4];
  enc_centres(dl, lane, S, dlt, i0, fp);
  double2* out = reinterpret_cast<double2*>(a.enc_noise + poly * 256);
  out[2 * lane] = make_double2(-fp[0], -fp[1]);
  out[2 * lane + 1] = make_double2(-fp[2], -fp[3]);
}

constexpr int kCdt2Waves = 16;
__host__ __device__ constexpr int cdt2_dig_off(int size) { return cdt_key_off(size) + kKeyWords * 4; }
__host__ __device__ constexpr int cdt2_jmax_off(int size) { return cdt2_dig_off(size) + kCdt2Waves * 1024; }
__host__ __device__ constexpr int cdt2_dyn_lds(int size) { return cdt2_jmax_off(size) + 128 * 4; }

__global__ __launch_bounds__(64 * kCdt2Waves) void cdt2_noise_kernel(SampleArgs a) {
  __shared__ uint32_t lds[kAesLds];
  extern __shared__ uint32_t dyn[];
  const CdtDev& C = a.cdt_enc;
  const int n = C.size;
  uint32_t* thi = dyn;
  uint8_t* guide = reinterpret_cast<uint8_t*>(dyn) + cdt_guide_off(n);
  uint32_t* keyl = dyn + cdt_key_off(n) / 4;
  const int wl = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint4* dl = reinterpret_cast<uint4*>(reinterpret_cast<char*>(dyn) + cdt2_dig_off(n) + wl * 1024);
  int* jmax = reinterpret_cast<int*>(reinterpret_cast<char*>(dyn) + cdt2_jmax_off(n));
  aes_lds_fill(lds, a.te0);
  aes_key_fill(keyl, a.key[kDomEncCdt]);
  for (int i = threadIdx.x; i < 128 * n; i += blockDim.x) thi[i] = (uint32_t)(C.tables[i] >> 32);
  for (int i = threadIdx.x; i < 128 * 257; i += blockDim.x) guide[i] = C.guide[i];
  for (int i = threadIdx.x; i < 128; i += blockDim.x) jmax[i] = a.cdt_jmax[i];
  __syncthreads();
  const JShape& S = a.s;
  const long long npoly = a.batch * (S.cols + 1) * S.rows;
  const double norm = sqrt(2.0 * M_PI) * C.sigma;
  const double two_s2 = 2.0 * C.sigma * C.sigma;
  const LdsKey key{keyl};
  const int sstride = n + 2;
  // deltaInv through the constant address space: scalar loads (a plain global load waits on
  // vmcnt(0) per digit, as the kernel's stores defeat the no-clobber analysis)
  const dconst_ptr dlt = (dconst_ptr)a.delta;
  int i0 = 0;  // first nonzero deltaInv
  while (i0 < S.exp && dlt[i0] == 0.0) ++i0;
  // chunks from a counter: a wave that drew cheap polynomials (COSAC hand-offs, skipped ones)
  // takes more, so the workgroups -- one per CU, whose last wave holds its CU -- end together
  for (;;) {
    int ch = 0;
    if (lane == 0) ch = atomicAdd(a.wq, 1);
    const long long p0 = (long long)__builtin_amdgcn_readlane(ch, 0) * kCdtChunk;
    if (p0 >= npoly) break;
    const long long p1 = p0 + kCdtChunk < npoly ? p0 + kCdtChunk : npoly;
    int row = (int)(p0 % S.rows), col = (int)((p0 / S.rows) % (S.cols + 1));
    uint4 gnext = reinterpret_cast<const uint4*>(a.digits + p0 * 256)[lane];
    for (long long poly = p0; poly < p1; ++poly) {  // (b, col, row) flattened
      if (poly > p0 && ++row == S.rows) {
        row = 0;
        if (++col == S.cols + 1) col = 0;
      }
      const uint4 g = gnext;
      if (poly + 1 < p1) gnext = reinterpret_cast<const uint4*>(a.digits + (poly + 1) * 256)[lane];
      long long* out = a.enc_noise + poly * 256;
      if (enc_skipped(S, col, row)) {  // the reference draws nothing for these (prover.go:101-105,118-123)
        reinterpret_cast<longlong2*>(out)[2 * lane] = make_longlong2(0, 0);
        reinterpret_cast<longlong2*>(out)[2 * lane + 1] = make_longlong2(0, 0);
        continue;
      }
      const double sd =
          col == S.cols ? (row == 0 ? a.sd_mask_blind : a.sd_mask) : (row == 0 ? a.sd_ecd_blind : a.sd_ecd);
      if (sd != a.sd_ecd) continue;  // a COSAC polynomial: cos_centre_kernel writes its centres
      dl[lane] = g;
      wave_lds_fence();
      double fp[4];
      enc_centres(dl, lane, S, dlt, i0, fp);
      wave_lds_fence();  // the slot is rewritten for the next polynomial after these reads
      const unsigned long long gpoly =
          a.first_commit * (unsigned long long)(S.cols + 1) * S.rows + (unsigned long long)poly;
      uint64_t u[4];
      ks_words_x2(key, gpoly, (uint64_t)(2 * lane), (uint64_t)(2 * lane + 1), lds, u);
      // TwinCDTGaussianSampler.Sample (twin_cdt.go:77-111).  Fast path: the guide bucket of u's
      // top byte in table c0 holds <= 3 entries and none shares u's high word, so the lower bound
      // is lo + #(entries below u) with no equality (three LDS word compares); and v0 <= jmax[c0],
      // for which the reference returns v0 whatever v1 is: if v1 == v0 trivially, else because
      // p = u / 2^64 <= t_c0[v0 + 1] / 2^64 < (1 - 2^-40) S[c0 + 1][v0] <= the cdf it compares
      // with (host-checked per table and index, rg_jindo_set_stddevs).  Other samples (a long
      // bucket, a high-word tie, an extreme v0) take the exact path below.
      int c0[4], v0[4];
      double cf[4], flo[4];
      uint32_t slow = 0;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const double center = -fp[h];
        flo[h] = floor(center);
        cf[h] = center - flo[h];
        c0[h] = (int)((int64_t)floor(128.0 * cf[h]) % 128);
        const int t = (int)(u[h] >> 56);
        const int lo = guide[c0[h] * 257 + t];
        const int len = guide[c0[h] * 257 + t + 1] - lo;
        const uint32_t uh = (uint32_t)(u[h] >> 32);
        const uint32_t* th = thi + c0[h] * n + lo;
        int cnt = 0;
        bool tie = false;
#pragma unroll
        for (int k = 0; k < 3; ++k)
          if (k < len) {
            const uint32_t x = th[k];
            cnt += x < uh ? 1 : 0;
            tie |= x == uh;
          }
        v0[h] = lo + cnt;
        if (len > 3 || tie || v0[h] > jmax[c0[h]]) slow |= 1u << h;
      }
      int64_t res[4];
      uint32_t pend = 0;
#pragma unroll
      for (int h = 0; h < 4; ++h) res[h] = (int64_t)v0[h] + C.tail_lo + (int64_t)flo[h];
      if (__ballot(slow != 0)) {  // the exact path, literally (rare)
#pragma unroll
        for (int h = 0; h < 4; ++h)
          if ((slow >> h) & 1) {
            const int a0 = c0[h], a1 = (int)((int64_t)ceil(128.0 * cf[h]) % 128);
            const int w0 = cdt_search_hi(thi + a0 * n, C.tables + (long long)a0 * n, n, u[h]);
            const int w1 = a1 == a0 ? w0 : cdt_search_hi(thi + a1 * n, C.tables + (long long)a1 * n, n, u[h]);
            v0[h] = w0;
            res[h] = (int64_t)w1 + C.tail_lo + (int64_t)flo[h];
            if (w0 != w1) {  // the tail: p < cdf -> v0's value (twin_cdt.go:95-110)
              const double p = __ull2double_rn(u[h]) / 18446744073709551616.0;
              const double lo_b = a.cdt_sbound[(a0 + 1) * sstride + w0 + 1] * (1.0 - 9.094947017729282e-13);
              const double hi_b = a.cdt_sbound[a0 * sstride + w0 + 1] * (1.0 + 9.094947017729282e-13);
              if (p < lo_b)
                res[h] = (int64_t)w0 + C.tail_lo + (int64_t)flo[h];
              else if (!(p >= hi_b))
                pend |= 1u << h;  // within the bounds' band: sum the terms below
            }
          }
      }
      for (;;) {  // the exact sums (p within ~1e-12 of the cdf), one sample at a time across the wave
        const uint64_t any = __ballot(pend != 0);
        if (!any) break;
        const int src = __builtin_amdgcn_readfirstlane(__builtin_ctzll(any));
        const int hs = __builtin_amdgcn_readlane(pend ? __builtin_ctz(pend) : 0, src);
        double c_frac = 0.0, p = 0.0;
        int vv = 0;
#pragma unroll
        for (int h = 0; h < 4; ++h)
          if (h == hs) {
            c_frac = cf[h];
            vv = v0[h];
            p = __ull2double_rn(u[h]) / 18446744073709551616.0;
          }
        c_frac = rl_f64(c_frac, src);
        vv = __builtin_amdgcn_readlane(vv, src);
        double cdf = 0.0;
        for (int64_t x0 = C.tail_lo; x0 <= vv; x0 += 64) {
          const double xf = (double)(x0 + lane);
          const double term = exp(-(xf - c_frac) * (xf - c_frac) / two_s2) / norm;
          const int nn = (int)std::min<int64_t>(64, (int64_t)vv - x0 + 1);
          for (int i = 0; i < nn; ++i) cdf += rl_f64(term, i);
        }
        if (lane == src) {
#pragma unroll
          for (int h = 0; h < 4; ++h)
            if (h == hs && p < cdf) res[h] = (int64_t)v0[h] + C.tail_lo + (int64_t)flo[h];
          pend &= pend - 1;
        }
      }
      reinterpret_cast<longlong2*>(out)[2 * lane] = make_longlong2(res[0], res[1]);
      reinterpret_cast<longlong2*>(out)[2 * lane + 1] = make_longlong2(res[2], res[3]);
    }
  }
}

// COSACSampler.Sample (gaussian_cosac.go:22-57) with its RoundedGaussianSampler's normFloat
// (gaussian_rounded.go:77-116) as a state machine in which every state consumes exactly one
// Sample() word, from the sampler's own instance (base) or the rounded sampler's (rnd):
enum { kCoStart = 0, kCoNorm, kCoTailU, kCoTailV, kCoWedge, kCoBit, kCoRR };
__device__ __forceinline__ int co_src(int st) { return (st >= kCoNorm && st <= kCoWedge) ? 1 : 0; }
__device__ __forceinline__ double float52(uint64_t w) { return (double)(w & 0xFFFFFFFFFFFFFull) * 2.220446049250313e-16; }

// ---- cosac2: COSAC samples through one state machine, one AES block per lane per step ------
// The COSAC samples of an encode polynomial come in groups of kCosGroup consecutive
// coefficients; group g of polynomial gpoly draws from instance gpoly * (d / kCosGroup) + g of
// both COSAC domains (the sampler's own UniformSampler and its RoundedGaussianSampler's), in
// coefficient order, each sample continuing the streams where the previous one stopped (as one
// Go COSACSampler would over those samples).  Per-sample instances (round 2) left the unused
// second word of each instance's last block behind: ~3.7 blocks per sample against ~3.0 here.
// Each wave's groups (its jobs' 16 groups each, in order) form a queue; a lane takes the next
// group when its current one is done, and every iteration
//   1. lets each lane consume its buffered word (the second word of its stream's last block)
//      while the state machine wants a word it has, then
//   2. computes ONE AES block per lane: the next block of whichever stream the lane's state
//      needs (keys selected per lane from LDS), and steps on its first word,
// so every lane with work computes a useful block on every iteration (a block is only ever
// computed when its first word is consumed at once).  The lane state is kept small (x / u / y
// share a register: each is live in disjoint states).
constexpr int kCos2Threads = 1024;
constexpr int kCos2KeyStride = kKeyWords + 4;  // keys of the two streams 4 banks apart

struct Cos2Lane {
  int g;                // queue index of the current group, -1: none
  int st;               // state | zi << 8 | zb << 15 | code << 16 | sample-in-group << 20
  unsigned long long oi;  // enc_noise index of the current sample
  uint32_t pos[2];      // next word of each stream's instance
  uint32_t have;        // bit s: spare[s] holds word pos[s]
  uint64_t spare[2];
  double c_int, c_frac, t, y_round;  // t: x (wedge), u (tail), y (bit / rr)
};

// One step of the state machine on word w; returns true when the sample is done (its output
// written).  Only the common states (Norm, Bit, RR without its exp) run unconditionally; the
// divisions and exp / log of the reference's comparisons sit in branches that only lanes
// needing them take:
//   START  r < exp(-(cFrac^2) / 2 sd^2) / (sqrt(2 pi) sd) can only hold when r < 1 / (sqrt(2 pi) sd)
//          (exp <= 1): the exp and division only then;
//   RR     rr < exp(arg), arg = -((yR + cFrac)^2 - y^2) / 2 sd^2 = -D / 2 sd^2: accepted when D <= 0
//          (arg >= +-0, exp >= 1 > rr), or when rr < (1 + a')(1 - 2^-48) with a' = -D (1 / 2 sd^2)
//          (1 + 2^-50) <= arg (the product form of the quotient, its rounding covered by the
//          2^-50) and exp(arg) >= 1 + arg (exp within an ulp, covered by the 2^-48); else the
//          reference's division and exp decide.
template <class Z>
__device__ __forceinline__ bool cos2_step(Cos2Lane& L, uint64_t w, const Z& Zg, const double* sdv, long long* en) {
  const double rn = 3.442619855899;
  const int st = L.st & 255, code = (L.st >> 16) & 3;
  const double fw = float52(w);
  bool have_nf = false, done = false;
  double nf = 0.0;
  int nst = st;
  if (st == kCoNorm) {  // gaussian_rounded.go:80-92
    const uint64_t b = w >> 63;
    const uint32_t i = (uint32_t)(w & 127u);
    const uint64_t j = (w >> 7) & 0xFFFFFFFFFFFFFull;
    const double x = (double)(int64_t)((j ^ (0ull - b)) + b) * Zg.wn[i];
    if (j < Zg.kn[i]) {
      nf = x;
      have_nf = true;
    } else if (i == 0) {
      L.st = (L.st & ~(1 << 15)) | ((int)b << 15);
      nst = kCoTailU;
    } else {
      L.st = (L.st & ~(127 << 8)) | ((int)i << 8);
      L.t = x;
      nst = kCoWedge;
    }
  } else if (st == kCoBit) {  // gaussian_cosac.go:43-50
    bool cmp;
    if ((w & 1) == 0) {
      L.y_round = round(L.t) - 1.0;
      cmp = L.y_round <= 0.5;
    } else {
      L.y_round = round(L.t) + 1.0;
      cmp = L.y_round >= -0.5;
    }
    nst = cmp ? kCoRR : kCoNorm;
  } else if (st == kCoRR) {  // gaussian_cosac.go:51-55
    const double D = (L.y_round + L.c_frac) * (L.y_round + L.c_frac) - L.t * L.t;
    bool acc = D <= 0.0;
    if (!acc) {
      const double ap = -D * sdv[4 * code + 1] * (1.0 + 8.881784197001252e-16);  // a' <= arg < 0
      acc = fw < (1.0 + ap) * 0.99999999999999644729;
      if (!acc) acc = fw < exp(-D / (2.0 * sdv[4 * code] * sdv[4 * code]));
    }
    if (acc) {
      en[L.oi] = (long long)L.y_round + (long long)L.c_int;
      done = true;
    } else {
      nst = kCoNorm;
    }
  } else if (st == kCoStart) {  // gaussian_cosac.go:36-40
    nst = kCoNorm;
    if (fw < sdv[4 * code + 3]) {  // r < 1 / lead: the reference's exp comparison decides
      const double sd = sdv[4 * code];
      if (fw < exp(-(L.c_frac * L.c_frac) / (2.0 * sd * sd)) / sdv[4 * code + 2]) {
        en[L.oi] = (long long)L.c_int;
        done = true;
      }
    }
  } else if (st == kCoWedge) {  // gaussian_rounded.go:109-113
    const int zi = (L.st >> 8) & 127;
    const double f0 = Zg.fn[zi - 1], f1 = Zg.fn[zi];
    if (fw * (f0 - f1) < exp(-0.5 * L.t * L.t) - f1) {
      nf = L.t;
      have_nf = true;
    } else {
      nst = kCoNorm;
    }
  } else {  // kCoTailU / kCoTailV, gaussian_rounded.go:94-101
    const double lg = -log(fw);
    if (st == kCoTailU) {
      L.t = lg * (1.0 / rn);
      nst = kCoTailV;
    } else if (lg + lg >= L.t * L.t) {
      const double uu = L.t + rn;
      nf = ((L.st >> 15) & 1) ? -uu : uu;
      have_nf = true;
    } else {
      nst = kCoTailU;
    }
  }
  if (have_nf) {
    L.t = sdv[4 * code] * nf;
    nst = kCoBit;
  }
  L.st = (L.st & ~255) | nst;
  return done;
}

__global__ __launch_bounds__(kCos2Threads, 1) void cosac2_noise_kernel(SampleArgs a) {
  __shared__ uint32_t lds[kAesLds];
  __shared__ uint32_t keys[2 * kCos2KeyStride];
  __shared__ uint64_t zig[384];  // kn, wn, fn
  __shared__ double sdv[12];     // per sd code: sd, 1 / (2 sd^2), sqrt(2 pi) sd, 1 / that
  aes_lds_fill(lds, a.te0);
  aes_key_fill(keys, a.key[kDomCosac]);
  aes_key_fill(keys + kCos2KeyStride, a.key[kDomCosacRnd]);
  for (int i = threadIdx.x; i < 128; i += blockDim.x) {
    zig[i] = a.zig.kn[i];
    zig[128 + i] = __double_as_longlong(a.zig.wn[i]);
    zig[256 + i] = __double_as_longlong(a.zig.fn[i]);
  }
  if (threadIdx.x < 3) {
    const double sd = threadIdx.x == 0 ? a.sd_ecd_blind : threadIdx.x == 1 ? a.sd_mask : a.sd_mask_blind;
    const double lead = sqrt(2.0 * M_PI) * sd;
    sdv[4 * threadIdx.x] = sd;
    sdv[4 * threadIdx.x + 1] = 1.0 / (2.0 * sd * sd);
    sdv[4 * threadIdx.x + 2] = lead;
    sdv[4 * threadIdx.x + 3] = 1.0 / lead;
  }
  __syncthreads();
  const ZigDev Z{zig, reinterpret_cast<const double*>(zig + 128), reinterpret_cast<const double*>(zig + 256)};
  const JShape& S = a.s;
  const int per = S.cols + S.rows;
  const long long njobs = a.batch * per;
  constexpr int NG = 256 / kCosGroup;  // groups per polynomial
  // a wave's queue is refilled kCos2Chunk jobs at a time from one counter (one atomic per chunk),
  // so waves whose groups drew few words take more jobs; results do not depend on which wave draws
  // a group
  constexpr int kCos2Chunk = 64 / NG;  // jobs per refill: one group per lane of the wave
  long long total = 0;   // groups in the wave's current chunk
  long long job0 = 0;    // the chunk's first job
  bool drained = false;  // the counter passed njobs
  unsigned long long* cq = reinterpret_cast<unsigned long long*>(a.wq + 2);
  const unsigned long long pbg = a.first_commit * (unsigned long long)(S.cols + 1) * S.rows * (unsigned long long)NG;
  auto mb = [](uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
  };
  auto start_sample = [&](Cos2Lane& L) {  // the group's next sample: its centre, state START
    const double center = __longlong_as_double(a.enc_noise[L.oi]);
    L.c_int = round(center);
    L.c_frac = L.c_int - center;
    L.st = (L.st & ~0xFFFF) | kCoStart;
  };
  Cos2Lane L;
  L.g = -1;
  L.st = 0;
  unsigned long long inst = 0;  // the group's instance (both streams)
  long long next = 0;
  for (;;) {
    bool can = L.g >= 0 && ((L.have >> co_src(L.st & 255)) & 1);
    uint64_t w = 0;
    if (!__ballot(can)) {
      // no lane can step on a buffered word: lanes without a group take the next ones of the
      // queue (groups of polynomials that draw nothing are dropped here), then every lane with
      // work computes the next block of the stream its state needs and steps on its first word
      for (;;) {
        const uint64_t need = __ballot(L.g < 0);
        if (!need) break;
        if (next >= total) {
          if (drained) break;
          unsigned long long base = 0;
          if ((threadIdx.x & 63) == 0) base = atomicAdd(cq, (unsigned long long)kCos2Chunk);
          job0 = (long long)(((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(base >> 32), 0) << 32) |
                             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)base, 0));
          if (job0 >= njobs) {
            drained = true;
            break;
          }
          next = 0;
          total = (njobs - job0 < kCos2Chunk ? njobs - job0 : kCos2Chunk) * NG;
        }
        const int rank = mb(need);
        if (L.g < 0 && next + rank < total) {
          const long long g = next + rank;
          const long long job = job0 + g / NG;
          const long long b = job / per;
          const int j = (int)(job % per);
          const int col = j < S.cols ? j : S.cols, row = j < S.cols ? 0 : j - S.cols;
          const int code = col < S.cols ? 0 : (row == 0 ? 2 : 1);
          if (!enc_skipped(S, col, row) && sdv[4 * code] != a.sd_ecd) {
            const long long poly = (b * (S.cols + 1) + col) * S.rows + row;
            L.g = (int)g;
            L.oi = (unsigned long long)(poly * 256 + (g % NG) * kCosGroup);
            inst = pbg + (unsigned long long)(poly * NG + g % NG);
            L.st = code << 16;
            L.pos[0] = L.pos[1] = 0;
            L.have = 0;
            start_sample(L);
          }
        }
        next += __builtin_popcountll(need);
      }
      if (!__ballot(L.g >= 0)) break;
      if (L.g >= 0) {
        const int s = co_src(L.st & 255);
        const uint32_t p = L.pos[s];
        const LdsKey k{keys + s * kCos2KeyStride};
        if (p < 1024) {
          uint64_t w1;
          ks_words(k, inst, p / 2, lds, w, w1);
          if (s)
            L.spare[1] = w1;
          else
            L.spare[0] = w1;
        } else {  // past the first 8 KiB buffer: the XOR-accumulated refill (rare)
          w = uniform_word_at(k, lds, inst, p);
        }
        // spare[s] is word p + 1, the stream's next word once the step below has taken word p
        L.have = p < 1024 ? (L.have | (1u << s)) : (L.have & ~(1u << s));
        can = true;
      }
    } else if (can) {
      const int s = co_src(L.st & 255);
      w = s ? L.spare[1] : L.spare[0];
      L.have &= ~(1u << s);
    }
    if (can) {
      ++L.pos[co_src(L.st & 255)];
      if (cos2_step(L, w, Z, sdv, a.enc_noise)) {  // done: the group's next sample continues its streams
        const int kk = ((L.st >> 20) & 15) + 1;
        if (kk == kCosGroup) {
          L.g = -1;
        } else {
          L.st = (L.st & ~(15 << 20)) | (kk << 20);
          ++L.oi;
          start_sample(L);
        }
      }
    }
  }
}

#pragma clang fp contract(on)

// thread = (commit, column, MLWE polynomial, coefficient pair) (prover.go:130-139).  Two
// instantiations: ROUND = false covers the key columns (mlweSampler, one AES block and two table
// searches per pair), ROUND = true the mask column (the rounded Gaussian with its exp / log), so
// the table-search launch is not held at the rounded path's register count (238 VGPRs, 2 waves
// per SIMD, when both were one kernel).
constexpr int kMlweLdsTab = 512;  // mlweSampler's table in LDS up to this size (configs: 123 entries)
template <bool ROUND>
__global__ __launch_bounds__(512) void mlwe_noise_kernel(SampleArgs a) {
  __shared__ uint32_t lds[kAesLds];
  __shared__ uint32_t key[kKeyWords];
  __shared__ uint64_t mtab[ROUND ? 1 : kMlweLdsTab];
  aes_lds_fill(lds, a.te0);
  const bool tab_lds = a.cdt_mlwe.size <= kMlweLdsTab;  // else the binary search reads global memory
  if constexpr (ROUND) {
    aes_key_fill(key, a.key[kDomMlweRnd]);
  } else if (tab_lds) {
    for (int i = threadIdx.x; i < a.cdt_mlwe.size; i += blockDim.x) mtab[i] = a.cdt_mlwe.tables[i];
  }
  __syncthreads();
  const JShape& S = a.s;
  const int nm = S.in_msis + S.mlwe, half = S.d / 2;
  const int ncol = ROUND ? 1 : S.cols;  // columns this launch covers
  const long long n = a.n_ml_pairs / (S.cols + 1) * ncol;
  // grid-stride: a bounded grid fills the 64 KiB LDS tables once per workgroup, not once per 512 pairs
  for (long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x; gid < n;
       gid += (long long)gridDim.x * blockDim.x) {
    int m, j, col;
    long long b;
    if (n <= 0xffffffffLL) {
      const uint32_t g = (uint32_t)gid, r = idx_div(g, a.d_half), r2 = idx_div(r, a.d_nm);
      m = (int)(g - r * (uint32_t)half);
      j = (int)(r - r2 * (uint32_t)nm);
      if constexpr (ROUND) {
        col = S.cols;
        b = r2;
      } else {
        const uint32_t r3 = idx_div(r2, a.d_cols);
        col = (int)(r2 - r3 * (uint32_t)S.cols);
        b = r3;
      }
    } else {
      m = (int)(gid % half);
      const long long r = gid / half;
      j = (int)(r % nm);
      const long long r2 = r / nm;
      col = ROUND ? S.cols : (int)(r2 % S.cols);
      b = ROUND ? r2 : r2 / S.cols;
    }
    const long long poly = (b * (S.cols + 1) + col) * nm + j;  // (b, col, j)
    long long* out = a.mlwe_noise + poly * S.d;
    const unsigned long long gpoly = a.first_commit * (unsigned long long)(S.cols + 1) * nm + (unsigned long long)poly;
    if constexpr (!ROUND) {  // mlweSampler.Sample(0): centre 0, one table, no float tail
      uint64_t w0, w1;
      ks_words(a.key[kDomMlweCdt], gpoly, (uint64_t)m, lds, w0, w1);
      int64_t v0, v1;
      if (tab_lds) {
        v0 = cdt_search(mtab, a.cdt_mlwe.size, w0);
        v1 = cdt_search(mtab, a.cdt_mlwe.size, w1);
      } else {
        v0 = cdt_search(a.cdt_mlwe.tables, a.cdt_mlwe.size, w0);
        v1 = cdt_search(a.cdt_mlwe.tables, a.cdt_mlwe.size, w1);
      }
      out[2 * m] = v0 + a.cdt_mlwe.tail_lo;
      out[2 * m + 1] = v1 + a.cdt_mlwe.tail_lo;
    } else {  // roundedSampler.Sample(0, maskMLWEStdDev)
      for (int h = 0; h < 2; ++h) {
        const int k = 2 * m + h;
        Uniform u;
        u.init(key, lds, gpoly * S.d + k);
        out[k] = rounded_gauss(a.zig, u, 0.0, a.sd_mask_mlwe);
      }
    }
  }
}

// thread = one MustSetRandom draw: lastRow[0 .. cols*slots-2] (the last entry is zero, not
// drawn: prover.go:68-72) and the mask column's rows x slots elements (prover.go:93-115).
// Uint.SetRandom (element.go:299-343): read k = ceil(bitLen/8) bytes, clear the unused top
// bits, reject while >= q.
template <int L>
struct UniArgs {
  JShape s;
  AesKey key;
  const uint32_t* te0;
  FieldParams<L> F;
  int kbytes;
  uint32_t top_mask;
  unsigned long long first_commit;
  uint64_t* last_row;  // [B][cols*slots][L]
  uint64_t* mask;      // [B][rows][slots][L]
  long long total;     // B * (cols*slots + rows*slots)
  IdxDiv d_per;        // cols*slots + rows*slots, for total < 2^32
};

template <int L>
__global__ __launch_bounds__(512) void uniform_elems_kernel(UniArgs<L> a) {
  __shared__ uint32_t lds[kAesLds];
  __shared__ uint32_t key[kKeyWords];
  aes_lds_fill(lds, a.te0);
  aes_key_fill(key, a.key);
  __syncthreads();
  // grid-stride (see mlwe_noise_kernel); one draw per iteration
  for (long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x; gid < a.total;
       gid += (long long)gridDim.x * blockDim.x) [&] {
  const JShape& S = a.s;
  const long long nl = (long long)S.cols * S.slots, per = nl + (long long)S.rows * S.slots;
  long long b, i;
  if (a.total <= 0xffffffffLL) {
    b = idx_div((uint32_t)gid, a.d_per);
    i = gid - b * per;
  } else {
    b = gid / per;
    i = gid % per;
  }
  uint64_t* dst = i < nl ? a.last_row + (b * nl + i) * L : a.mask + (b * (per - nl) + (i - nl)) * L;
  if (i == nl - 1) {
#pragma unroll
    for (int l = 0; l < L; ++l) dst[l] = 0;
    return;
  }
  const unsigned long long inst = (a.first_commit + (unsigned long long)b) * (unsigned long long)per + (unsigned long long)i;
  if ((L % 2) == 0 && a.kbytes == 8 * L) {  // whole words (e.g. q255: 32 bytes): a try = L/2 blocks, in parallel
    const uint64_t topm = ((uint64_t)a.top_mask << 56) | 0x00FFFFFFFFFFFFFFull;
    for (uint64_t t = 0;; ++t) {
      uint64_t z[L];
      if ((t + 1) * L <= 1024) {
#pragma unroll
        for (int h = 0; h < L / 2; ++h) ks_words(LdsKey{key}, inst, t * (L / 2) + h, lds, z[2 * h], z[2 * h + 1]);
      } else {  // past the first 8 KiB buffer (uniform.go:64-82)
#pragma unroll
        for (int l = 0; l < L; ++l) z[l] = uniform_word_at(LdsKey{key}, lds, inst, t * L + l);
      }
      z[L - 1] &= topm;  // the last byte's unused top bits (element.go:320-325)
      if (!geq_q<L>(z, a.F)) {
#pragma unroll
        for (int l = 0; l < L; ++l) dst[l] = z[l];
        return;
      }
    }
  }
  Uniform u;
  u.init(key, lds, inst);
  uint64_t word = 0;
  int left = 0;  // unread bytes of `word`
  for (;;) {
    uint64_t z[L];
#pragma unroll
    for (int l = 0; l < L; ++l) z[l] = 0;
    for (int j = 0; j < a.kbytes; ++j) {
      if (!left) {
        word = u.sample();
        left = 8;
      }
      uint64_t byte = word & 255u;
      word >>= 8;
      --left;
      if (j == a.kbytes - 1) byte &= a.top_mask;
#pragma unroll
      for (int l = 0; l < L; ++l)
        if ((j >> 3) == l) z[l] |= byte << (8 * (j & 7));
    }
    if (!geq_q<L>(z, a.F)) {
#pragma unroll
      for (int l = 0; l < L; ++l) dst[l] = z[l];
      return;
    }
  }
  }();
}

// Whole-word draws (kbytes = 8 L, e.g. q255) within the first 8 KiB of each instance: a try is
// L / 2 AES blocks in parallel, up to 1024 / L tries.  A draw that needs more (its probability is
// 0.475^256 at q255) is left as all-ones -- never a value below q -- and flagged for
// uniform_fix_kernel, so this kernel carries no XOR-accumulated refill: 112 VGPRs (4 waves/SIMD)
// against the general kernel's 164 (2 waves/SIMD with its 64 KiB of LDS).
template <int L>
__global__ __launch_bounds__(512) void uniform_whole_kernel(UniArgs<L> a, int* flag, int max_tries) {
  __shared__ uint32_t lds[kAesLds];
  __shared__ uint32_t key[kKeyWords];
  aes_lds_fill(lds, a.te0);
  aes_key_fill(key, a.key);
  __syncthreads();
  const JShape& S = a.s;
  const long long nl = (long long)S.cols * S.slots, per = nl + (long long)S.rows * S.slots;
  const uint64_t topm = ((uint64_t)a.top_mask << 56) | 0x00FFFFFFFFFFFFFFull;
  const long long stride = (long long)gridDim.x * blockDim.x;
  // One try per iteration, and a lane moves on to its next element (grid-stride) as soon as its
  // current one is accepted: the wave no longer waits, element by element, for its slowest lane
  // (a try is accepted with probability q / 2^bitlen(q-1), 0.52 at q255: the most tries among 64
  // lanes averages ~6 against 1.9 per lane).  Same draws: element i's try t reads the same blocks.
  long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t* dst = nullptr;
  unsigned long long inst = 0;
  int t = 0;
  auto next = [&]() {  // from gid: the element's destination and instance; skips lastRow's last entry
    while (gid < a.total) {
      long long b, i;
      if (a.total <= 0xffffffffLL) {
        b = idx_div((uint32_t)gid, a.d_per);
        i = gid - b * per;
      } else {
        b = gid / per;
        i = gid % per;
      }
      dst = i < nl ? a.last_row + (b * nl + i) * L : a.mask + (b * (per - nl) + (i - nl)) * L;
      if (i != nl - 1) {
        inst = (a.first_commit + (unsigned long long)b) * (unsigned long long)per + (unsigned long long)i;
        t = 0;
        return;
      }
#pragma unroll
      for (int l = 0; l < L; ++l) dst[l] = 0;  // genFirstLastRow leaves it zero
      gid += stride;
    }
  };
  next();
  static_assert(L % 2 == 0, "whole 16-byte blocks per try");
  while (gid < a.total) {
    uint64_t z[L];
    bool ok = false;
    if (max_tries > 0) {  // (0: every draw left to the fix-up, the experiments build's test)
      if constexpr (L >= 4) {
#pragma unroll
        for (int h = 0; h < L / 4; ++h)
          ks_words_x2(LdsKey{key}, inst, (uint64_t)t * (L / 2) + 2 * h, (uint64_t)t * (L / 2) + 2 * h + 1, lds,
                      z + 4 * h);
      }
      if constexpr (L % 4 != 0)
        ks_words(LdsKey{key}, inst, (uint64_t)t * (L / 2) + (L / 2 - 1), lds, z[L - 2], z[L - 1]);
      z[L - 1] &= topm;  // the last byte's unused top bits (element.go:320-325)
      ok = !geq_q<L>(z, a.F);
    }
    if (ok || t + 1 >= max_tries) {
      if (!ok) *flag = 1;
#pragma unroll
      for (int l = 0; l < L; ++l) dst[l] = ok ? z[l] : ~0ull;
      gid += stride;
      next();
    } else {
      ++t;
    }
  }
}

// uniform_whole_kernel's leftovers: nothing unless a draw was flagged; then every all-ones element
// is drawn again by the general kernel's loop, refill included
template <int L>
__global__ __launch_bounds__(512) void uniform_fix_kernel(UniArgs<L> a, const int* flag) {
  if (*flag == 0) return;
  __shared__ uint32_t lds[kAesLds];
  __shared__ uint32_t key[kKeyWords];
  aes_lds_fill(lds, a.te0);
  aes_key_fill(key, a.key);
  __syncthreads();
  const JShape& S = a.s;
  const long long nl = (long long)S.cols * S.slots, per = nl + (long long)S.rows * S.slots;
  const uint64_t topm = ((uint64_t)a.top_mask << 56) | 0x00FFFFFFFFFFFFFFull;
  for (long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x; gid < a.total;
       gid += (long long)gridDim.x * blockDim.x) {
    long long b, i;
    if (a.total <= 0xffffffffLL) {
      b = idx_div((uint32_t)gid, a.d_per);
      i = gid - b * per;
    } else {
      b = gid / per;
      i = gid % per;
    }
    uint64_t* dst = i < nl ? a.last_row + (b * nl + i) * L : a.mask + (b * (per - nl) + (i - nl)) * L;
    bool ones = i != nl - 1;
#pragma unroll
    for (int l = 0; l < L; ++l) ones = ones && dst[l] == ~0ull;
    if (!ones) continue;
    const unsigned long long inst = (a.first_commit + (unsigned long long)b) * (unsigned long long)per + (unsigned long long)i;
    for (uint64_t t = 0;; ++t) {
      uint64_t z[L];
      if ((t + 1) * L <= 1024) {
#pragma unroll
        for (int h = 0; h < L / 2; ++h) ks_words(LdsKey{key}, inst, t * (L / 2) + h, lds, z[2 * h], z[2 * h + 1]);
      } else {  // past the first 8 KiB buffer (uniform.go:64-82)
#pragma unroll
        for (int l = 0; l < L; ++l) z[l] = uniform_word_at(LdsKey{key}, lds, inst, t * L + l);
      }
      z[L - 1] &= topm;
      if (!geq_q<L>(z, a.F)) {
#pragma unroll
        for (int l = 0; l < L; ++l) dst[l] = z[l];
        break;
      }
    }
  }
}

// raw Sample() words of one UniformSampler instance (rg_uniform_words_dev)
__global__ __launch_bounds__(512) void uniform_words_kernel(AesKey key, const uint32_t* te0, unsigned long long inst,
                                                            unsigned long long first, long long n, uint64_t* out) {
  __shared__ uint32_t lds[kAesLds];
  __shared__ uint32_t kl[kKeyWords];
  aes_lds_fill(lds, te0);
  aes_key_fill(kl, key);
  __syncthreads();
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n) return;
  Uniform u;
  u.init(kl, lds, inst);
  out[gid] = u.word_at(first + (unsigned long long)gid);
}
// ------------------------------------------------------------------------------------------
// 7. Verifier.Verify (verifier.go:50-282), challenges injected.  The MACs run on mac_kernel,
// the lifted inner commitments on round_kernel (cut 0, ringQOut -> ringQ); these kernels add:
//   norm_kernel    workgroup per polynomial: IMForm, INTT, centred CRT, sum of squares
//                  (verifyNorm :262-276) -> kNormW words per polynomial
//   combine_kernel A * 2^cut - B per residue (MulRNSScalarMontgomery, ...ThenSub)
//   neq_kernel     any word of x != y -> flag (verifyConsistency :203-221)
//   decode_kernel  workgroup per polynomial: IMForm, INTT, centred CRT, SetBigInt mod p,
//                  Horner in base b over the slots (DecodeTo, encoder.go:203-219)
//   dot2_kernel    one workgroup: sum right * dcd and sum batchDcd[0] * y (verifyEval :224-259)
// ------------------------------------------------------------------------------------------
constexpr int kNormW = 10;  // words of a sum of squares (|value| < 2^240, <= 2^20 values)

struct NormArgs {
  int d;
  RingDev R;
  CrtDev crt;
  const uint64_t* in;  // [npoly] at stride in_stride, R.n limbs
  long long in_stride;
  uint64_t* out;       // [npoly][kNormW]
};

__device__ __forceinline__ void mw_add(uint64_t* a, const uint64_t* b, int n) {
  uint32_t c = 0;
  for (int i = 0; i < n; ++i) a[i] = addc(a[i], b[i], c);
}

__global__ __launch_bounds__(256) void norm_kernel(NormArgs a) {
  extern __shared__ uint64_t poly_lds[];
  const int d = a.d, tid = threadIdx.x, ns = a.R.n;
  auto poly = [&](int l) { return poly_lds + (long long)l * d; };
  const long long pid = blockIdx.x;
  const uint64_t* in = a.in + pid * a.in_stride;
  for (int k = tid; k < ns * d; k += blockDim.x) {
    const int l = k / d;
    const RnsPrime& P = a.R.p[l];
    poly(l)[k % d] = sh_mul(in[k], P.rinv, P.rinv_sh, P.q);  // IMForm
  }
  __syncthreads();
  const int half = blockDim.x >> 1;
  for (int l0 = 0; l0 < ns; l0 += 2) {
    const int l = l0 + (tid >= half ? 1 : 0);
    const bool active = l < ns;
    const int lc = active ? l : l0;
    intt_lds(poly(lc), d, a.R.bwd + (long long)lc * d, a.R.p[lc], tid % half, half, active);
  }
  uint64_t acc[kNormW];
  for (int i = 0; i < kNormW; ++i) acc[i] = 0;
  for (int k = tid; k < d; k += blockDim.x) {
    uint64_t r[kMaxQ], mag[4];
    for (int l = 0; l < ns; ++l) r[l] = poly(l)[k];
    crt_centred(a.crt, ns, r, mag);
    uint64_t sq[kNormW];
    for (int i = 0; i < kNormW; ++i) sq[i] = 0;
    for (int i = 0; i < 4; ++i) {
      uint64_t carry = 0;
      for (int j = 0; j < 4; ++j) {
        uint64_t lo, hi;
        mul_wide(mag[i], mag[j], lo, hi);
        uint32_t c = 0;
        lo = addc(lo, sq[i + j], c);
        hi += c;
        c = 0;
        lo = addc(lo, carry, c);
        hi += c;
        sq[i + j] = lo;
        carry = hi;
      }
      sq[i + 4] += carry;
    }
    mw_add(acc, sq, kNormW);
  }
  __syncthreads();  // poly_lds is reused for the reduction
  for (int i = 0; i < kNormW; ++i) poly_lds[tid * kNormW + i] = acc[i];
  __syncthreads();
  for (int s = blockDim.x >> 1; s > 0; s >>= 1) {
    if (tid < s) mw_add(poly_lds + tid * kNormW, poly_lds + (tid + s) * kNormW, kNormW);
    __syncthreads();
  }
  if (tid < kNormW) a.out[pid * kNormW + tid] = poly_lds[tid];
}

// out[p][l][k] = A[p][l][k] * c_l - B[p][l][k] mod q_l  (A, B, out: [npoly][nl][d] contiguous)
__global__ __launch_bounds__(256) void combine_kernel(const uint64_t* A, const uint64_t* B, uint64_t* out,
                                                      long long n, int nl, int d, RingDev R, uint64_t c0,
                                                      uint64_t c1, uint64_t c2, uint64_t c3) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int l = (int)((i / d) % nl);
  const RnsPrime& P = R.p[l];
  const uint64_t c = l == 0 ? c0 : l == 1 ? c1 : l == 2 ? c2 : c3;
  const uint64_t cp = (uint64_t)(((unsigned __int128)c << 64) / P.q);
  out[i] = mod_sub(sh_mul(A[i], c, cp, P.q), B[i], P.q);
}

__global__ __launch_bounds__(256) void neq_kernel(const uint64_t* x, const uint64_t* y, long long n, int* flag) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && x[i] != y[i]) atomicOr(flag, 1);
}

template <int L>
struct DecodeArgs {
  int d, slots, exp, nout;
  RingDev R;
  CrtDev crt;
  FieldParams<L> F;
  uint64_t pw[4][L];  // 2^(64 i) R^2 mod p: montmul(w, pw[i]) = w 2^(64 i) R
  uint64_t bmont[L];  // base in Montgomery form
  const uint64_t* in;  // [npoly][R.n][d]
  uint64_t* out;       // [npoly][nout][L]
};

template <int L>
__global__ __launch_bounds__(256) void decode_kernel(DecodeArgs<L> a) {
  extern __shared__ uint64_t poly_lds[];  // R.n * d words, then d * L words of coefficients
  const int d = a.d, tid = threadIdx.x, ns = a.R.n;
  auto poly = [&](int l) { return poly_lds + (long long)l * d; };
  uint64_t* ce = poly_lds + (long long)ns * d;
  const long long pid = blockIdx.x;
  const uint64_t* in = a.in + pid * ns * d;
  for (int k = tid; k < ns * d; k += blockDim.x) {
    const int l = k / d;
    const RnsPrime& P = a.R.p[l];
    poly(l)[k % d] = sh_mul(in[k], P.rinv, P.rinv_sh, P.q);  // IMForm
  }
  __syncthreads();
  const int half = blockDim.x >> 1;
  for (int l0 = 0; l0 < ns; l0 += 2) {
    const int l = l0 + (tid >= half ? 1 : 0);
    const bool active = l < ns;
    const int lc = active ? l : l0;
    intt_lds(poly(lc), d, a.R.bwd + (long long)lc * d, a.R.p[lc], tid % half, half, active);
  }
  for (int k = tid; k < d; k += blockDim.x) {  // reconstructTo, then SetBigInt (mod p)
    uint64_t r[kMaxQ], mag[4];
    for (int l = 0; l < ns; ++l) r[l] = poly(l)[k];
    const bool neg = crt_centred(a.crt, ns, r, mag);
    uint64_t v[L], t[L], w[L];
#pragma unroll
    for (int i = 0; i < L; ++i) v[i] = 0;
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < L; ++j) w[j] = j == 0 ? mag[i] : 0;
      if (L == 1) w[0] = mag[i] % a.F.q[0];  // a word may exceed a one-limb p
      f_mul<L>(t, w, a.pw[i], a.F);
      f_add<L>(v, v, t, a.F);
    }
    if (neg) f_neg<L>(v, v, a.F);
#pragma unroll
    for (int j = 0; j < L; ++j) ce[(long long)k * L + j] = v[j];
  }
  __syncthreads();
  for (int i = tid; i < a.nout; i += blockDim.x) {  // Horner over j = exp-1 .. 0
    uint64_t v[L];
#pragma unroll
    for (int j = 0; j < L; ++j) v[j] = 0;
    for (int j = a.exp - 1; j >= 0; --j) {
      f_mul<L>(v, v, a.bmont, a.F);
      f_add<L>(v, v, ce + (long long)(j * a.slots + i) * L, a.F);
    }
#pragma unroll
    for (int j = 0; j < L; ++j) a.out[(pid * a.nout + i) * L + j] = v[j];
  }
}

// one workgroup: out[0] = sum_i x1[i] * y1[i] (n1 terms), out[1] = sum_i x2[i] * y2[i] (n2)
template <int L>
__global__ __launch_bounds__(256) void dot2_kernel(FieldParams<L> F, const uint64_t* x1, const uint64_t* y1,
                                                   long long n1, const uint64_t* x2, const uint64_t* y2, long long n2,
                                                   uint64_t* out) {
  __shared__ uint64_t red[256 * L];
  for (int which = 0; which < 2; ++which) {
    const uint64_t* x = which ? x2 : x1;
    const uint64_t* y = which ? y2 : y1;
    const long long n = which ? n2 : n1;
    uint64_t acc[L], t[L];
#pragma unroll
    for (int j = 0; j < L; ++j) acc[j] = 0;
    for (long long i = threadIdx.x; i < n; i += blockDim.x) {
      f_mul<L>(t, x + i * L, y + i * L, F);
      f_add<L>(acc, acc, t, F);
    }
#pragma unroll
    for (int j = 0; j < L; ++j) red[threadIdx.x * L + j] = acc[j];
    __syncthreads();
    for (int s = blockDim.x >> 1; s > 0; s >>= 1) {
      if ((int)threadIdx.x < s) f_add<L>(red + threadIdx.x * L, red + threadIdx.x * L, red + (threadIdx.x + s) * L, F);
      __syncthreads();
    }
    if (threadIdx.x < L) out[which * L + threadIdx.x] = red[threadIdx.x];
    __syncthreads();
  }
}
}  // namespace rg

// ------------------------------------------------------------------------------------------
// host
// ------------------------------------------------------------------------------------------
// Scratch of one commit stream: digits [B][cols+1][rows][d] u32, inner commitments
// [B][cols+1][inMSIS][nq][d], outer [B][outMSIS][nqo][d].  One per stream, so calls on
// different streams never share scratch (calls on one stream are ordered by the stream).
struct rg_jindo_scratch {
  rg::DevBuf digits, com, ocom;
  rg::DevBuf last, mask, en, mn;  // the sampled randomness of rg_jindo_commit_sampled_dev
  rg::DevBuf wq;                  // cdt2_noise_kernel's chunk counter
};

// Sampler setup (rg_jindo_set_stddevs): the reference's six standard deviations and the tables
// derived from them on the host (csprng_host.hpp)
struct rg_jindo_samplers {
  bool ready = false;
  double sd[6];  // ecd, ecd_blind, mask, mask_blind, mlwe, mask_mlwe
  rg::DevBuf te0, cdt_enc, cdt_guide, cdt_sbound, cdt_jmax, cdt_mlwe, zig, delta;
  int cdt_enc_size = 0, cdt_mlwe_size = 0;
  int64_t tail_lo_enc = 0, tail_lo_mlwe = 0;
  std::vector<double> h_delta;
};

struct rg_jindo {
  rg_jindo_params p;
  rg_field field;
  int device = 0;  // the handle's buffers live on this device
  rg::RnsPrime rq[rg::kMaxQ], ro[rg::kMaxQ];
  rg::DevBuf rootsq_f, rootsq_b, rootso_f, rootso_b;
  rg::CrtDev crt_q, crt_o;
  rg::DstDev dst_o, dst_q;
  rg::DevBuf ck_in, ck_mlwe, ck_out;  // the commit key, device-resident (entities.go:21-73 layouts)
  rg::DevBuf ckm_in, ckm_out;  // the same as base-256 digits for mac_mfma (inner, outer)
  int mfma_q = 0, mfma_o = 0;  // digits per residue of the MFMA MAC (0: mac_kernel)
  uint64_t base_inv;
  std::mutex mu;  // guards `scratch` and `aux`
  std::map<hipStream_t, std::unique_ptr<rg_jindo_scratch>> scratch;
  rg_jindo_samplers smp;
  // the sampled commit's helper streams and events, one set per caller stream (lazily created):
  // s[0] runs the COSAC centres + cosac2, s[1] the MLWE samplers and their prep (commit_sampled_dev)
  struct Aux {
    hipStream_t s[2] = {nullptr, nullptr};
    hipEvent_t e[4] = {nullptr, nullptr, nullptr, nullptr};
  };
  std::map<hipStream_t, Aux> aux;
  ~rg_jindo() {
    for (auto& kv : aux) {
      for (hipStream_t x : kv.second.s)
        if (x) (void)hipStreamDestroy(x);
      for (hipEvent_t x : kv.second.e)
        if (x) (void)hipEventDestroy(x);
    }
  }
};

namespace rg {

// ring.PrimitiveRoot: smallest g >= 3 that generates Z_q^* (factors by trial division +
// Pollard rho; q < 2^62)
static bool is_prime_u64(uint64_t n) {
  if (n < 2) return false;
  static const uint64_t sp[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
  for (uint64_t p : sp)
    if (n % p == 0) return n == p;
  uint64_t d = n - 1;
  int r = 0;
  while (!(d & 1)) d >>= 1, ++r;
  for (uint64_t a : sp) {
    uint64_t x = h_powmod(a, d, n);
    if (x == 1 || x == n - 1) continue;
    bool ok = false;
    for (int k = 1; k < r && !ok; ++k) {
      x = h_mulmod(x, x, n);
      ok = x == n - 1;
    }
    if (!ok) return false;
  }
  return true;
}
static uint64_t gcd_u64(uint64_t a, uint64_t b) {
  while (b) {
    uint64_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}
static uint64_t rho(uint64_t n) {
  if (!(n & 1)) return 2;
  for (uint64_t c = 1;; ++c) {
    uint64_t x = 2, y = 2, g = 1;
    while (g == 1) {
      x = (h_mulmod(x, x, n) + c) % n;
      y = (h_mulmod(y, y, n) + c) % n;
      y = (h_mulmod(y, y, n) + c) % n;
      g = gcd_u64(x > y ? x - y : y - x, n);
    }
    if (g != n) return g;
  }
}
static void factor(uint64_t n, std::vector<uint64_t>& f) {
  if (n == 1) return;
  if (is_prime_u64(n)) {
    if (std::find(f.begin(), f.end(), n) == f.end()) f.push_back(n);
    return;
  }
  uint64_t dv = rho(n);
  factor(dv, f);
  factor(n / dv, f);
}
static uint64_t primitive_root(uint64_t q) {
  std::vector<uint64_t> f;
  factor(q - 1, f);
  for (uint64_t g = 3;; ++g) {
    bool ok = true;
    for (uint64_t p : f) ok = ok && h_powmod(g, (q - 1) / p, q) != 1;
    if (ok) return g;
  }
}
static uint64_t brv(uint64_t x, int logn) {
  uint64_t r = 0;
  for (int i = 0; i < logn; ++i) r = (r << 1) | ((x >> i) & 1);
  return r;
}

static rg_status make_ring(int d, const uint64_t* primes, int n, uint64_t base, RnsPrime* P, DevBuf& fwd, DevBuf& bwd) {
  int logd = 0;
  while ((1 << logd) < d) ++logd;
  std::vector<ulonglong2> f((size_t)n * d), b((size_t)n * d);
  for (int l = 0; l < n; ++l) {
    const uint64_t q = primes[l];
    if (!is_prime_u64(q) || (q - 1) % (2 * (uint64_t)d) || (q >> 62)) return RG_ERR_INVALID;
    RnsPrime& R = P[l];
    R.q = q;
    R.r64 = (uint64_t)(((unsigned __int128)1 << 64) % q);
    R.r64_sh = h_shoup(R.r64, q);
    R.rinv = h_powmod(R.r64, q - 2, q);
    R.rinv_sh = h_shoup(R.rinv, q);
    R.one_sh = h_shoup(1, q);
    R.ninv = h_powmod((uint64_t)d, q - 2, q);
    R.ninv_sh = h_shoup(R.ninv, q);
    R.bmod = base % q;
    R.bmod_sh = h_shoup(R.bmod, q);
    const uint64_t g = primitive_root(q);
    const uint64_t psi = h_powmod(g, (q - 1) / (2 * (uint64_t)d), q), psii = h_powmod(psi, q - 2, q);
    uint64_t x = 1, y = 1;
    for (int j = 0; j < d; ++j) {
      const size_t k = (size_t)l * d + brv((uint64_t)j, logd);
      f[k].x = x;
      f[k].y = h_shoup(x, q);
      b[k].x = y;
      b[k].y = h_shoup(y, q);
      x = h_mulmod(x, psi, q);
      y = h_mulmod(y, psii, q);
    }
    R.rw1 = h_mulmod(R.r64, f[(size_t)l * d + 1].x, q);
    R.rw1_sh = h_shoup(R.rw1, q);
  }
  RG_TRY(fwd.upload(f.data(), f.size() * sizeof(ulonglong2)));
  RG_TRY(bwd.upload(b.data(), b.size() * sizeof(ulonglong2)));
  return RG_OK;
}

static void make_crt(const uint64_t* primes, int n, CrtDev& C) {
  memset(&C, 0, sizeof(C));
  C.n = n;
  for (int j = 0; j < n; ++j) {
    C.q[j] = primes[j];
    for (int k = 0; k < j; ++k) {
      C.inv[j][k] = h_powmod(primes[k] % primes[j], primes[j] - 2, primes[j]);
      C.inv_sh[j][k] = h_shoup(C.inv[j][k], primes[j]);
    }
  }
  unsigned __int128 acc;
  uint64_t Q[5] = {1, 0, 0, 0, 0};
  for (int j = 0; j < n; ++j) {
    uint64_t carry = 0;
    for (int i = 0; i < 4; ++i) {
      acc = (unsigned __int128)Q[i] * primes[j] + carry;
      Q[i] = (uint64_t)acc;
      carry = (uint64_t)(acc >> 64);
    }
  }
  for (int i = 0; i < 4; ++i) {
    C.Q[i] = Q[i];
    C.Qhalf[i] = (Q[i] >> 1) | (i + 1 < 4 ? Q[i + 1] << 63 : 0);
  }
}

static void make_dst(const uint64_t* primes, int n, DstDev& D) {
  memset(&D, 0, sizeof(D));
  D.n = n;
  for (int l = 0; l < n; ++l) {
    const uint64_t q = primes[l];
    uint64_t p = 1 % q;
    const uint64_t r64 = (uint64_t)(((unsigned __int128)1 << 64) % q);
    for (int i = 0; i < 4; ++i) {
      D.pw[l][i] = p;
      D.pw_sh[l][i] = h_shoup(p, q);
      p = h_mulmod(p, r64, q);
    }
  }
}

static RingDev ring_dev(const RnsPrime* P, int n, const DevBuf& f, const DevBuf& b) {
  RingDev R;
  memset(&R, 0, sizeof(R));
  R.n = n;
  for (int l = 0; l < n; ++l) R.p[l] = P[l];
  R.fwd = f.as<const ulonglong2>();
  R.bwd = b.as<const ulonglong2>();
  return R;
}

static JShape shape_of(const rg_jindo_params& p, long long nv) {
  JShape s;
  s.rank = p.rank;
  s.rows = p.rows;
  s.cols = p.cols;
  s.slots = p.slots;
  s.exp = p.exp;
  s.d = p.d;
  s.in_msis = p.in_msis;
  s.out_msis = p.out_msis;
  s.mlwe = p.mlwe;
  s.dcmp = p.dcmp;
  s.log_in_cut = p.log_in_cut;
  s.log_out_cut = p.log_out_cut;
  s.nq = p.nq;
  s.nqo = p.nqo;
  s.base = p.base;
  s.nv = nv;
  return s;
}

static rg_status validate(const rg_jindo_params* p) {
  if (!p) return RG_ERR_INVALID;
  if (p->nq < 1 || p->nq > kMaxQ || p->nqo < 1 || p->nqo > kMaxQ || p->nqo > p->nq) return RG_ERR_INVALID;
  if (p->d < 2 || p->d > kMaxD || (p->d & (p->d - 1))) return RG_ERR_INVALID;
  if (p->rows < 2 || p->cols < 1 || p->slots < 1 || p->exp < 1 || p->slots * p->exp > p->d) return RG_ERR_INVALID;
  if (p->in_msis < 1 || p->in_msis > kMaxJ || p->out_msis < 1 || p->out_msis > kMaxJ || p->mlwe < 0) return RG_ERR_INVALID;
  if (p->dcmp != (p->cols + 1) * p->in_msis) return RG_ERR_INVALID;
  if (p->base < 2 || (p->base >> 32)) return RG_ERR_INVALID;
  for (int l = 0; l < p->nq; ++l)
    if (p->q[l] <= p->base) return RG_ERR_INVALID;  // digits (<= b) are used as residues directly
  for (int l = 0; l < p->nqo; ++l)
    if (p->qo[l] <= p->base) return RG_ERR_INVALID;
  if (!(p->field_limbs == 1 || p->field_limbs == 2 || p->field_limbs == 4 || p->field_limbs == 7 ||
        p->field_limbs == 14))
    return RG_ERR_UNSUPPORTED;
  return RG_OK;
}

static rg_status build(rg_jindo* J) {
  const rg_jindo_params& p = J->p;
  if (!init_field(&J->field, p.field_limbs, p.field_q)) return RG_ERR_INVALID;
  RG_TRY(make_ring(p.d, p.q, p.nq, p.base, J->rq, J->rootsq_f, J->rootsq_b));
  RG_TRY(make_ring(p.d, p.qo, p.nqo, p.base, J->ro, J->rootso_f, J->rootso_b));
  make_crt(p.q, p.nq, J->crt_q);
  make_crt(p.qo, p.nqo, J->crt_o);
  make_dst(p.qo, p.nqo, J->dst_o);
  make_dst(p.q, p.nq, J->dst_q);
  J->base_inv = (uint64_t)(((unsigned __int128)1 << 64) / p.base);
  return RG_OK;
}

static size_t ck_sizes(const rg_jindo_params& p, size_t* in, size_t* ml, size_t* out) {
  *in = (size_t)p.in_msis * p.rows * p.nq * p.d;
  *ml = (size_t)p.in_msis * p.mlwe * p.nq * p.d;
  *out = (size_t)p.out_msis * p.dcmp * p.nqo * p.d;
  return *in + *ml + *out;
}

template <int L>
static rg_status launch_digits(const rg_jindo* J, size_t batch, const uint64_t* v, long long nv, const uint64_t* last,
                               const uint64_t* mask, uint32_t* digits, hipStream_t st) {
  DigitArgs<L> a;
  a.s = shape_of(J->p, nv);
  memcpy(a.F.q, J->field.q, 8 * L);
  a.F.qinv = J->field.qinv;
  a.base_inv = J->base_inv;
  const uint64_t b2 = (uint64_t)J->p.base * J->p.base;
  a.b2 = (b2 >> 32) ? 0 : b2;
  a.b2_inv = a.b2 ? (uint64_t)(((unsigned __int128)1 << 64) / b2) : 0;
  int qbits = 0;
  for (int l = L - 1; l >= 0 && !qbits; --l)
    if (J->field.q[l]) qbits = 64 * l + 64 - __builtin_clzll(J->field.q[l]);
  a.dc = dc_constants((uint64_t)J->p.base, J->p.exp, L, qbits);
  a.v = v;
  a.last_row = last;
  a.mask = mask;
  a.digits = digits;
  a.total = (long long)batch * (J->p.cols + 1) * J->p.rows * J->p.slots;
  a.d_slots = make_idxdiv((uint32_t)J->p.slots);
  a.d_rows = make_idxdiv((uint32_t)J->p.rows);
  a.d_cols1 = make_idxdiv((uint32_t)(J->p.cols + 1));
  const long long blocks = (a.total + 255) / 256;
  hipLaunchKernelGGL(digits_kernel<L>, dim3((unsigned)blocks), dim3(256), 0, st, a);
  return check_launch("jindo digits");
}

// The calling stream's scratch, grown to `batch` commits.  Growing first drains the stream (its
// earlier commits may still read the old buffers); other streams are untouched.
static rg_status stream_scratch(rg_jindo* J, size_t batch, hipStream_t st, rg_jindo_scratch** out) {
  const rg_jindo_params& p = J->p;
  const size_t d = p.d;
  std::lock_guard<std::mutex> lk(J->mu);
  std::unique_ptr<rg_jindo_scratch>& S = J->scratch[st];
  if (!S) S.reset(new rg_jindo_scratch());
  const size_t b_dig = batch * (p.cols + 1) * p.rows * d * 4, b_com = batch * (p.cols + 1) * p.in_msis * p.nq * d * 8,
               b_oc = batch * p.out_msis * p.nqo * d * 8;
  if (S->digits.bytes < b_dig || S->com.bytes < b_com || S->ocom.bytes < b_oc) RG_HIP(hipStreamSynchronize(st));
  RG_TRY(S->digits.alloc(b_dig));
  RG_TRY(S->com.alloc(b_com));
  RG_TRY(S->ocom.alloc(b_oc));
  *out = S.get();
  return RG_OK;
}

static MfmaPrime mfma_prime(const RnsPrime& P) { return MfmaPrime{P.q, P.rinv, P.rinv_sh, P.one_sh}; }

// MacArgs (legacy kernel layout) -> MfmaMacArgs over the digit key `key` (mac_mfma_key_dev)
static MfmaMacArgs mfma_args(const MacArgs& m, const DevBuf& key) {
  MfmaMacArgs a;
  memset(&a, 0, sizeof(a));
  a.per_col = (long long)m.nl * m.d;
  a.ncols = m.ncols;
  a.J = m.J;
  a.T1 = m.T1;
  a.T2 = m.T2;
  a.Tc = (m.T1 + m.T2 + 7) / 8;
  mac_mfma_key_ptrs(key, a.per_col, m.T1 + m.T2, &a.Ak, &a.corr);
  a.B1 = m.B1;
  a.b1_col = m.b1_col;
  a.b1_term = m.b1_term;
  a.B2 = m.B2;
  a.b2_col = m.b2_col;
  a.b2_term = m.b2_term;
  a.C = m.C;
  a.c_col = m.c_col;
  a.c_j = m.c_j;
  a.out = m.out;
  a.d = m.d;
  for (int l = 0; l < m.nl && l < kMfmaMaxQ; ++l) a.P[l] = mfma_prime(m.P[l]);
  return a;
}

// A handle's buffers belong to the device it was created on
static rg_status on_device(const rg_jindo* J) {
  int cur = -1;
  RG_HIP(hipGetDevice(&cur));
  if (cur != J->device) {
    set_last_error("rg_jindo handle used on device " + std::to_string(cur) + ", created on " +
                   std::to_string(J->device));
    return RG_ERR_INVALID;
  }
  return RG_OK;
}

// The deterministic Ajtai core (prover.go:144-202) over a batch of NTT-domain openings:
// inner MAC, rounding into Opening.InCommit, outer MAC and rounding into Commitment.Value.
// CRT rounding of `npoly` polynomials: round256_kernel (a wave per polynomial) for d = 256 and
// primes below 2^62 (its lazy butterflies need 2q < 2^63), round_kernel otherwise.  round256
// against round_kernel at configs[4]: 429 vs 513 us per launch (profiles/r05s_round_wave_ab.txt)
static rg_status launch_round(RoundArgs ra, long long npoly, hipStream_t st) {
  ra.npoly = npoly;
  bool small = ra.d == 256;
  for (int l = 0; l < ra.src.n; ++l) small = small && ra.src.p[l].q < (1ull << 62);
  for (int l = 0; l < ra.dst.n; ++l) small = small && ra.dst.p[l].q < (1ull << 62);
  if (small) {
    const int rows = (std::max(ra.src.n, ra.dst.n) + 1) & ~1;
    const size_t lds = (size_t)(ra.src.n + ra.dst.n) * 256 * sizeof(ulonglong2) + (size_t)kRoundWaves * rows * 288 * 8;
    hipLaunchKernelGGL(round256_kernel, dim3((unsigned)((npoly + kRoundWaves - 1) / kRoundWaves)), dim3(64 * kRoundWaves),
                       lds, st, ra);
  } else {
    hipLaunchKernelGGL(round_kernel, dim3((unsigned)npoly), dim3(256),
                       (size_t)std::max(ra.src.n, ra.dst.n) * ra.d * 8, st, ra);
  }
  return check_launch("jindo round");
}

static rg_status commit_core(rg_jindo* J, size_t batch, const uint64_t* d_enc, const uint64_t* d_mlwe,
                             uint64_t* d_incom, uint64_t* d_com, rg_jindo_scratch* sc, hipStream_t st) {
  const rg_jindo_params& p = J->p;
  const int d = p.d, nq = p.nq, nqo = p.nqo, nm = p.in_msis + p.mlwe;
  // 3. inner MAC
  MacArgs ma;
  memset(&ma, 0, sizeof(ma));
  ma.d = d;
  ma.nl = nq;
  ma.J = p.in_msis;
  ma.ncols = (long long)batch * (p.cols + 1);
  ma.T1 = p.rows;
  ma.A1 = J->ck_in.as<uint64_t>();
  ma.B1 = d_enc;
  ma.b1_col = (long long)p.rows * nq * d;
  ma.b1_term = (long long)nq * d;
  ma.T2 = p.mlwe;
  ma.A2 = J->ck_mlwe.as<uint64_t>();
  ma.B2 = d_mlwe;
  ma.b2_col = (long long)nm * nq * d;
  ma.b2_term = (long long)nq * d;
  ma.C = d_mlwe + (long long)p.mlwe * nq * d;  // MLWE[i][mlwe + j]
  ma.c_col = (long long)nm * nq * d;
  ma.c_j = (long long)nq * d;
  ma.out = sc->com.as<uint64_t>();
  for (int l = 0; l < nq; ++l) ma.P[l] = J->rq[l];
  if (J->mfma_q) {
    RG_TRY(launch_mac_mfma(mfma_args(ma, J->ckm_in), J->mfma_q, st));
  } else {
    RG_TRY(launch_mac(ma, st));
  }
  // 4. inner round -> Opening.InCommit (column i, j -> index i*inMSIS + j)
  RoundArgs ra;
  memset(&ra, 0, sizeof(ra));
  ra.d = d;
  ra.cut = p.log_in_cut;
  ra.src = ring_dev(J->rq, nq, J->rootsq_f, J->rootsq_b);
  ra.dst = ring_dev(J->ro, nqo, J->rootso_f, J->rootso_b);
  ra.crt = J->crt_q;
  ra.dm = J->dst_o;
  ra.in = sc->com.as<uint64_t>();
  ra.out = d_incom;
  ra.out_stride = (long long)nqo * d;
  ra.out_rows = nqo;
  {
    const long long npoly = (long long)batch * (p.cols + 1) * p.in_msis;  // == batch * dcmp, same order
    RG_TRY(launch_round(ra, npoly, st));
  }
  // 5. outer MAC + round -> Commitment.Value (ringQ-shaped rows, rows >= nqo zero)
  MacArgs mo;
  memset(&mo, 0, sizeof(mo));
  mo.d = d;
  mo.nl = nqo;
  mo.J = p.out_msis;
  mo.ncols = (long long)batch;
  mo.T1 = p.dcmp;
  mo.A1 = J->ck_out.as<uint64_t>();
  mo.B1 = d_incom;
  mo.b1_col = (long long)p.dcmp * nqo * d;
  mo.b1_term = (long long)nqo * d;
  mo.out = sc->ocom.as<uint64_t>();
  for (int l = 0; l < nqo; ++l) mo.P[l] = J->ro[l];
  if (J->mfma_o) {
    RG_TRY(launch_mac_mfma(mfma_args(mo, J->ckm_out), J->mfma_o, st));
  } else {
    RG_TRY(launch_mac(mo, st));
  }
  RoundArgs ro = ra;
  ro.cut = p.log_out_cut;
  ro.src = ring_dev(J->ro, nqo, J->rootso_f, J->rootso_b);
  ro.crt = J->crt_o;
  ro.in = sc->ocom.as<uint64_t>();
  ro.out = d_com;
  ro.out_stride = (long long)nq * d;
  ro.out_rows = nq;
  RG_TRY(launch_round(ro, (long long)batch * p.out_msis, st));
  RG_TRY(check_launch("jindo round(out)"));
  return RG_OK;
}

// 1. digits of every encode's source elements into the stream's scratch
static rg_status digits_stage(rg_jindo* J, size_t batch, const uint64_t* d_v, size_t nv, const uint64_t* d_last,
                              const uint64_t* d_mask, uint32_t* digits, hipStream_t st) {
  switch (J->p.field_limbs) {
    case 1: return launch_digits<1>(J, batch, d_v, (long long)nv, d_last, d_mask, digits, st);
    case 2: return launch_digits<2>(J, batch, d_v, (long long)nv, d_last, d_mask, digits, st);
    case 4: return launch_digits<4>(J, batch, d_v, (long long)nv, d_last, d_mask, digits, st);
    case 7: return launch_digits<7>(J, batch, d_v, (long long)nv, d_last, d_mask, digits, st);
    default: return launch_digits<14>(J, batch, d_v, (long long)nv, d_last, d_mask, digits, st);
  }
}

// 2. encode tails + MLWE finalize with their NTTs (prep256_kernel): jobs [0, n_enc) are the encode
// polynomials, [n_enc, n_enc + n_ml) the MLWE ones; `part` selects both or one of the two sets
enum PrepPart { kPrepAll = 3, kPrepEnc = 1, kPrepMlwe = 2 };
static rg_status prep_launch(rg_jindo* J, size_t batch, size_t nv, const uint32_t* digits, const int64_t* d_en,
                             const int64_t* d_mn, uint64_t* d_enc, uint64_t* d_mlwe, int part, hipStream_t st) {
  const rg_jindo_params& p = J->p;
  const int d = p.d, nq = p.nq, nm = p.in_msis + p.mlwe;
  PrepArgs pa;
  pa.s = shape_of(p, (long long)nv);
  pa.R = ring_dev(J->rq, nq, J->rootsq_f, J->rootsq_b);
  pa.digits = digits;
  pa.enc_noise = reinterpret_cast<const long long*>(d_en);
  pa.mlwe_noise = reinterpret_cast<const long long*>(d_mn);
  pa.enc = d_enc;
  pa.mlwe = d_mlwe;
  pa.n_enc = (part & kPrepEnc) ? (long long)batch * (p.cols + 1) * p.rows : 0;
  const long long n_ml = (part & kPrepMlwe) ? (long long)batch * (p.cols + 1) * nm : 0;
  pa.n_ml = n_ml;
  pa.clim = (long long)(((uint64_t)1 << 61) / p.base);
  if (pa.n_enc + n_ml == 0) return RG_OK;
  bool q61 = true;  // prep256's lazy [0, 8q) needs q < 2^61 (every configs ring prime is <= 59 bits)
  for (int l = 0; l < nq; ++l) q61 = q61 && J->rq[l].q < (1ull << 61);
  if (d == 256 && q61) {  // else prep_kernel: a workgroup per polynomial, any d and q
    const long long jobs = pa.n_enc + n_ml;
    const dim3 g((unsigned)((jobs + kPrepWaves - 1) / kPrepWaves)), b(64 * kPrepWaves);
    const size_t twl = (size_t)nq * 256 * sizeof(ulonglong2);
    // large launches (configs[4]'s encode prep, 2.4 M jobs): 12-wave workgroups, so each table
    // staging serves 12 polynomials instead of 4 (configs[4] +1.2%; at configs[2]'s 0.3 M jobs the
    // 4-wave form is 1% faster: profiles/r05ao_prep_workgroup_ab.txt)
    constexpr int kBigWaves = 12;
    // (minimum waves per SIMD 8 or 1 instead of 6, round 2-5's RINGO_JINDO_PREP_W: slower at both
    // configs shapes, removed in round 6)
    bool lazy = true;  // every ring prime below 2^64 / 36: prep_round skips its x reductions
    for (int l = 0; l < nq; ++l) lazy = lazy && J->rq[l].q < ~0ull / 36;
    if (nq <= 2 && jobs >= (1LL << 20)) {
      const dim3 gb((unsigned)((jobs + kBigWaves - 1) / kBigWaves)), bb(64 * kBigWaves);
      if (lazy)
        hipLaunchKernelGGL((prep256_kernel<2, true, kBigWaves, true>), gb, bb, twl, st, pa);
      else
        hipLaunchKernelGGL((prep256_kernel<2, true, kBigWaves>), gb, bb, twl, st, pa);
    } else if (nq <= 2 && lazy)
      hipLaunchKernelGGL((prep256_kernel<6, true, kPrepWaves, true>), g, b, twl, st, pa);
    else if (nq <= 2)
      hipLaunchKernelGGL((prep256_kernel<6, true>), g, b, twl, st, pa);
    else
      hipLaunchKernelGGL((prep256_kernel<6, false>), g, b, twl, st, pa);
  } else {
    hipLaunchKernelGGL(prep_kernel, dim3((unsigned)(pa.n_enc + n_ml)), dim3(256), 0, st, pa);
  }
  return check_launch("jindo prep");
}

// 2.-5. from the digits and the randomness: encode tails + MLWE finalize with their NTTs, then the core
static rg_status commit_from_digits(rg_jindo* J, size_t batch, size_t nv, const uint32_t* digits, const int64_t* d_en,
                                    const int64_t* d_mn, uint64_t* d_incom, uint64_t* d_enc, uint64_t* d_mlwe,
                                    uint64_t* d_com, rg_jindo_scratch* sc, hipStream_t st) {
  RG_TRY(prep_launch(J, batch, nv, digits, d_en, d_mn, d_enc, d_mlwe, kPrepAll, st));
  return commit_core(J, batch, d_enc, d_mlwe, d_incom, d_com, sc, st);
}

static rg_status commit_dev(rg_jindo* J, size_t batch, const uint64_t* d_v, size_t nv, const uint64_t* d_last,
                            const uint64_t* d_mask, const int64_t* d_en, const int64_t* d_mn, uint64_t* d_incom,
                            uint64_t* d_enc, uint64_t* d_mlwe, uint64_t* d_com, hipStream_t st) {
  const rg_jindo_params& p = J->p;
  if (nv < 1 || nv > (size_t)p.rank) return RG_ERR_RANK;
  if (batch == 0) return RG_OK;
  RG_TRY(on_device(J));
  rg_jindo_scratch* sc = nullptr;
  RG_TRY(stream_scratch(J, batch, st, &sc));
  uint32_t* digits = sc->digits.as<uint32_t>();
  RG_TRY(digits_stage(J, batch, d_v, nv, d_last, d_mask, digits, st));
  return commit_from_digits(J, batch, nv, digits, d_en, d_mn, d_incom, d_enc, d_mlwe, d_com, sc, st);
}

// ---- sampling (csprng.hpp) -------------------------------------------------------------
static rg_status make_keys(const rg_jindo_seeds* seeds, AesKey* keys) {
  const uint8_t* sd[kNumDom] = {seeds->enc_cdt, seeds->enc_cosac, seeds->enc_cosac_round,
                                seeds->mlwe_cdt, seeds->mlwe_round, seeds->uniform};
  for (int i = 0; i < kNumDom; ++i) {
    uint8_t r[48];
    if (!sha384(sd[i], 32, r)) {
      set_last_error("libcrypto SHA384 unavailable");
      return RG_ERR_UNSUPPORTED;
    }
    aes256_expand(r, keys[i].rk);
    for (int w = 0; w < 4; ++w)
      keys[i].iv[w] = ((uint32_t)r[32 + 4 * w] << 24) | ((uint32_t)r[33 + 4 * w] << 16) | ((uint32_t)r[34 + 4 * w] << 8) |
                      r[35 + 4 * w];
  }
  return RG_OK;
}

template <int L>
static rg_status launch_uniform(const rg_jindo* J, size_t batch, const AesKey& key, unsigned long long first,
                                uint64_t* last, uint64_t* mask, int* flag, hipStream_t st) {
  UniArgs<L> a;
  a.s = shape_of(J->p, 1);
  a.key = key;
  a.te0 = J->smp.te0.as<uint32_t>();
  memcpy(a.F.q, J->field.q, 8 * L);
  a.F.qinv = J->field.qinv;
  // element.go:305-318: bitLen of q - 1, k bytes, top-byte mask
  int bitlen = 0;
  {
    uint64_t qm1[16];
    memcpy(qm1, J->field.q, 8 * L);
    for (int l = 0; l < L; ++l)
      if (qm1[l]--) break;
    for (int l = L - 1; l >= 0; --l)
      if (qm1[l]) {
        bitlen = 64 * l + 64 - __builtin_clzll(qm1[l]);
        break;
      }
  }
  a.kbytes = (bitlen + 7) / 8;
  const int bb = bitlen % 8 ? bitlen % 8 : 8;
  a.top_mask = (1u << bb) - 1u;
  a.first_commit = first;
  a.last_row = last;
  a.mask = mask;
  a.total = (long long)batch * ((long long)J->p.cols * J->p.slots + (long long)J->p.rows * J->p.slots);
  a.d_per = make_idxdiv((uint32_t)(J->p.cols * J->p.slots + J->p.rows * J->p.slots));
  const dim3 ug((unsigned)std::min<long long>((a.total + 511) / 512, 1024));
  // whole-word draws: about 4 elements per lane (the flattened try loop balances lanes only over
  // several elements), at least one workgroup per CU
  const dim3 ugw((unsigned)std::max<long long>(std::min<long long>((a.total + 512 * 4 - 1) / (512 * 4), 1024), std::min<long long>((a.total + 511) / 512, 256)));
  if constexpr (L % 2 == 0) {
    if (a.kbytes == 8 * L) {  // whole words: the common draws, then the (practically never) long ones
      const char* kt = knob(Knob::JindoUniTries);  // experiments build: cap the tries (fix-up test)
      const int tries = std::max(0, std::min(1024 / L, kt ? atoi(kt) : 1024 / L));
      RG_HIP(hipMemsetAsync(flag, 0, sizeof(int), st));
      hipLaunchKernelGGL(uniform_whole_kernel<L>, ugw, dim3(512), 0, st, a, flag, tries);
      RG_TRY(check_launch("jindo uniform (whole words)"));
      hipLaunchKernelGGL(uniform_fix_kernel<L>, ug, dim3(512), 0, st, a, (const int*)flag);
      return check_launch("jindo uniform (long draws)");
    }
  }
  hipLaunchKernelGGL(uniform_elems_kernel<L>, ug, dim3(512), 0, st, a);
  return check_launch("jindo uniform");
}

// lastRow/mask (crypto/rand), then digits, then every Gaussian sample of the batch
// Streams: st runs MustSetRandom, the digits, the COSAC centres and TwinCDT (cdt2); s_cos, once the
// centres are done (event e_dig), cosac2; s_ml, once st reaches this call (event e_start),
// the MLWE samplers, which need neither.  s_cos / s_ml may be st itself (one stream, no events).
// The caller joins s_cos and s_ml back into st before it reads their outputs.
static rg_status sample_stage(rg_jindo* J, size_t batch, const uint64_t* d_v, size_t nv, const rg_jindo_seeds* seeds,
                              unsigned long long first, uint64_t* d_last, uint64_t* d_mask, int64_t* d_en,
                              int64_t* d_mn, uint32_t* digits, rg_jindo_scratch* sc, hipStream_t st,
                              hipStream_t s_cos = nullptr, hipStream_t s_ml = nullptr, hipEvent_t e_start = nullptr,
                              hipEvent_t e_dig = nullptr) {
  if (!s_cos) s_cos = st;
  if (!s_ml) s_ml = st;
  const rg_jindo_params& p = J->p;
  if (!J->smp.ready) {
    set_last_error("rg_jindo_set_stddevs was not called on this handle");
    return RG_ERR_INVALID;
  }
  const rg_jindo_samplers& S = J->smp;
  // the shapes the device samplers cover (every NewParameters shape of a field with exp <= 64)
  if (p.d != 256 || p.slots % 4 != 0 || S.cdt_enc_size > kCdtLdsMaxSize ||
      cdt2_dyn_lds(S.cdt_enc_size) + (int)sizeof(uint32_t) * kAesLds > 163840) {
    set_last_error("device sampling needs d = 256, slots % 4 == 0 and an encode TwinCDT table of <= 96 entries (got d = " +
                   std::to_string(p.d) + ", slots = " + std::to_string(p.slots) + ", table " +
                   std::to_string(S.cdt_enc_size) + ")");
    return RG_ERR_UNSUPPORTED;
  }
  SampleArgs a;
  memset(&a, 0, sizeof(a));
  RG_TRY(make_keys(seeds, a.key));
  rg_status s;
  if (!sc->wq.p) {  // [0] cdt2's chunk counter, [2..3] cosac2's job counter, [4] uniform's long-draw flag
    std::lock_guard<std::mutex> lk(J->mu);
    RG_TRY(sc->wq.alloc(256));
  }
  int* uflag = sc->wq.as<int>() + 4;
  if (s_ml != st) {
    RG_HIP(hipEventRecord(e_start, st));
    RG_HIP(hipStreamWaitEvent(s_ml, e_start, 0));
  }
  switch (p.field_limbs) {
    case 1: s = launch_uniform<1>(J, batch, a.key[kDomUniform], first, d_last, d_mask, uflag, st); break;
    case 2: s = launch_uniform<2>(J, batch, a.key[kDomUniform], first, d_last, d_mask, uflag, st); break;
    case 4: s = launch_uniform<4>(J, batch, a.key[kDomUniform], first, d_last, d_mask, uflag, st); break;
    case 7: s = launch_uniform<7>(J, batch, a.key[kDomUniform], first, d_last, d_mask, uflag, st); break;
    default: s = launch_uniform<14>(J, batch, a.key[kDomUniform], first, d_last, d_mask, uflag, st); break;
  }
  RG_TRY(s);
  RG_TRY(digits_stage(J, batch, d_v, nv, d_last, d_mask, digits, st));
  a.s = shape_of(p, (long long)nv);
  a.te0 = S.te0.as<uint32_t>();
  a.first_commit = first;
  a.digits = digits;
  a.delta = S.delta.as<double>();
  a.cdt_enc = CdtDev{S.cdt_enc.as<uint64_t>(), S.cdt_guide.as<uint8_t>(), S.cdt_enc_size, S.tail_lo_enc, S.sd[0]};
  a.cdt_mlwe = CdtDev{S.cdt_mlwe.as<uint64_t>(), nullptr, S.cdt_mlwe_size, S.tail_lo_mlwe, S.sd[4]};
  const uint64_t* zg = S.zig.as<uint64_t>();
  a.zig = ZigDev{zg, reinterpret_cast<const double*>(zg + 128), reinterpret_cast<const double*>(zg + 256)};
  a.sd_ecd = S.sd[0];
  a.sd_ecd_blind = S.sd[1];
  a.sd_mask = S.sd[2];
  a.sd_mask_blind = S.sd[3];
  a.sd_mask_mlwe = S.sd[5];
  a.enc_noise = reinterpret_cast<long long*>(d_en);
  a.mlwe_noise = reinterpret_cast<long long*>(d_mn);
  const int nm = p.in_msis + p.mlwe;
  a.n_enc_pairs = (long long)batch * (p.cols + 1) * p.rows * (p.d / 2);
  a.n_ml_pairs = (long long)batch * (p.cols + 1) * nm * (p.d / 2);
  a.d_half = make_idxdiv((uint32_t)(p.d / 2));
  a.d_nm = make_idxdiv((uint32_t)nm);
  a.d_cols = make_idxdiv((uint32_t)std::max(p.cols, 1));
  a.batch = (long long)batch;
  {
    const long long npoly = (long long)batch * (p.cols + 1) * p.rows;
    const unsigned g = (unsigned)std::min<long long>((npoly + kCdt2Waves - 1) / kCdt2Waves, 256);
    a.cdt_sbound = S.cdt_sbound.as<double>();
    a.cdt_jmax = S.cdt_jmax.as<int>();
    a.wq = sc->wq.as<int>();
    RG_HIP(hipMemsetAsync(a.wq, 0, 4 * sizeof(int), st));  // [0]: cdt2's chunks, [2..3]: cosac2's jobs (u64)
    // the COSAC centres (small) ahead of cdt2 on st: launched on s_cos beside cdt2 they wait for
    // cdt2's one-per-CU workgroups to finish (configs[4]: 6.9 ms), and cosac2 with them
    const long long ncos = (long long)batch * (p.cols + p.rows);  // COSAC jobs
    hipLaunchKernelGGL(cos_centre_kernel, dim3((unsigned)((ncos + kCentreWaves - 1) / kCentreWaves)),
                       dim3(64 * kCentreWaves), 0, st, a);
    RG_TRY(check_launch("jindo enc noise (COSAC centres)"));
    if (s_cos != st) {
      RG_HIP(hipEventRecord(e_dig, st));
      RG_HIP(hipStreamWaitEvent(s_cos, e_dig, 0));
    }
    hipLaunchKernelGGL(cdt2_noise_kernel, dim3(g), dim3(64 * kCdt2Waves), cdt2_dyn_lds(S.cdt_enc_size), st, a);
    RG_TRY(check_launch("jindo enc noise (TwinCDT)"));
    const long long w2 = kCos2Threads / 64;
    const unsigned g2 = (unsigned)std::min<long long>((ncos + w2 - 1) / w2, 256);
    hipLaunchKernelGGL(cosac2_noise_kernel, dim3(g2), dim3(kCos2Threads), 0, s_cos, a);
    RG_TRY(check_launch("jindo enc noise (COSAC)"));
  }
  {
    const long long per_col = a.n_ml_pairs / (p.cols + 1);
    if (p.cols > 0) {
      const long long n = per_col * p.cols;
      hipLaunchKernelGGL(mlwe_noise_kernel<false>, dim3((unsigned)std::min<long long>((n + 511) / 512, 1024)),
                         dim3(512), 0, s_ml, a);
      RG_TRY(check_launch("jindo mlwe noise (table)"));
    }
    hipLaunchKernelGGL(mlwe_noise_kernel<true>, dim3((unsigned)std::min<long long>((per_col + 511) / 512, 1024)),
                       dim3(512), 0, s_ml, a);
  }
  return check_launch("jindo mlwe noise (rounded)");
}

// scratch for the sampled randomness of `batch` commits
static rg_status sample_scratch(rg_jindo* J, size_t batch, rg_jindo_scratch* sc, hipStream_t st) {
  const rg_jindo_params& p = J->p;
  const size_t L = p.field_limbs, d = p.d, nm = p.in_msis + p.mlwe;
  const size_t bl = batch * p.cols * p.slots * L * 8, bm = batch * p.rows * p.slots * L * 8,
               be = batch * (p.cols + 1) * p.rows * d * 8, bn = batch * (p.cols + 1) * nm * d * 8;
  std::lock_guard<std::mutex> lk(J->mu);
  if (sc->last.bytes < bl || sc->mask.bytes < bm || sc->en.bytes < be || sc->mn.bytes < bn)
    RG_HIP(hipStreamSynchronize(st));
  RG_TRY(sc->last.alloc(bl));
  RG_TRY(sc->mask.alloc(bm));
  RG_TRY(sc->en.alloc(be));
  RG_TRY(sc->mn.alloc(bn));
  return RG_OK;
}

// ------------------------------------------------------------------------------------------
// Prover.Evaluate core (prover.go:205-324): the MulCoeffsMontgomeryThenAdd loops, with the
// Fiat-Shamir challenges (batch, left, chals) injected by the caller.  Every loop is a
// per-(limb, coeff) dot product, so each maps onto mac_kernel with J = 1 and the loop's own
// strides.
// ------------------------------------------------------------------------------------------
static MacArgs dot_args(const RnsPrime* P, int nl, int d, long long nout, int T, const uint64_t* A, const uint64_t* B,
                        long long b_out, long long b_term, uint64_t* out) {
  MacArgs m;
  memset(&m, 0, sizeof(m));
  m.d = d;
  m.nl = nl;
  m.J = 1;
  m.ncols = nout;
  m.T1 = T;
  m.A1 = A;
  m.B1 = B;
  m.b1_col = b_out;
  m.b1_term = b_term;
  m.out = out;
  for (int l = 0; l < nl; ++l) m.P[l] = P[l];
  return m;
}

// Prover.Evaluate's batch combination (prover.go:254-266): a J = 1 dot product over the batch's
// T commits, out[col][lk] = (sum_t A[t][lk] B[col][t][lk]) 2^-64 mod q, read once from HBM.
// T = batch is the long axis (512 at the configs[4] shard) and the column count is modest (the
// 144 InCommit / 432 MLWE polynomials), so mac_kernel's thread per (4 columns, lk) left too few
// waves in flight for the opening stream.  Here a 256-thread workgroup owns 64 lk x NC columns
// and its 4 waves split the terms (wave w: t = w, w + 4, ...), each term's loads unrolled x2;
// the four exact 128-bit partial sums are added through LDS, then reduced once.
constexpr int kDotNC = 4;
__global__ __launch_bounds__(256) void dot_split_kernel(MacArgs a) {
  __shared__ uint64_t red[3][kDotNC][2][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long per_col = (long long)a.nl * a.d;
  const long long nlkb = per_col / 64;
  const long long lk = (blockIdx.x % nlkb) * 64 + lane;
  const long long col0 = (blockIdx.x / nlkb) * kDotNC;
  const int nc = (int)min((long long)kDotNC, a.ncols - col0);
  const int T = a.T1;
  Acc<false> acc[kDotNC];
#pragma unroll
  for (int c = 0; c < kDotNC; ++c) acc[c].zero();
  const uint64_t* A = a.A1 + lk;
  const uint64_t* Bp = a.B1 + lk;
#pragma unroll 2
  for (int t = w; t < T; t += 4) {
    const uint64_t av = A[(long long)t * per_col];
    uint64_t bv[kDotNC];
#pragma unroll
    for (int c = 0; c < kDotNC; ++c) bv[c] = c < nc ? Bp[(col0 + c) * a.b1_col + t * a.b1_term] : 0;
#pragma unroll
    for (int c = 0; c < kDotNC; ++c) acc[c].mac(av, bv[c]);
  }
  if (w > 0) {
#pragma unroll
    for (int c = 0; c < kDotNC; ++c) {
      red[w - 1][c][0][lane] = acc[c].lo;
      red[w - 1][c][1][lane] = acc[c].hi;
    }
  }
  __syncthreads();
  if (w != 0) return;
  const RnsPrime& P = a.P[(int)(lk / a.d)];
#pragma unroll
  for (int c = 0; c < kDotNC; ++c) {
#pragma unroll
    for (int v = 0; v < 3; ++v) {  // exact: (lo, hi) += (lo', hi'), the sum stays below 2^128
      uint32_t cy = 0;
      acc[c].lo = addc(acc[c].lo, red[v][c][0][lane], cy);
      acc[c].hi += red[v][c][1][lane] + cy;
    }
    if (c < nc) a.out[(col0 + c) * per_col + lk] = acc[c].reduce(P);
  }
}

static rg_status launch_dot(const MacArgs& m, hipStream_t st) {
  uint64_t qmax = 0;
  for (int l = 0; l < m.nl; ++l) qmax = std::max(qmax, m.P[l].q);
  const bool narrow = 2.0 * log2((double)(qmax - 1)) + log2((double)m.T1 + 1.0) < 127.5;
  if (m.J != 1 || m.T2 != 0 || m.C || !narrow || (m.nl * m.d) % 64 != 0)
    return launch_mac(m, st);
  const long long blocks = (m.ncols + kDotNC - 1) / kDotNC * ((long long)m.nl * m.d / 64);
  hipLaunchKernelGGL(dot_split_kernel, dim3((unsigned)blocks), dim3(256), 0, st, m);
  return check_launch("jindo eval dot");
}

static rg_status eval_batch(const rg_jindo* J, size_t batch, const uint64_t* incom, const uint64_t* enc,
                            const uint64_t* mlwe, const uint64_t* bq, const uint64_t* bo, uint64_t* ob_incom,
                            uint64_t* ob_enc, uint64_t* ob_mlwe, hipStream_t st) {
  const rg_jindo_params& p = J->p;
  const long long pq = (long long)p.nq * p.d, po = (long long)p.nqo * p.d, nm = p.in_msis + p.mlwe;
  const long long n_inc = p.dcmp, n_enc = (long long)(p.cols + 1) * p.rows, n_ml = (long long)(p.cols + 1) * nm;
  if (!bq) {  // params.batch == 1: openBatch = open[0] (prover.go:267-269)
    RG_HIP(hipMemcpyAsync(ob_incom, incom, 8 * n_inc * po, hipMemcpyDeviceToDevice, st));
    RG_HIP(hipMemcpyAsync(ob_enc, enc, 8 * n_enc * pq, hipMemcpyDeviceToDevice, st));
    RG_HIP(hipMemcpyAsync(ob_mlwe, mlwe, 8 * n_ml * pq, hipMemcpyDeviceToDevice, st));
    return RG_OK;
  }
  const int T = (int)batch;  // term i = commit i, scaled by its batch challenge (:254-266)
  RG_TRY(launch_dot(dot_args(J->ro, p.nqo, p.d, n_inc, T, bo, incom, po, n_inc * po, ob_incom), st));
  RG_TRY(launch_dot(dot_args(J->rq, p.nq, p.d, n_enc, T, bq, enc, pq, n_enc * pq, ob_enc), st));
  RG_TRY(launch_dot(dot_args(J->rq, p.nq, p.d, n_ml, T, bq, mlwe, pq, n_ml * pq, ob_mlwe), st));
  return RG_OK;
}

// x mod q over limb-planar polynomials (Shoup by 1 reduces any 64-bit word): folds the
// cross-GPU sum of partial openBatches (each < q, at most 2^64 / q of them) back to residues
__global__ __launch_bounds__(256) void rns_reduce_kernel(uint64_t* x, long long npoly, int nl, int d, RingDev R) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npoly * nl * d) return;
  const RnsPrime& P = R.p[(int)((i / d) % nl)];
  x[i] = sh_mul(x[i], 1, P.one_sh, P.q);
}

}  // namespace rg

using namespace rg;

// ---- Verifier.Verify (verifier.go:50-282) ----------------------------------------------------
// nmTest < nm with nmTest = Float64(isqrt(S)) (verifyNorm :278-281), decided exactly: the test is
// S < K^2 with K the smallest integer whose float64 is >= nm (ceil(nm) up to 2^53; above, the
// midpoint below nm, + 1 when nm's mantissa is odd, as ties round to even).
static bool norm_below(const uint64_t* S, double nm) {
  constexpr int NW = kNormW;
  if (!(nm > 0)) return false;
  uint64_t K[NW] = {0}, K2[2 * NW] = {0};
  int e;
  const double fr = frexp(nm, &e);
  const uint64_t M = (uint64_t)ldexp(fr, 53);
  const int E = e - 53;
  if (E <= 0) {
    const double c = ceil(nm);
    if (c >= 18446744073709551616.0) return true;
    K[0] = (uint64_t)c;
  } else {
    if (E / 64 >= NW) return true;
    const int sub_e = (M == (1ull << 52)) ? E - 2 : E - 1;  // half the gap to the double below
    K[E / 64] = M << (E % 64);
    if (E % 64 && E / 64 + 1 < NW) K[E / 64 + 1] = M >> (64 - E % 64);
    uint64_t h[NW] = {0};
    if (sub_e >= 0) h[sub_e / 64] = 1ull << (sub_e % 64);
    HostField::sub_n(K, K, h, NW);
    if (M & 1)
      for (int k = 0; k < NW; ++k)
        if (++K[k]) break;
  }
  for (int a = 0; a < NW; ++a) {
    uint64_t c = 0;
    for (int b = 0; b < NW; ++b) {
      const unsigned __int128 t = (unsigned __int128)K[a] * K[b] + K2[a + b] + c;
      K2[a + b] = (uint64_t)t;
      c = (uint64_t)(t >> 64);
    }
    K2[a + NW] += c;
  }
  for (int w = 2 * NW - 1; w >= NW; --w)
    if (K2[w]) return true;
  for (int w = NW - 1; w >= 0; --w)
    if (S[w] != K2[w]) return S[w] < K2[w];
  return false;
}

template <int L>
static rg_status launch_decode(const rg_jindo* J, const uint64_t* in, long long npoly, int nout, uint64_t* out,
                               hipStream_t st) {
  if (npoly == 0) return RG_OK;
  const rg_jindo_params& p = J->p;
  DecodeArgs<L> a;
  memset(&a, 0, sizeof(a));
  a.d = p.d;
  a.slots = p.slots;
  a.exp = p.exp;
  a.nout = nout;
  a.R = ring_dev(J->rq, p.nq, J->rootsq_f, J->rootsq_b);
  a.crt = J->crt_q;
  memcpy(a.F.q, J->field.q, 8 * L);
  a.F.qinv = J->field.qinv;
  const HostField H(&J->field);
  uint64_t t32[16], t64[16];
  H.from_u64(t32, 1ull << 32);
  H.mul(t64, t32, t32);  // Montgomery form of 2^64
  memcpy(a.pw[0], J->field.r2, 8 * L);
  for (int i = 1; i < 4; ++i) H.mul(a.pw[i], a.pw[i - 1], t64);
  H.from_u64(a.bmont, p.base);
  a.in = in;
  a.out = out;
  const size_t lds = ((size_t)p.nq * p.d + (size_t)p.d * L) * 8;
  hipLaunchKernelGGL(decode_kernel<L>, dim3((unsigned)npoly), dim3(256), lds, st, a);
  return check_launch("jindo decode");
}

template <int L>
static rg_status launch_dot2(const rg_jindo* J, const uint64_t* x1, const uint64_t* y1, long long n1,
                             const uint64_t* x2, const uint64_t* y2, long long n2, uint64_t* out, hipStream_t st) {
  FieldParams<L> F;
  memcpy(F.q, J->field.q, 8 * L);
  F.qinv = J->field.qinv;
  hipLaunchKernelGGL(dot2_kernel<L>, dim3(1), dim3(256), 0, st, F, x1, y1, n1, x2, y2, n2, out);
  return check_launch("jindo dot");
}

static rg_status decode_any(const rg_jindo* J, const uint64_t* in, long long npoly, int nout, uint64_t* out,
                            hipStream_t st) {
  switch (J->p.field_limbs) {
    case 1: return launch_decode<1>(J, in, npoly, nout, out, st);
    case 2: return launch_decode<2>(J, in, npoly, nout, out, st);
    case 4: return launch_decode<4>(J, in, npoly, nout, out, st);
    case 7: return launch_decode<7>(J, in, npoly, nout, out, st);
    default: return launch_decode<14>(J, in, npoly, nout, out, st);
  }
}
static rg_status dot2_any(const rg_jindo* J, const uint64_t* x1, const uint64_t* y1, long long n1, const uint64_t* x2,
                          const uint64_t* y2, long long n2, uint64_t* out, hipStream_t st) {
  switch (J->p.field_limbs) {
    case 1: return launch_dot2<1>(J, x1, y1, n1, x2, y2, n2, out, st);
    case 2: return launch_dot2<2>(J, x1, y1, n1, x2, y2, n2, out, st);
    case 4: return launch_dot2<4>(J, x1, y1, n1, x2, y2, n2, out, st);
    case 7: return launch_dot2<7>(J, x1, y1, n1, x2, y2, n2, out, st);
    default: return launch_dot2<14>(J, x1, y1, n1, x2, y2, n2, out, st);
  }
}

static rg_status launch_norm(const rg_jindo* J, bool outer, const uint64_t* in, long long npoly, long long stride,
                             uint64_t* out, hipStream_t st) {
  if (npoly == 0) return RG_OK;
  const rg_jindo_params& p = J->p;
  NormArgs a;
  memset(&a, 0, sizeof(a));
  a.d = p.d;
  a.R = outer ? ring_dev(J->ro, p.nqo, J->rootso_f, J->rootso_b) : ring_dev(J->rq, p.nq, J->rootsq_f, J->rootsq_b);
  a.crt = outer ? J->crt_o : J->crt_q;
  a.in = in;
  a.in_stride = stride;
  a.out = out;
  const size_t lds = std::max((size_t)a.R.n * p.d, (size_t)256 * kNormW) * 8;
  hipLaunchKernelGGL(norm_kernel, dim3((unsigned)npoly), dim3(256), lds, st, a);
  return check_launch("jindo norm");
}

static rg_status launch_combine(const RnsPrime* P, int nl, int d, int cut, const uint64_t* A, const uint64_t* B,
                                uint64_t* out, long long npoly, hipStream_t st) {
  uint64_t c[4] = {0, 0, 0, 0};
  RingDev R;
  memset(&R, 0, sizeof(R));
  R.n = nl;
  for (int l = 0; l < nl; ++l) {
    R.p[l] = P[l];
    unsigned __int128 x = 1;
    for (int i = 0; i < cut; ++i) x = (x * 2) % P[l].q;  // 2^cut mod q
    c[l] = (uint64_t)x;
  }
  const long long n = npoly * nl * d;
  hipLaunchKernelGGL(combine_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, A, B, out, n, nl, d, R, c[0],
                     c[1], c[2], c[3]);
  return check_launch("jindo combine");
}

extern "C" {

rg_status rg_jindo_eval_batch_dev(const rg_jindo* J, size_t batch, const uint64_t* d_incom, const uint64_t* d_enc,
                                  const uint64_t* d_mlwe, const uint64_t* d_bq, const uint64_t* d_bo,
                                  uint64_t* d_ob_incom, uint64_t* d_ob_enc, uint64_t* d_ob_mlwe, void* stream) {
  if (!J || batch == 0 || !d_incom || !d_enc || !d_mlwe || !d_ob_incom || !d_ob_enc || !d_ob_mlwe ||
      (!d_bq != !d_bo) || (!d_bq && batch != 1))
    return RG_ERR_INVALID;
  return eval_batch(J, batch, d_incom, d_enc, d_mlwe, d_bq, d_bo, d_ob_incom, d_ob_enc, d_ob_mlwe, as_stream(stream));
}

rg_status rg_jindo_eval_partial_dev(const rg_jindo* J, const uint64_t* d_ob_enc, const uint64_t* d_left,
                                    uint64_t* d_partial, void* stream) {
  if (!J || !d_ob_enc || !d_left || !d_partial) return RG_ERR_INVALID;
  const rg_jindo_params& p = J->p;
  const long long pq = (long long)p.nq * p.d;
  // out i in [0, cols]: sum_j left[j] * Enc[i][j] (prover.go:274-282); i = cols is PartialMask
  return launch_mac(dot_args(J->rq, p.nq, p.d, p.cols + 1, p.rows, d_left, d_ob_enc, (long long)p.rows * pq, pq,
                             d_partial),
                    as_stream(stream));
}

rg_status rg_jindo_eval_respond_dev(const rg_jindo* J, const uint64_t* d_ob_enc, const uint64_t* d_ob_mlwe,
                                    const uint64_t* d_chals, uint64_t* d_pf_enc, uint64_t* d_pf_mlwe, void* stream) {
  if (!J || !d_ob_enc || !d_ob_mlwe || !d_chals || !d_pf_enc || !d_pf_mlwe) return RG_ERR_INVALID;
  const rg_jindo_params& p = J->p;
  const long long pq = (long long)p.nq * p.d, nm = p.in_msis + p.mlwe;
  hipStream_t st = as_stream(stream);
  // pf.Encode[i] = Enc[cols][i] + sum_j chals[j] * Enc[j][i] (prover.go:300-306)
  MacArgs e = dot_args(J->rq, p.nq, p.d, p.rows, p.cols, d_chals, d_ob_enc, pq, (long long)p.rows * pq, d_pf_enc);
  e.C = d_ob_enc + (long long)p.cols * p.rows * pq;
  e.c_col = pq;
  RG_TRY(launch_mac(e, st));
  // pf.MLWE[i] = MLWE[cols][i] + sum_j chals[j] * MLWE[j][i] (:308-314)
  MacArgs m = dot_args(J->rq, p.nq, p.d, nm, p.cols, d_chals, d_ob_mlwe, pq, nm * pq, d_pf_mlwe);
  m.C = d_ob_mlwe + (long long)p.cols * nm * pq;
  m.c_col = pq;
  return launch_mac(m, st);
}


rg_status rg_jindo_verify_dev(const rg_jindo* J, size_t batch, const uint64_t* d_com, const uint64_t* d_bq,
                              const uint64_t* d_bo, const uint64_t* d_chals, const uint64_t* d_left,
                              const uint64_t* d_right, const uint64_t* d_y, const uint64_t* d_pf_incom,
                              const uint64_t* d_pf_partial, const uint64_t* d_pf_enc, const uint64_t* d_pf_mlwe,
                              double in_com_dcmp_two_nm, double res_two_nm, rg_jindo_verify_result* res,
                              void* stream) {
  if (!J || !res || !d_com || !d_chals || !d_left || !d_right || !d_y || !d_pf_incom || !d_pf_partial || !d_pf_enc ||
      !d_pf_mlwe)
    return RG_ERR_INVALID;
  if (batch < 1 || (batch > 1 && (!d_bq || !d_bo))) return RG_ERR_INVALID;
  RG_TRY(on_device(J));
  const rg_jindo_params& p = J->p;
  const int d = p.d, nq = p.nq, nqo = p.nqo, L = p.field_limbs;
  const long long pq = (long long)nq * d, po = (long long)nqo * d, nm = p.in_msis + p.mlwe;
  hipStream_t st = as_stream(stream);
  const long long n_out = p.dcmp + p.out_msis, n_in = p.rows + nm + p.in_msis;
  DevBuf a_out, b_out, c_out, lift, a_in, b_in, c_in, p1, p2, norms, flag, dcd, bd, ev;
  RG_TRY(a_out.alloc(8 * p.out_msis * po));
  RG_TRY(b_out.alloc(8 * p.out_msis * po));
  RG_TRY(c_out.alloc(8 * p.out_msis * po));
  RG_TRY(lift.alloc(8 * p.dcmp * pq));
  RG_TRY(a_in.alloc(8 * p.in_msis * pq));
  RG_TRY(b_in.alloc(8 * p.in_msis * pq));
  RG_TRY(c_in.alloc(8 * p.in_msis * pq));
  RG_TRY(p1.alloc(8 * pq));
  RG_TRY(p2.alloc(8 * pq));
  RG_TRY(norms.alloc(8 * (n_out + n_in) * kNormW));
  RG_TRY(flag.alloc(sizeof(int)));
  RG_TRY(dcd.alloc(8 * (size_t)p.cols * p.slots * L));
  RG_TRY(bd.alloc(8 * (size_t)batch * L));
  RG_TRY(ev.alloc(8 * 2 * (size_t)L));
  uint64_t* nrm = norms.as<uint64_t>();
  // verifyOuterCommitment (:136-161): A = sum_j com[j][i] * batchOut[j] (or com[0][i]),
  // C = A * 2^logOutCut - sum_j Out[i][j] * Proof.InCommit[j]
  if (batch > 1) {
    MacArgs m = dot_args(J->ro, nqo, d, p.out_msis, (int)batch, d_bo, d_com, pq, (long long)p.out_msis * pq,
                         a_out.as<uint64_t>());
    RG_TRY(launch_mac(m, st));
  } else {
    RG_HIP(hipMemcpy2DAsync(a_out.p, 8 * po, d_com, 8 * pq, 8 * po, p.out_msis, hipMemcpyDeviceToDevice, st));
  }
  {
    MacArgs m = dot_args(J->ro, nqo, d, 1, p.dcmp, J->ck_out.as<uint64_t>(), d_pf_incom, 0, po, b_out.as<uint64_t>());
    m.J = p.out_msis;
    RG_TRY(launch_mac(m, st));
  }
  RG_TRY(launch_combine(J->ro, nqo, d, p.log_out_cut, a_out.as<uint64_t>(), b_out.as<uint64_t>(), c_out.as<uint64_t>(),
                        p.out_msis, st));
  RG_TRY(launch_norm(J, true, d_pf_incom, p.dcmp, po, nrm, st));
  RG_TRY(launch_norm(J, true, c_out.as<uint64_t>(), p.out_msis, po, nrm + p.dcmp * kNormW, st));
  // verifyInnerCommitment (:164-200): lift = MForm(NTT(ModUpQtoP(pfInv.InCommit))) (centred),
  // A = sum_{j<cols} lift[j in_msis + i] * chals[j] + lift[cols in_msis + i],
  // C = A * 2^logInCut - (sum In[i][j] * Encode[j] + sum MLWE_ck[i][j] * MLWE[j] + MLWE[mlwe + i])
  {
    RoundArgs ra;
    memset(&ra, 0, sizeof(ra));
    ra.d = d;
    ra.cut = 0;
    ra.src = ring_dev(J->ro, nqo, J->rootso_f, J->rootso_b);
    ra.dst = ring_dev(J->rq, nq, J->rootsq_f, J->rootsq_b);
    ra.crt = J->crt_o;
    ra.dm = J->dst_q;
    ra.in = d_pf_incom;
    ra.out = lift.as<uint64_t>();
    ra.out_stride = pq;
    ra.out_rows = nq;
    RG_TRY(launch_round(ra, p.dcmp, st));
  }
  {
    MacArgs m = dot_args(J->rq, nq, d, p.in_msis, p.cols, d_chals, lift.as<uint64_t>(), pq, (long long)p.in_msis * pq,
                         a_in.as<uint64_t>());
    m.C = lift.as<uint64_t>() + (long long)p.cols * p.in_msis * pq;
    m.c_col = pq;
    RG_TRY(launch_mac(m, st));
  }
  {
    MacArgs m = dot_args(J->rq, nq, d, 1, p.rows, J->ck_in.as<uint64_t>(), d_pf_enc, 0, pq, b_in.as<uint64_t>());
    m.J = p.in_msis;
    m.T2 = p.mlwe;
    m.A2 = J->ck_mlwe.as<uint64_t>();
    m.B2 = d_pf_mlwe;
    m.b2_term = pq;
    m.C = d_pf_mlwe + (long long)p.mlwe * pq;
    m.c_j = pq;
    RG_TRY(launch_mac(m, st));
  }
  RG_TRY(launch_combine(J->rq, nq, d, p.log_in_cut, a_in.as<uint64_t>(), b_in.as<uint64_t>(), c_in.as<uint64_t>(),
                        p.in_msis, st));
  uint64_t* nin = nrm + n_out * kNormW;
  RG_TRY(launch_norm(J, false, d_pf_enc, p.rows, pq, nin, st));
  RG_TRY(launch_norm(J, false, d_pf_mlwe, nm, pq, nin + p.rows * kNormW, st));
  RG_TRY(launch_norm(J, false, c_in.as<uint64_t>(), p.in_msis, pq, nin + (p.rows + nm) * kNormW, st));
  // verifyConsistency (:203-221): sum left[i] * Encode[i] == sum chals[i] * Partial[i] + PartialMask
  RG_TRY(launch_mac(dot_args(J->rq, nq, d, 1, p.rows, d_left, d_pf_enc, 0, pq, p1.as<uint64_t>()), st));
  {
    MacArgs m = dot_args(J->rq, nq, d, 1, p.cols, d_chals, d_pf_partial, 0, pq, p2.as<uint64_t>());
    m.C = d_pf_partial + (long long)p.cols * pq;
    RG_TRY(launch_mac(m, st));
  }
  RG_HIP(hipMemsetAsync(flag.p, 0, sizeof(int), st));
  hipLaunchKernelGGL(neq_kernel, dim3((unsigned)((pq + 255) / 256)), dim3(256), 0, st, p1.as<uint64_t>(),
                     p2.as<uint64_t>(), pq, flag.as<int>());
  RG_TRY(check_launch("jindo consistency"));
  // verifyEval (:224-259): sum_{i,j} right[i slots + j] * Decode(pfInv.Partial[i])[j] ==
  // sum_i Decode(INTT(IMForm(batch[i])))[0] * y[i]  (or y[0])
  RG_TRY(decode_any(J, d_pf_partial, p.cols, p.slots, dcd.as<uint64_t>(), st));
  const uint64_t* yb = d_y;
  if (batch > 1) {
    RG_TRY(decode_any(J, d_bq, (long long)batch, 1, bd.as<uint64_t>(), st));
    yb = bd.as<uint64_t>();
  }
  RG_TRY(dot2_any(J, d_right, dcd.as<uint64_t>(), (long long)p.cols * p.slots, yb, d_y, batch > 1 ? (long long)batch : 0,
                  ev.as<uint64_t>(), st));
  // results to the host
  std::vector<uint64_t> hn((size_t)(n_out + n_in) * kNormW), he(2 * L);
  int hf = 0;
  RG_HIP(hipMemcpyAsync(hn.data(), nrm, hn.size() * 8, hipMemcpyDeviceToHost, st));
  RG_HIP(hipMemcpyAsync(he.data(), ev.p, he.size() * 8, hipMemcpyDeviceToHost, st));
  RG_HIP(hipMemcpyAsync(&hf, flag.p, sizeof(int), hipMemcpyDeviceToHost, st));
  RG_HIP(hipStreamSynchronize(st));
  memset(res, 0, sizeof(*res));
  for (long long i = 0; i < n_out; ++i) {
    uint32_t c = 0;
    for (int w = 0; w < kNormW; ++w) {
      const unsigned __int128 t = (unsigned __int128)res->outer_norm_sq[w] + hn[i * kNormW + w] + c;
      res->outer_norm_sq[w] = (uint64_t)t;
      c = (uint32_t)(t >> 64);
    }
  }
  for (long long i = n_out; i < n_out + n_in; ++i) {
    uint32_t c = 0;
    for (int w = 0; w < kNormW; ++w) {
      const unsigned __int128 t = (unsigned __int128)res->inner_norm_sq[w] + hn[i * kNormW + w] + c;
      res->inner_norm_sq[w] = (uint64_t)t;
      c = (uint32_t)(t >> 64);
    }
  }
  res->outer_ok = norm_below(res->outer_norm_sq, in_com_dcmp_two_nm);
  res->inner_ok = norm_below(res->inner_norm_sq, res_two_nm);
  res->consistency_ok = hf == 0;
  memcpy(res->eval_lhs, he.data(), 8 * L);
  if (batch > 1) {
    memcpy(res->eval_rhs, he.data() + L, 8 * L);
  } else {
    RG_HIP(hipMemcpy(res->eval_rhs, d_y, 8 * L, hipMemcpyDeviceToHost));
  }
  res->eval_ok = memcmp(res->eval_lhs, res->eval_rhs, 8 * L) == 0;
  res->ok = res->outer_ok && res->inner_ok && res->consistency_ok && res->eval_ok;
  return RG_OK;
}

static rg_status jindo_new(const rg_jindo_params* p, rg_jindo** out, rg_jindo** J) {
  if (!out) return RG_ERR_INVALID;
  *out = nullptr;
  RG_TRY(validate(p));
  *J = new rg_jindo();
  (*J)->p = *p;
  if (hipGetDevice(&(*J)->device) != hipSuccess) (*J)->device = 0;
  rg_status s = build(*J);
  if (s != RG_OK) {
    delete *J;
    *J = nullptr;
  }
  return s;
}

// The commit key is device-resident from here on: ck_in/ck_mlwe/ck_out hold it in the
// entities.go layouts; the MAC kernels' key images (the MFMA MAC's digits
// words) are built from them on the device, only for the MAC each product runs on.
static rg_status finish_ck(rg_jindo* J, hipStream_t st) {
  const rg_jindo_params& p = J->p;
  // RINGO_JINDO_MAC (experiments build): l = mac_kernel; default = the MFMA MAC where it applies,
  // else mac_kernel
  const char* mk = knob(Knob::JindoMac);
  const bool legacy = mk && mk[0] == 'l';
  const bool no_mfma = legacy;
  const size_t pcq = (size_t)p.nq * p.d, pco = (size_t)p.nqo * p.d;
  {
    uint64_t pq[kMaxQ], po[kMaxQ];
    MfmaPrime mq[kMaxQ], mo[kMaxQ];
    for (int l = 0; l < p.nq; ++l) pq[l] = J->rq[l].q, mq[l] = mfma_prime(J->rq[l]);
    for (int l = 0; l < p.nqo; ++l) po[l] = J->ro[l].q, mo[l] = mfma_prime(J->ro[l]);
    J->mfma_q = no_mfma ? 0 : mac_mfma_nb(pq, p.nq, p.in_msis, p.rows + p.mlwe, p.d);
    J->mfma_o = no_mfma ? 0 : mac_mfma_nb(po, p.nqo, p.out_msis, p.dcmp, p.d);
    if (J->mfma_q)
      RG_TRY(mac_mfma_key_dev(J->ck_in.as<uint64_t>(), p.rows, J->ck_mlwe.as<uint64_t>(), p.mlwe, p.in_msis,
                              (long long)pcq, p.d, J->mfma_q, mq, p.nq, J->ckm_in, st));
    if (J->mfma_o)
      RG_TRY(mac_mfma_key_dev(J->ck_out.as<uint64_t>(), p.dcmp, nullptr, 0, p.out_msis, (long long)pco, p.d,
                              J->mfma_o, mo, p.nqo, J->ckm_out, st));
  }
  RG_HIP(hipStreamSynchronize(st));
  return RG_OK;
}

// ck_* host (kind = H2D) or device (kind = D2D) arrays -> the handle's device buffers
static rg_status take_ck(rg_jindo* J, const uint64_t* ck_in, const uint64_t* ck_mlwe, const uint64_t* ck_out,
                         hipMemcpyKind kind, hipStream_t st) {
  size_t a, b, c;
  ck_sizes(J->p, &a, &b, &c);
  RG_TRY(J->ck_in.alloc(a * 8));
  RG_TRY(J->ck_mlwe.alloc(b * 8));
  RG_TRY(J->ck_out.alloc(c * 8));
  RG_HIP(hipMemcpyAsync(J->ck_in.p, ck_in, a * 8, kind, st));
  if (b) RG_HIP(hipMemcpyAsync(J->ck_mlwe.p, ck_mlwe, b * 8, kind, st));
  RG_HIP(hipMemcpyAsync(J->ck_out.p, ck_out, c * 8, kind, st));
  return finish_ck(J, st);
}

rg_status rg_jindo_create(const rg_jindo_params* p, const uint64_t* ck_in, const uint64_t* ck_mlwe,
                          const uint64_t* ck_out, rg_jindo** out) {
  if (!ck_in || !ck_out || (!ck_mlwe && p && p->mlwe)) return RG_ERR_INVALID;
  rg_jindo* J = nullptr;
  RG_TRY(jindo_new(p, out, &J));
  rg_status s = take_ck(J, ck_in, ck_mlwe, ck_out, hipMemcpyHostToDevice, nullptr);
  if (s != RG_OK) {
    delete J;
    return s;
  }
  *out = J;
  return RG_OK;
}

rg_status rg_jindo_create_dev(const rg_jindo_params* p, const uint64_t* d_ck_in, const uint64_t* d_ck_mlwe,
                              const uint64_t* d_ck_out, void* stream, rg_jindo** out) {
  if (!d_ck_in || !d_ck_out || (!d_ck_mlwe && p && p->mlwe)) return RG_ERR_INVALID;
  rg_jindo* J = nullptr;
  RG_TRY(jindo_new(p, out, &J));
  rg_status s = take_ck(J, d_ck_in, d_ck_mlwe, d_ck_out, hipMemcpyDeviceToDevice, as_stream(stream));
  if (s != RG_OK) {
    delete J;
    return s;
  }
  *out = J;
  return RG_OK;
}

rg_status rg_jindo_create_from_crs(const rg_jindo_params* p, const uint8_t* crs, size_t crs_len, rg_jindo** out) {
  if (!crs && crs_len) return RG_ERR_INVALID;
  rg_jindo* J = nullptr;
  RG_TRY(jindo_new(p, out, &J));
  const rg_jindo_params& P = J->p;
  CtrStream u(crs, crs_len);
  if (!u.ok) {
    delete J;
    set_last_error("libcrypto (SHA384/AES-256-CTR) unavailable");
    return RG_ERR_UNSUPPORTED;
  }
  size_t a, b, c;
  ck_sizes(P, &a, &b, &c);
  std::vector<uint64_t> h_in(a), h_ml(b), h_out(c);
  const size_t d = P.d;
  // entities.go:24-61: In, then MLWE, then Out; coefficient-major, limb-minor draws
  for (int i = 0; i < P.in_msis; ++i)
    for (int j = 0; j < P.rows; ++j)
      for (size_t k = 0; k < d; ++k)
        for (int l = 0; l < P.nq; ++l) h_in[(((size_t)i * P.rows + j) * P.nq + l) * d + k] = u.sample_n(P.q[l]);
  for (int i = 0; i < P.in_msis; ++i)
    for (int j = 0; j < P.mlwe; ++j)
      for (size_t k = 0; k < d; ++k)
        for (int l = 0; l < P.nq; ++l) h_ml[(((size_t)i * P.mlwe + j) * P.nq + l) * d + k] = u.sample_n(P.q[l]);
  for (int i = 0; i < P.out_msis; ++i)
    for (int j = 0; j < P.dcmp; ++j)
      for (size_t k = 0; k < d; ++k)
        for (int l = 0; l < P.nqo; ++l) h_out[(((size_t)i * P.dcmp + j) * P.nqo + l) * d + k] = u.sample_n(P.qo[l]);
  rg_status s = take_ck(J, h_in.data(), h_ml.data(), h_out.data(), hipMemcpyHostToDevice, nullptr);
  if (s != RG_OK) {
    delete J;
    return s;
  }
  *out = J;
  return RG_OK;
}

void rg_jindo_destroy(rg_jindo* j) {
  if (j) (void)hipDeviceSynchronize();  // scratch may still be in use by queued commits
  delete j;
}

rg_status rg_jindo_commit_key(const rg_jindo* J, uint64_t* ck_in, uint64_t* ck_mlwe, uint64_t* ck_out) {
  if (!J) return RG_ERR_INVALID;
  size_t a, b, c;
  ck_sizes(J->p, &a, &b, &c);
  if (ck_in) RG_HIP(hipMemcpy(ck_in, J->ck_in.p, a * 8, hipMemcpyDeviceToHost));
  if (ck_mlwe && b) RG_HIP(hipMemcpy(ck_mlwe, J->ck_mlwe.p, b * 8, hipMemcpyDeviceToHost));
  if (ck_out) RG_HIP(hipMemcpy(ck_out, J->ck_out.p, c * 8, hipMemcpyDeviceToHost));
  return RG_OK;
}

rg_status rg_jindo_commit_key_dev(const rg_jindo* J, const uint64_t** d_ck_in, const uint64_t** d_ck_mlwe,
                                  const uint64_t** d_ck_out) {
  if (!J) return RG_ERR_INVALID;
  if (d_ck_in) *d_ck_in = J->ck_in.as<const uint64_t>();
  if (d_ck_mlwe) *d_ck_mlwe = J->ck_mlwe.as<const uint64_t>();
  if (d_ck_out) *d_ck_out = J->ck_out.as<const uint64_t>();
  return RG_OK;
}

size_t rg_jindo_scratch_bytes(const rg_jindo* J, size_t batch) {
  if (!J) return 0;
  const rg_jindo_params& p = J->p;
  const size_t d = p.d;
  return batch * (p.cols + 1) * p.rows * d * 4 + batch * (p.cols + 1) * p.in_msis * p.nq * d * 8 +
         batch * p.out_msis * p.nqo * d * 8;
}

rg_status rg_jindo_commit_dev(const rg_jindo* J, size_t batch, const uint64_t* d_v, size_t nv, const uint64_t* d_last,
                              const uint64_t* d_mask, const int64_t* d_en, const int64_t* d_mn, uint64_t* d_incom,
                              uint64_t* d_enc, uint64_t* d_mlwe, uint64_t* d_com, void* stream) {
  if (!J) return RG_ERR_INVALID;
  if (batch && (!d_v || !d_last || !d_mask || !d_en || !d_mn || !d_incom || !d_enc || !d_mlwe || !d_com))
    return RG_ERR_INVALID;
  return commit_dev(const_cast<rg_jindo*>(J), batch, d_v, nv, d_last, d_mask, d_en, d_mn, d_incom, d_enc, d_mlwe, d_com,
                    as_stream(stream));
}

rg_status rg_jindo_commit_core_dev(const rg_jindo* J, size_t batch, const uint64_t* d_enc, const uint64_t* d_mlwe,
                                   uint64_t* d_incom, uint64_t* d_com, void* stream) {
  if (!J) return RG_ERR_INVALID;
  if (batch == 0) return RG_OK;
  if (!d_enc || !d_mlwe || !d_incom || !d_com) return RG_ERR_INVALID;
  RG_TRY(on_device(J));
  rg_jindo* Jm = const_cast<rg_jindo*>(J);
  hipStream_t st = as_stream(stream);
  rg_jindo_scratch* sc = nullptr;
  RG_TRY(stream_scratch(Jm, batch, st, &sc));
  return commit_core(Jm, batch, d_enc, d_mlwe, d_incom, d_com, sc, st);
}

rg_status rg_jindo_commit_core(const rg_jindo* J, const uint64_t* enc, const uint64_t* mlwe, uint64_t* o_incom,
                               uint64_t* o_com) {
  if (!J || !enc || !mlwe || !o_incom || !o_com) return RG_ERR_INVALID;
  const rg_jindo_params& p = J->p;
  const size_t d = p.d, nm = p.in_msis + p.mlwe;
  const size_t b_enc = (size_t)(p.cols + 1) * p.rows * p.nq * d * 8, b_ml = (size_t)(p.cols + 1) * nm * p.nq * d * 8;
  const size_t b_inc = (size_t)p.dcmp * p.nqo * d * 8, b_com = (size_t)p.out_msis * p.nq * d * 8;
  DevBuf enc_, ml_, inc_, com_;
  RG_TRY(enc_.upload(enc, b_enc));
  RG_TRY(ml_.upload(mlwe, b_ml));
  RG_TRY(inc_.alloc(b_inc));
  RG_TRY(com_.alloc(b_com));
  RG_TRY(rg_jindo_commit_core_dev(J, 1, enc_.as<uint64_t>(), ml_.as<uint64_t>(), inc_.as<uint64_t>(),
                                  com_.as<uint64_t>(), nullptr));
  RG_HIP(hipMemcpy(o_incom, inc_.p, b_inc, hipMemcpyDeviceToHost));
  RG_HIP(hipMemcpy(o_com, com_.p, b_com, hipMemcpyDeviceToHost));
  return RG_OK;
}

rg_status rg_jindo_commit(const rg_jindo* J, const uint64_t* v, size_t nv, const uint64_t* last_row,
                          const uint64_t* mask, const int64_t* enc_noise, const int64_t* mlwe_noise, uint64_t* o_incom,
                          uint64_t* o_enc, uint64_t* o_mlwe, uint64_t* o_com) {
  if (!J || !v || !last_row || !mask || !enc_noise || !mlwe_noise || !o_incom || !o_enc || !o_mlwe || !o_com)
    return RG_ERR_INVALID;
  const rg_jindo_params& p = J->p;
  if (nv < 1 || nv > (size_t)p.rank) return RG_ERR_RANK;
  const size_t L = p.field_limbs, d = p.d, nm = p.in_msis + p.mlwe;
  const size_t b_v = nv * L * 8, b_last = (size_t)p.cols * p.slots * L * 8, b_mask = (size_t)p.rows * p.slots * L * 8;
  const size_t b_en = (size_t)(p.cols + 1) * p.rows * d * 8, b_mn = (size_t)(p.cols + 1) * nm * d * 8;
  const size_t b_inc = (size_t)p.dcmp * p.nqo * d * 8, b_enc = (size_t)(p.cols + 1) * p.rows * p.nq * d * 8;
  const size_t b_ml = (size_t)(p.cols + 1) * nm * p.nq * d * 8, b_com = (size_t)p.out_msis * p.nq * d * 8;
  DevBuf v_, l_, m_, en_, mn_, inc_, enc_, ml_, com_;
  RG_TRY(v_.upload(v, b_v));
  RG_TRY(l_.upload(last_row, b_last));
  RG_TRY(m_.upload(mask, b_mask));
  RG_TRY(en_.upload(enc_noise, b_en));
  RG_TRY(mn_.upload(mlwe_noise, b_mn));
  RG_TRY(inc_.alloc(b_inc));
  RG_TRY(enc_.alloc(b_enc));
  RG_TRY(ml_.alloc(b_ml));
  RG_TRY(com_.alloc(b_com));
  RG_TRY(rg_jindo_commit_dev(J, 1, v_.as<uint64_t>(), nv, l_.as<uint64_t>(), m_.as<uint64_t>(), en_.as<int64_t>(),
                             mn_.as<int64_t>(), inc_.as<uint64_t>(), enc_.as<uint64_t>(), ml_.as<uint64_t>(),
                             com_.as<uint64_t>(), nullptr));
  RG_HIP(hipMemcpy(o_incom, inc_.p, b_inc, hipMemcpyDeviceToHost));
  RG_HIP(hipMemcpy(o_enc, enc_.p, b_enc, hipMemcpyDeviceToHost));
  RG_HIP(hipMemcpy(o_mlwe, ml_.p, b_ml, hipMemcpyDeviceToHost));
  RG_HIP(hipMemcpy(o_com, com_.p, b_com, hipMemcpyDeviceToHost));
  return RG_OK;
}

rg_status rg_jindo_set_stddevs(rg_jindo* J, const rg_jindo_stddevs* sd) {
  if (!J || !sd) return RG_ERR_INVALID;
  const double v[6] = {sd->ecd, sd->ecd_blind, sd->mask, sd->mask_blind, sd->mlwe, sd->mask_mlwe};
  for (double x : v)
    if (!(x > 0.0) || !std::isfinite(x)) return RG_ERR_INVALID;  // RoundedGaussianSampler panics on <= 0
  rg_jindo_samplers& S = J->smp;
  std::lock_guard<std::mutex> lk(J->mu);
  S.ready = false;
  memcpy(S.sd, v, sizeof(v));
  uint32_t te0[256];
  aes_te0(te0);
  RG_TRY(S.te0.upload(te0, sizeof(te0)));
  // Encoder.twinCDT: 128 centre tables at ecdStdDev (twin_cdt.go:48-58); Prover.mlweSampler:
  // the same at mlweStdDev, of which Sample(0) reads table 0
  std::vector<uint64_t> enc, ml;
  for (int c = 0; c < 128; ++c) {
    const std::vector<uint64_t> t = compute_cdt((double)c / 128.0, v[0]);
    enc.insert(enc.end(), t.begin(), t.end());
    S.cdt_enc_size = (int)t.size();
  }
  ml = compute_cdt(0.0, v[4]);
  S.cdt_mlwe_size = (int)ml.size();
  S.tail_lo_enc = -(int64_t)std::ceil(9.0 * v[0]);
  S.tail_lo_mlwe = -(int64_t)std::ceil(9.0 * v[4]);
  RG_TRY(S.cdt_enc.upload(enc.data(), enc.size() * 8));
  if (S.cdt_enc_size <= 255) {  // guide: per table, lower_bound of t * 2^56 for t = 0..256
    std::vector<uint8_t> guide(128 * 257);
    for (int c = 0; c < 128; ++c) {
      const uint64_t* t = enc.data() + (size_t)c * S.cdt_enc_size;
      for (int b = 0; b <= 256; ++b) {
        int i = 0;
        if (b == 256)
          i = S.cdt_enc_size;
        else
          while (i < S.cdt_enc_size && t[i] < ((uint64_t)b << 56)) ++i;
        guide[c * 257 + b] = (uint8_t)i;
      }
    }
    RG_TRY(S.cdt_guide.upload(guide.data(), guide.size()));
  }
  {  // cdt2's tail bounds: the reference's tail cdf (twin_cdt.go:101-105) at centres c / 128, c = 0..128
    const int n = S.cdt_enc_size;
    const double sigma = v[0], norm = std::sqrt(2.0 * M_PI) * sigma;
    std::vector<double> sb((size_t)129 * (n + 2));
    for (int c = 0; c <= 128; ++c) {
      const double cf = (double)c / 128.0;
      double cdf = 0.0;
      int64_t x = S.tail_lo_enc;
      for (int j = -1; j <= n; ++j) {  // entry j + 1: sum over x = tailLo .. j
        for (; x <= j; ++x) {
          const double xf = (double)x;
          cdf += std::exp(-(xf - cf) * (xf - cf) / (2.0 * sigma * sigma)) / norm;
        }
        sb[(size_t)c * (n + 2) + j + 1] = cdf;
      }
    }
    RG_TRY(S.cdt_sbound.upload(sb.data(), sb.size() * 8));
    // jmax[c]: the largest J with, for every v0 = j in [-1, J] of table c, the bound on p
    // (t_c[j + 1] / 2^64, or 1 past the table) below the smallest cdf the reference can compare it
    // with (S[c + 1][j] (1 - 2^-40)), again shrunk by 2^-40 for the double rounding of p
    std::vector<int> jm(128);
    for (int c = 0; c < 128; ++c) {
      const uint64_t* t = enc.data() + (size_t)c * n;
      int J = -2;
      for (int j = -1; j <= n; ++j) {
        const double pu = (j + 1 < n ? (double)t[j + 1] / 18446744073709551616.0 : 1.0) * (1.0 + 9.094947017729282e-13);
        if (!(pu < sb[(size_t)(c + 1) * (n + 2) + j + 1] * (1.0 - 9.094947017729282e-13))) break;
        J = j;
      }
      jm[c] = J;
    }
    RG_TRY(S.cdt_jmax.upload(jm.data(), jm.size() * 4));
  }
  RG_TRY(S.cdt_mlwe.upload(ml.data(), ml.size() * 8));
  const Ziggurat Z = make_ziggurat();
  std::vector<uint64_t> zg(384);
  memcpy(zg.data(), Z.kn, 128 * 8);
  memcpy(zg.data() + 128, Z.wn, 128 * 8);
  memcpy(zg.data() + 256, Z.fn, 128 * 8);
  RG_TRY(S.zig.upload(zg.data(), zg.size() * 8));
  S.h_delta = compute_delta_inv(J->p.base, J->p.exp);
  RG_TRY(S.delta.upload(S.h_delta.data(), S.h_delta.size() * 8));
  S.ready = true;
  return RG_OK;
}

rg_status rg_jindo_delta_inv(const rg_jindo* J, double* out) {
  if (!J || !out) return RG_ERR_INVALID;
  const std::vector<double> d = compute_delta_inv(J->p.base, J->p.exp);
  memcpy(out, d.data(), d.size() * 8);
  return RG_OK;
}

// Every sampler instance of commits [first, first + batch) must have a u64 number (so that no two
// instances share a window; csprng.hpp ks_words): the largest per-commit count of a domain is
// (cols+1) rows d (COSAC, per sample), (cols+1) (in_msis+mlwe) d (rounded MLWE, per sample) or
// (cols + rows) slots (MustSetRandom, per element).
static rg_status instances_in_range(const rg_jindo* J, unsigned long long first, size_t batch) {
  const rg_jindo_params& p = J->p;
  const unsigned __int128 per_enc = (unsigned __int128)(p.cols + 1) * p.rows * p.d;
  const unsigned __int128 per_ml = (unsigned __int128)(p.cols + 1) * (p.in_msis + p.mlwe) * p.d;
  const unsigned __int128 per_uni = (unsigned __int128)(p.cols + p.rows) * p.slots;
  const unsigned __int128 per = std::max(per_enc, std::max(per_ml, per_uni));
  const unsigned __int128 end = (unsigned __int128)first + batch;
  if (end > ((unsigned __int128)1 << 64) / per) {
    set_last_error("first_commit + batch: sampler instance numbers would exceed 2^64");
    return RG_ERR_INVALID;
  }
  return RG_OK;
}

rg_status rg_jindo_sample_dev(const rg_jindo* J, size_t batch, const uint64_t* d_v, size_t nv,
                              const rg_jindo_seeds* seeds, unsigned long long first_commit, uint64_t* d_last_row,
                              uint64_t* d_mask, int64_t* d_enc_noise, int64_t* d_mlwe_noise, void* stream) {
  if (!J || !seeds) return RG_ERR_INVALID;
  if (nv < 1 || nv > (size_t)J->p.rank) return RG_ERR_RANK;
  RG_TRY(instances_in_range(J, first_commit, batch));
  if (batch == 0) return RG_OK;
  if (!d_v || !d_last_row || !d_mask || !d_enc_noise || !d_mlwe_noise) return RG_ERR_INVALID;
  RG_TRY(on_device(J));
  rg_jindo* Jm = const_cast<rg_jindo*>(J);
  hipStream_t st = as_stream(stream);
  rg_jindo_scratch* sc = nullptr;
  RG_TRY(stream_scratch(Jm, batch, st, &sc));
  return sample_stage(Jm, batch, d_v, nv, seeds, first_commit, d_last_row, d_mask, d_enc_noise, d_mlwe_noise,
                      sc->digits.as<uint32_t>(), sc, st);
}

rg_status rg_jindo_commit_sampled_dev(const rg_jindo* J, size_t batch, const uint64_t* d_v, size_t nv,
                                      const rg_jindo_seeds* seeds, unsigned long long first_commit, uint64_t* d_incom,
                                      uint64_t* d_enc, uint64_t* d_mlwe, uint64_t* d_com, void* stream) {
  if (!J || !seeds) return RG_ERR_INVALID;
  if (nv < 1 || nv > (size_t)J->p.rank) return RG_ERR_RANK;
  RG_TRY(instances_in_range(J, first_commit, batch));
  if (batch == 0) return RG_OK;
  if (!d_v || !d_incom || !d_enc || !d_mlwe || !d_com) return RG_ERR_INVALID;
  RG_TRY(on_device(J));
  rg_jindo* Jm = const_cast<rg_jindo*>(J);
  hipStream_t st = as_stream(stream);
  rg_jindo_scratch* sc = nullptr;
  RG_TRY(stream_scratch(Jm, batch, st, &sc));
  RG_TRY(sample_scratch(Jm, batch, sc, st));
  uint32_t* digits = sc->digits.as<uint32_t>();
  int64_t *en = sc->en.as<int64_t>(), *mn = sc->mn.as<int64_t>();
  // The batch as one DAG over three streams (the caller's st and two helpers of this caller
  // stream), so that each sampler's tail overlaps other work instead of idling the chip:
  //   st:   MustSetRandom -> digits -> cdt2 (TwinCDT) ...................... -> prep(encode) -> core
  //   s[0]:                    (digits) -> COSAC centres -> cosac2 ----------^
  //   s[1]: mlwe samplers -> prep(MLWE) -------------------------------------^
  // Results do not depend on the schedule: every sampler instance is numbered per commit, and
  // each buffer has one writer ordered before its readers by the events.
  static const bool one_stream = [] {  // RINGO_JINDO_SPLIT=0: everything on st (per-kernel profiling)
    const char* e = knob(Knob::JindoSplit);
    return e && e[0] == '0';
  }();
  rg_jindo::Aux* ax = nullptr;
  if (!one_stream) {
    std::lock_guard<std::mutex> lk(Jm->mu);
    rg_jindo::Aux& x = Jm->aux[st];
    for (hipStream_t& s : x.s)
      if (!s) RG_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (hipEvent_t& e : x.e)
      if (!e) RG_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ax = &x;
  }
  hipStream_t s_cos = ax ? ax->s[0] : st, s_ml = ax ? ax->s[1] : st;
  rg_status s = sample_stage(Jm, batch, d_v, nv, seeds, first_commit, sc->last.as<uint64_t>(), sc->mask.as<uint64_t>(),
                             en, mn, digits, sc, st, s_cos, s_ml, ax ? ax->e[0] : nullptr, ax ? ax->e[1] : nullptr);
  if (s == RG_OK) s = prep_launch(Jm, batch, nv, digits, en, mn, d_enc, d_mlwe, kPrepMlwe, s_ml);
  // (the TwinCDT rows' prep right behind cdt2, beside cosac2, measured no faster: r05i)
  if (ax) {
    // join: the encode prep needs both samplers' noise; the core needs the MLWE prep.  Joined on
    // every exit path, so that after a failed launch the caller's stream still orders whatever
    // helper work was queued before this handle's scratch (wq, en, mn) is reused; the first error
    // is the one returned
    const hipError_t j[4] = {hipEventRecord(ax->e[2], s_cos), hipEventRecord(ax->e[3], s_ml),
                             hipStreamWaitEvent(st, ax->e[2], 0), hipStreamWaitEvent(st, ax->e[3], 0)};
    for (hipError_t e : j)
      if (e != hipSuccess && s == RG_OK) {
        set_last_error(std::string("jindo sampled commit: joining the helper streams: ") + hipGetErrorString(e));
        s = RG_ERR_DEVICE;
      }
  }
  RG_TRY(s);
  RG_TRY(prep_launch(Jm, batch, nv, digits, en, mn, d_enc, d_mlwe, kPrepEnc, st));
  return commit_core(Jm, batch, d_enc, d_mlwe, d_incom, d_com, sc, st);
}

rg_status rg_jindo_release_stream(rg_jindo* J, void* stream) {
  if (!J) return RG_ERR_INVALID;
  RG_TRY(on_device(J));
  hipStream_t st = as_stream(stream);
  std::lock_guard<std::mutex> lk(J->mu);
  RG_HIP(hipStreamSynchronize(st));
  auto a = J->aux.find(st);
  if (a != J->aux.end()) {
    for (hipStream_t x : a->second.s)
      if (x) {
        RG_HIP(hipStreamSynchronize(x));
        J->scratch.erase(x);
        (void)hipStreamDestroy(x);
      }
    for (hipEvent_t x : a->second.e)
      if (x) (void)hipEventDestroy(x);
    J->aux.erase(a);
  }
  J->scratch.erase(st);
  return RG_OK;
}

rg_status rg_jindo_mac_kinds(const rg_jindo* J, int* inner, int* outer) {
  if (!J || !inner || !outer) return RG_ERR_INVALID;
  *inner = J->mfma_q ? RG_MAC_MFMA : RG_MAC_GENERIC;
  *outer = J->mfma_o ? RG_MAC_MFMA : RG_MAC_GENERIC;
  return RG_OK;
}

rg_status rg_uniform_words_dev(const uint8_t* seed, size_t seed_len, unsigned long long instance,
                               unsigned long long first_word, size_t n, uint64_t* d_out, void* stream) {
  if ((!seed && seed_len) || (!d_out && n)) return RG_ERR_INVALID;
  if (n == 0) return RG_OK;
  uint8_t r[48];
  if (!sha384(seed, seed_len, r)) {
    set_last_error("libcrypto SHA384 unavailable");
    return RG_ERR_UNSUPPORTED;
  }
  AesKey K;
  aes256_expand(r, K.rk);
  for (int w = 0; w < 4; ++w)
    K.iv[w] = ((uint32_t)r[32 + 4 * w] << 24) | ((uint32_t)r[33 + 4 * w] << 16) | ((uint32_t)r[34 + 4 * w] << 8) |
              r[35 + 4 * w];
  uint32_t te0[256];
  aes_te0(te0);
  DevBuf t;
  RG_TRY(t.upload(te0, sizeof(te0)));
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(uniform_words_kernel, dim3((unsigned)((n + 511) / 512)), dim3(512), 0, st, K, t.as<uint32_t>(),
                     instance, first_word, (long long)n, d_out);
  RG_TRY(check_launch("uniform words"));
  RG_HIP(hipStreamSynchronize(st));  // `t` is freed on return
  return RG_OK;
}

rg_status rg_jindo_eval_reduce_dev(const rg_jindo* J, uint64_t* d_ob_incom, uint64_t* d_ob_enc, uint64_t* d_ob_mlwe,
                                   void* stream) {
  if (!J || !d_ob_incom || !d_ob_enc || !d_ob_mlwe) return RG_ERR_INVALID;
  const rg_jindo_params& p = J->p;
  hipStream_t st = as_stream(stream);
  const long long nm = p.in_msis + p.mlwe, n_enc = (long long)(p.cols + 1) * p.rows, n_ml = (long long)(p.cols + 1) * nm;
  const RingDev rq = ring_dev(J->rq, p.nq, J->rootsq_f, J->rootsq_b), ro = ring_dev(J->ro, p.nqo, J->rootso_f, J->rootso_b);
  auto go = [&](uint64_t* x, long long npoly, int nl, const RingDev& R) {
    const long long n = npoly * nl * p.d;
    hipLaunchKernelGGL(rns_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, npoly, nl, p.d, R);
    return check_launch("jindo eval reduce");
  };
  RG_TRY(go(d_ob_incom, p.dcmp, p.nqo, ro));
  RG_TRY(go(d_ob_enc, n_enc, p.nq, rq));
  return go(d_ob_mlwe, n_ml, p.nq, rq);
}

}  // extern "C"
