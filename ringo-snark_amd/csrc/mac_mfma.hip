// mac_mfma.hip -- the Jindo Ajtai multiply-accumulate on the gfx950 matrix cores.
//
// Per (limb, coefficient) lk the inner commitment (prover.go:149-157) and the outer one
// (prover.go:180-191) are a modular GEMM over the commit key A (J x T, Montgomery words):
//     out[col][j][lk] = (sum_t A[j][t][lk] B[col][t][lk]) 2^-64 mod q   (+ C, the MLWE term)
// (the summed MulCoeffsMontgomeryThenAdd of the reference, mac3h_kernel's semantics).
//
// Exact integer products on v_mfma_i32_16x16x64_i8.  A residue x < q < 2^(8 NB - 2) is written in
// NB signed base-256 digits.  The key uses balanced digits a_0 .. a_{NB-1} in [-128, 127] (an
// exact representation, computed once per prover); an opening word b uses its own bytes with
// bytes 0 .. NB-2 offset by -128 (b XOR bxor read as signed int8), i.e. the digits of
// b' = b - bxor.  The product sum splits into 2 NB - 1 diagonals
//     D_s[j][col] = sum_t sum_{a + b = s} a_a[j][t] b'_b[t][col]
// and ONE MFMA per diagonal and 8-term chunk computes D_s with its K = 64 running over
// (term, digit b) pairs: lane l of the wave holds, as the B operand, the raw 16 bytes of
// b'[t][col] for t = 2 (l >> 4) + {0, 1}, col = l & 15, and as the A operand the digits
// a_{s - b}[j][t] (j = l & 15) in the same byte positions.  Held byte-reversed (R), the key word
// of a term becomes that A operand by ONE 64-bit shift per diagonal (R >> 8(NB-1-s) or
// R << 8(s-NB+1)); bytes outside 0 .. NB-1 meet zero bytes of b'.  Then
//     sum_t A b = sum_s D_s 256^s + bxor sum_t A[j][t]
// whose second term is a per-(lk, j) constant (`corr`, with the 2^-64 folded in).  The diagonal
// sums are int32-exact while T NB 2^14 < 2^31.
//
// Workgroup = 16 lk (one 128-B line of each opening row) x 16 columns, 16 waves, wave w = lk0 + w.
// The opening (HBM) and the key chunks (1 KiB per wave, from L2) stream into LDS by LDS-DMA
// (global_load_lds_dwordx4), one 32-KiB stage per 8-term chunk in a ring of kMfmaStages, counted
// vmcnt waits and a raw s_barrier per chunk (the compiler sees none of these loads).  Blocks are mapped XCD-major, so an XCD's CUs work through the
// column tiles of one lk group together and share its key in their L2.  After the last chunk
// every lane folds its 4 outputs (rows 4 (l >> 4) + r, column l & 15) from the 2 NB - 1
// diagonals into one residue and the workgroup writes 128-B rows through LDS.
#include <algorithm>
#include <cmath>

#include "field.hpp"
#include "mac_mfma.hpp"

namespace rg {

typedef int mfma_v4i __attribute__((ext_vector_type(4)));

constexpr int kMfmaStages = 4;  // LDS ring depth (3 / 4 / 5 measured within 1%, round 4)
constexpr int kMfmaLk = 16;     // lk per workgroup: 16 (1024 threads, one 128-B line); 8 (512 threads,
                                // 2 per CU) measured 30% slower

__device__ __forceinline__ void mfma_glds16(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_dst)
      : "memory");
}
template <int N>
__device__ __forceinline__ void mfma_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LK lk x 16 columns per workgroup, wave w = lk0 + w.  Stage image (u64 words): the opening
// [t 8][lk pair LK/2][col 16][2] (LK KiB), then the waves' key chunks [w][64 lanes][2] (LK KiB).
template <int NB, int LK>
__global__ __launch_bounds__(64 * LK, 16 / LK) void mac_mfma_kernel(MfmaMacArgs a) {
  constexpr int ND = 2 * NB - 1;      // diagonals
  constexpr int NP = LK / 2;          // lk pairs
  constexpr int BW = 8 * NP * 16 * 2;  // opening words per stage
  constexpr int SW = BW + LK * 128;    // stage words
  static_assert(16 * 16 * LK <= kMfmaStages * SW, "output stage must fit the ring");
  __shared__ uint64_t ring[kMfmaStages * SW];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const long long nct = (a.ncols + 15) / 16;
  unsigned g = blockIdx.x;
  if ((gridDim.x & 7) == 0) g = (g & 7) * (gridDim.x >> 3) + (g >> 3);  // XCD-major
  const long long lk0 = (long long)(g / nct) * LK, c0 = (long long)(g % nct) * 16;
  const int T = a.T1 + a.T2, Tc = a.Tc;
  const uint32_t ring_lds = (uint32_t)(uintptr_t)ring;
  // the lane's opening chunk of every stage: position w * 64 + lane of [t][lk pair][col]
  constexpr int PW = NP * 16;  // chunks per term
  const int dpos = w * 64 + lane, dt = dpos / PW, dp = (dpos % PW) >> 4, dcol = lane & 15;
  const long long dc = std::min<long long>(c0 + dcol, a.ncols - 1);
  // the wave's key chunk (1 KiB of [lk][chunk][64 lanes][2]): the lane's own 16 B
  const uint64_t* akey = a.Ak + (lk0 + w) * Tc * 128 + 2 * lane;
  // stage `chunk`: 2 LDS-DMAs per wave (16 B of opening, 16 B of key per lane); past the last
  // chunk they reload valid addresses into a free stage, so every iteration issues the same count
  auto stage = [&](int chunk) {
    int t = chunk * 8 + dt;
    if (t >= T) t = T - 1;  // the key's padded terms are zero
    const uint64_t* src = t < a.T1 ? a.B1 + dc * a.b1_col + (long long)t * a.b1_term
                                   : a.B2 + dc * a.b2_col + (long long)(t - a.T1) * a.b2_term;
    const uint32_t base = ring_lds + (uint32_t)((chunk % kMfmaStages) * SW) * 8u;
    mfma_glds16(src + lk0 + 2 * dp, base + (uint32_t)(w * 128) * 8u);
    mfma_glds16(akey + (long long)std::min(chunk, Tc - 1) * 128, base + (uint32_t)(BW + w * 128) * 8u);
  };
  mfma_v4i acc[ND];
#pragma unroll
  for (int s = 0; s < ND; ++s) acc[s] = mfma_v4i{0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < kMfmaStages - 1; ++k) stage(k);
  // LDS words of the lane's two opening values: terms 2 (lane >> 4) + {0, 1}, lk = lk0 + w
  // (pair w >> 1, half w & 1), column lane & 15
  const int rd = ((2 * (lane >> 4) * NP + (w >> 1)) * 16 + (lane & 15)) * 2 + (w & 1);
  for (int c = 0; c < Tc; ++c) {
    mfma_wait_vm<2 * (kMfmaStages - 2)>();  // stage c landed (stages c+1 .. c+S-2 may be in flight)
    __builtin_amdgcn_s_barrier();           // ... for every wave; stage c - 1 is free
    stage(c + kMfmaStages - 1);
    const uint64_t* st = ring + (c % kMfmaStages) * SW;
    const uint64_t b0 = st[rd] ^ a.bxor, b1 = st[rd + NP * 32] ^ a.bxor;  // + NP 32 words: term + 1
    const ulonglong2 ak = *reinterpret_cast<const ulonglong2*>(st + BW + w * 128 + 2 * lane);
    mfma_v4i bv;
    bv[0] = (int)(uint32_t)b0;
    bv[1] = (int)(uint32_t)(b0 >> 32);
    bv[2] = (int)(uint32_t)b1;
    bv[3] = (int)(uint32_t)(b1 >> 32);
#pragma unroll
    for (int s = 0; s < ND; ++s) {
      const int sh = NB - 1 - s;  // A operand of diagonal s: byte b = digit s - b
      const uint64_t x0 = sh >= 0 ? ak.x >> (8 * sh) : ak.x << (-8 * sh);
      const uint64_t x1 = sh >= 0 ? ak.y >> (8 * sh) : ak.y << (-8 * sh);
      mfma_v4i av;
      av[0] = (int)(uint32_t)x0;
      av[1] = (int)(uint32_t)(x0 >> 32);
      av[2] = (int)(uint32_t)x1;
      av[3] = (int)(uint32_t)(x1 >> 32);
      acc[s] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, acc[s], 0, 0, 0);
    }
  }
  mfma_wait_vm<0>();
  __syncthreads();
  // fold: the lane holds rows j = 4 (lane >> 4) + r of column lane & 15 for lk = lk0 + w
  const long long lk = lk0 + w;
  const MfmaPrime& P = a.P[(int)(lk0 / a.d)];
  const uint64_t q = P.q;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = 4 * (lane >> 4) + r;
    __int128 S = 0;
#pragma unroll
    for (int s = 0; s < ND; ++s) S += (__int128)(long long)acc[s][r] << (8 * s);
    const uint64_t lo = (uint64_t)S;
    const long long hi = (long long)(S >> 64);
    uint64_t res = shoup_mul(lo, P.rinv, P.rinv_sh, q);
    if (hi >= 0) {
      res = mod_add(res, shoup_mul((uint64_t)hi, 1, P.one_sh, q), q);
    } else {
      res = mod_sub(res, shoup_mul((uint64_t)(-(hi + 1)) + 1, 1, P.one_sh, q), q);
    }
    res = mod_add(res, a.corr[lk * 16 + j], q);
    // [col][j][lk], each 16-word row rotated by 2 col: the wave's 64 lanes (16 columns, rows 16
    // words apart) then spread over 8 bank pairs instead of one (4-way, not 32-way, conflicts);
    // even rotations keep each lk pair 16-B aligned for the reads below
    ring[((lane & 15) * 16 + j) * LK + ((w + 2 * (lane & 15)) & (LK - 1))] = res;
  }
  __syncthreads();
  // 256 rows (col, j) of LK lk (LK * 8 B): LK / 2 threads x 16 B per row
  for (int i = tid; i < 256 * NP; i += 64 * LK) {
    const int row = i / NP, part = i % NP, cl = row >> 4, j = row & 15;
    const long long col = c0 + cl;
    if (j >= a.J || col >= a.ncols) continue;
    const int rp = (2 * part + 2 * cl) & (LK - 1);  // the write's rotation
    uint64_t r0 = ring[row * LK + rp], r1 = ring[row * LK + rp + 1];
    const long long l = lk0 + 2 * part;
    if (a.C) {
      const ulonglong2 cv = *reinterpret_cast<const ulonglong2*>(a.C + col * a.c_col + (long long)j * a.c_j + l);
      r0 = mod_add(cv.x, r0, q);
      r1 = mod_add(cv.y, r1, q);
    }
    *reinterpret_cast<ulonglong2*>(a.out + (col * a.J + j) * a.per_col + l) = make_ulonglong2(r0, r1);
  }
}

// key digits: thread per (lk, chunk, lane, half): term t = 8 chunk + 2 (lane >> 4) + half, row
// j = lane & 15; the NB balanced digits of A[j][t] byte-reversed within NB bytes (zero outside)
template <int NB>
__global__ __launch_bounds__(256) void mac_mfma_key_kernel(const uint64_t* A1, int T1, const uint64_t* A2, int T2,
                                                           int J, long long per_col, int Tc, uint64_t* out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= per_col * Tc * 128) return;
  const int half = (int)(i & 1), ln = (int)((i >> 1) & 63);
  const long long ck = i >> 7;
  const int chunk = (int)(ck % Tc);
  const long long lk = ck / Tc;
  const int j = ln & 15, t = chunk * 8 + 2 * (ln >> 4) + half;
  uint64_t x = 0;
  if (j < J && t < T1 + T2)
    x = t < T1 ? A1[((long long)j * T1 + t) * per_col + lk] : A2[((long long)j * T2 + (t - T1)) * per_col + lk];
  uint64_t R = 0;
  long long v = (long long)x;  // x < 2^62
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    long long dg = v & 255;
    if (dg >= 128) dg -= 256;
    v = (v - dg) >> 8;
    R |= (uint64_t)(uint8_t)(int8_t)dg << (8 * (NB - 1 - k));
  }
  out[i] = R;
}

// corr[lk][j] = bxor * sum_t A[j][t] * 2^-64 mod q
__global__ __launch_bounds__(256) void mac_mfma_corr_kernel(const uint64_t* A1, int T1, const uint64_t* A2, int T2,
                                                            int J, long long per_col, int d, uint64_t bxor,
                                                            MfmaPrime P0, MfmaPrime P1, MfmaPrime P2, MfmaPrime P3,
                                                            uint64_t* corr) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= per_col * 16) return;
  const int j = (int)(i & 15);
  const long long lk = i >> 4;
  const int limb = (int)(lk / d);
  const MfmaPrime P = limb == 0 ? P0 : limb == 1 ? P1 : limb == 2 ? P2 : P3;
  const uint64_t q = P.q;
  uint64_t s = 0;
  if (j < J) {
    for (int t = 0; t < T1; ++t) s = mod_add(s, A1[((long long)j * T1 + t) * per_col + lk] % q, q);
    for (int t = 0; t < T2; ++t) s = mod_add(s, A2[((long long)j * T2 + t) * per_col + lk] % q, q);
  }
  uint64_t lo, hi;
  mul_wide(s, bxor % q, lo, hi);  // < q^2 < 2^124: (lo + hi 2^64) 2^-64 = lo 2^-64 + hi
  corr[i] = mod_add(shoup_mul(lo, P.rinv, P.rinv_sh, q), hi % q, q);
}

uint64_t mac_mfma_bxor(int NB) {
  uint64_t m = 0;
  for (int k = 0; k < NB - 1; ++k) m |= 0x80ull << (8 * k);
  return m;
}

int mac_mfma_nb(const uint64_t* primes, int nl, int J, int T, int d) {
  if (J < 1 || J > 16 || d % 16 != 0 || nl < 1 || nl > kMfmaMaxQ || T < 1) return 0;
  int bits = 0;
  for (int l = 0; l < nl; ++l) bits = std::max(bits, 64 - __builtin_clzll(primes[l] - 1));
  const int NB = std::max(4, (bits + 2 + 7) / 8);  // q < 2^(8 NB - 2): the balanced top digit fits
  if (NB > 8) return 0;
  if ((double)((T + 7) / 8 * 8) * NB * 16384.0 >= 2147483648.0) return 0;  // int32 diagonal sums
  // |sum_t A b'| < T q max(q, bxor) must stay below 2^126, so that the fold's signed 128-bit
  // value and its high word (int64) cannot overflow (configs[4]: 545 x 2^58 x 2^58 = 2^125.1)
  double lq = 0;
  for (int l = 0; l < nl; ++l) lq = std::max(lq, std::log2((double)primes[l]));
  const double lx = std::log2((double)mac_mfma_bxor(NB) + 1.0);
  if (std::log2((double)T) + lq + std::max(lq, lx) >= 126.0) return 0;
  return NB;
}

void mac_mfma_key_ptrs(const DevBuf& key, long long per_col, int T, const uint64_t** Ak, const uint64_t** corr) {
  const int Tc = (T + 7) / 8;
  *Ak = static_cast<const uint64_t*>(key.p);
  *corr = static_cast<const uint64_t*>(key.p) + per_col * Tc * 128;
}

rg_status mac_mfma_key_dev(const uint64_t* A1, int T1, const uint64_t* A2, int T2, int J, long long per_col, int d,
                           int NB, const MfmaPrime* P, int nl, DevBuf& out, hipStream_t st) {
  const int Tc = (T1 + T2 + 7) / 8;
  const long long nk = per_col * Tc * 128, nc = per_col * 16;
  RG_TRY(out.alloc((size_t)(nk + nc) * 8));
  uint64_t* k = out.as<uint64_t>();
  const dim3 gk((unsigned)((nk + 255) / 256)), b(256);
  switch (NB) {
    case 4: hipLaunchKernelGGL(mac_mfma_key_kernel<4>, gk, b, 0, st, A1, T1, A2, T2, J, per_col, Tc, k); break;
    case 5: hipLaunchKernelGGL(mac_mfma_key_kernel<5>, gk, b, 0, st, A1, T1, A2, T2, J, per_col, Tc, k); break;
    case 6: hipLaunchKernelGGL(mac_mfma_key_kernel<6>, gk, b, 0, st, A1, T1, A2, T2, J, per_col, Tc, k); break;
    case 7: hipLaunchKernelGGL(mac_mfma_key_kernel<7>, gk, b, 0, st, A1, T1, A2, T2, J, per_col, Tc, k); break;
    default: hipLaunchKernelGGL(mac_mfma_key_kernel<8>, gk, b, 0, st, A1, T1, A2, T2, J, per_col, Tc, k); break;
  }
  RG_TRY(check_launch("jindo mfma key"));
  MfmaPrime Q[kMfmaMaxQ] = {};
  for (int l = 0; l < nl && l < kMfmaMaxQ; ++l) Q[l] = P[l];
  hipLaunchKernelGGL(mac_mfma_corr_kernel, dim3((unsigned)((nc + 255) / 256)), b, 0, st, A1, T1, A2, T2, J, per_col, d,
                     mac_mfma_bxor(NB), Q[0], Q[1], Q[2], Q[3], k + nk);
  return check_launch("jindo mfma corr");
}

rg_status launch_mac_mfma(const MfmaMacArgs& args, int NB, hipStream_t st) {
  MfmaMacArgs a = args;
  a.bxor = mac_mfma_bxor(NB);  // the offset the key's correction table was built with
  if (a.per_col % 16 != 0 || a.d % 16 != 0 || a.J > 16 || a.ncols < 1) {
    set_last_error("mac_mfma: shape outside the kernel's assumptions");
    return RG_ERR_INVALID;
  }
  constexpr int LK = kMfmaLk;
  const long long blocks = (a.per_col / LK) * ((a.ncols + 15) / 16);
  const dim3 g((unsigned)blocks), b(64 * LK);
  switch (NB) {
    case 4: hipLaunchKernelGGL((mac_mfma_kernel<4, LK>), g, b, 0, st, a); break;
    case 5: hipLaunchKernelGGL((mac_mfma_kernel<5, LK>), g, b, 0, st, a); break;
    case 6: hipLaunchKernelGGL((mac_mfma_kernel<6, LK>), g, b, 0, st, a); break;
    case 7: hipLaunchKernelGGL((mac_mfma_kernel<7, LK>), g, b, 0, st, a); break;
    default: hipLaunchKernelGGL((mac_mfma_kernel<8, LK>), g, b, 0, st, a); break;
  }
  return check_launch("jindo mac_mfma");
}

}  // namespace rg
