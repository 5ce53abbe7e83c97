// poly_ops.hip -- the remaining bigpoly operators Buckler uses, for
// gfx950:
//   * CyclicEvaluator.QuoRemByVanishing (math/bigpoly/cyclic.go:18-37): one lane per residue
//     class k mod M; the reference's top-down loop is, per class, a suffix sum:
//     quo[k + (t-1) M] = sum_{s >= t} p[k + s M] (t >= 1), rem[k] = p[k] + quo[k], rem[k + tM] = 0;
//   * CyclotomicEvaluator.AutTo (cyclotomic.go:29-86): coefficient domain as a signed scatter
//     (j = i idx mod 2N, negated when j >= N), NTT domain as one gather through the bit
//     reversals (out[k] = p[brv(((2 brv(k) + 1) idx mod 2N - 1) / 2)]);
//   * Poly.Evaluate (poly.go:64-76): a Horner tree -- Horner over 64-coefficient chunks (one
//     lane each) in x, then over 64-value chunks of those in x^64, ... down to one value; the
//     same field element as the reference's single Horner pass;
//   * CyclotomicEvaluator.ModSwitchTo (cyclotomic.go:97-124): one lane per coefficient, the
//     reference's big-integer rounding division in fixed multiword arithmetic (below).
// All field arithmetic is the Montgomery form of field.hpp (gnark's representation), so every
// output limb equals the reference's.
#include <cstring>
#include <vector>

#include "common.hpp"
#include "field.hpp"

namespace rg {

template <int L>
struct PolyArgs {
  FieldParams<L> F;
  uint64_t* out;   // quo / aut output / chunk values
  uint64_t* out2;  // rem
  const uint64_t* in;
  long long rank;  // coefficients per polynomial
  long long batch;
  long long m;     // vanishing degree M, or automorphism index, or chunk count
  int logn;
};

template <int L>
__device__ __forceinline__ void cp(uint64_t* d, const uint64_t* s) {
#pragma unroll
  for (int l = 0; l < L; ++l) d[l] = s[l];
}

// ---- QuoRemByVanishing ----------------------------------------------------------------------
template <int L>
__global__ __launch_bounds__(256) void quorem_kernel(PolyArgs<L> a) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long M = a.m, N = a.rank;
  if (gid >= a.batch * M) return;
  const long long b = gid / M, k = gid % M;
  const uint64_t* p = a.in + b * N * L;
  uint64_t* quo = a.out + b * N * L;
  uint64_t* rem = a.out2 + b * N * L;
  uint64_t s[L];
#pragma unroll
  for (int l = 0; l < L; ++l) s[l] = 0;
  const long long top = (N - 1 - k) / M;  // largest t with k + tM < N
  for (long long t = top; t >= 1; --t) {
    uint64_t x[L];
    cp<L>(x, p + (k + t * M) * L);
    f_add<L>(s, s, x, a.F);
    cp<L>(quo + (k + (t - 1) * M) * L, s);
    uint64_t z[L] = {0};
    cp<L>(rem + (k + t * M) * L, z);
  }
  {  // the class's last quotient slot k + top M (>= N - M) receives nothing: zero
    uint64_t z[L] = {0};
    cp<L>(quo + (k + top * M) * L, z);
  }
  uint64_t x[L];
  cp<L>(x, p + k * L);
  f_add<L>(x, x, s, a.F);
  cp<L>(rem + k * L, x);
}

// M >= rank: quotient 0, remainder p (the reference's loop does not run)
template <int L>
__global__ __launch_bounds__(256) void quorem_trivial_kernel(PolyArgs<L> a) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.batch * a.rank * L) return;
  a.out[i] = 0;
  a.out2[i] = a.in[i];
}

// ---- AutTo ------------------------------------------------------------------------------------
template <int L>
__global__ __launch_bounds__(256) void aut_coeff_kernel(PolyArgs<L> a) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long N = a.rank;
  if (gid >= a.batch * N) return;
  const long long b = gid / N, i = gid % N;
  const long long j = (long long)(((unsigned long long)i * (unsigned long long)a.m) % (unsigned long long)(2 * N));
  uint64_t x[L];
  cp<L>(x, a.in + (b * N + i) * L);
  if (j < N) {
    cp<L>(a.out + (b * N + j) * L, x);
  } else {
    uint64_t y[L];
    f_neg<L>(y, x, a.F);
    cp<L>(a.out + (b * N + j - N) * L, y);
  }
}

__device__ __forceinline__ long long brv_n(long long x, int logn) {
  return logn ? (long long)(__brevll((unsigned long long)x) >> (64 - logn)) : 0;
}

template <int L>
__global__ __launch_bounds__(256) void aut_ntt_kernel(PolyArgs<L> a) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long N = a.rank;
  if (gid >= a.batch * N) return;
  const long long b = gid / N, k = gid % N;
  const long long i = brv_n(k, a.logn);
  const long long j = (long long)((((unsigned long long)(2 * i + 1) * (unsigned long long)a.m) % (unsigned long long)(2 * N) - 1) >> 1);
  cp<L>(a.out + (b * N + k) * L, a.in + (b * N + brv_n(j, a.logn)) * L);
}

// ---- Evaluate -------------------------------------------------------------------------------
constexpr int kEvalChunk = 64;

// one level of a Horner tree: out[c] = sum_{i < 64} in[64 c + i] y^i (z = z y + in_i from the
// top, poly.go:71-74), y = x^(64^level); the level-0 input is the polynomial itself
template <int L>
__global__ __launch_bounds__(256) void eval_level_kernel(FieldParams<L> F, const uint64_t* in, long long n,
                                                         const uint64_t* y, uint64_t* out) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= (n + kEvalChunk - 1) / kEvalChunk) return;
  uint64_t yv[L], z[L] = {0};
  cp<L>(yv, y);
  const long long lo = c * kEvalChunk, hi = min(n, lo + kEvalChunk);
  for (long long i = hi - 1; i >= lo; --i) {
    uint64_t t[L], pi[L];
    f_mul<L>(t, z, yv, F);
    cp<L>(pi, in + i * L);
    f_add<L>(z, t, pi, F);
  }
  cp<L>(out + c * L, z);
}

// y' = y^64 (six squarings), one lane
template <int L>
__global__ void eval_pow_kernel(FieldParams<L> F, const uint64_t* y, uint64_t* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t v[L];
  cp<L>(v, y);
  for (int s = 0; s < 6; ++s) f_mul<L>(v, v, v, F);
  cp<L>(out, v);
}

template <int L>
static PolyArgs<L> args_of(const rg_field* f) {
  PolyArgs<L> a;
  memset(&a, 0, sizeof(a));
  memcpy(a.F.q, f->q, 8 * L);
  a.F.qinv = f->qinv;
  return a;
}

static unsigned grid_of(long long n) { return (unsigned)((n + 255) / 256); }

template <int L>
static rg_status quorem_L(const rg_field* f, long long rank, long long m, uint64_t* quo, uint64_t* rem,
                          const uint64_t* p, long long batch, hipStream_t st) {
  PolyArgs<L> a = args_of<L>(f);
  a.out = quo;
  a.out2 = rem;
  a.in = p;
  a.rank = rank;
  a.batch = batch;
  a.m = m;
  if (m >= rank)
    hipLaunchKernelGGL(quorem_trivial_kernel<L>, dim3(grid_of(batch * rank * L)), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(quorem_kernel<L>, dim3(grid_of(batch * m)), dim3(256), 0, st, a);
  return check_launch("quorem");
}

template <int L>
static rg_status aut_L(const rg_field* f, long long rank, long long idx, bool ntt, uint64_t* out, const uint64_t* p,
                       long long batch, hipStream_t st) {
  PolyArgs<L> a = args_of<L>(f);
  a.out = out;
  a.in = p;
  a.rank = rank;
  a.batch = batch;
  a.m = idx;
  while ((1LL << a.logn) < rank) ++a.logn;
  if (ntt)
    hipLaunchKernelGGL(aut_ntt_kernel<L>, dim3(grid_of(batch * rank)), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(aut_coeff_kernel<L>, dim3(grid_of(batch * rank)), dim3(256), 0, st, a);
  return check_launch("aut");
}

// levels: n -> ceil(n/64) -> ... -> 1 value; scratch holds two value arrays and two powers
template <int L>
static rg_status eval_L(const rg_field* f, const uint64_t* p, long long n, const uint64_t* x, uint64_t* out,
                        uint64_t* scratch, hipStream_t st) {
  const PolyArgs<L> a = args_of<L>(f);
  const long long m0 = (n + kEvalChunk - 1) / kEvalChunk;
  uint64_t* buf[2] = {scratch, scratch + m0 * L};
  uint64_t* pw[2] = {scratch + 2 * m0 * L, scratch + 2 * m0 * L + L};
  const uint64_t* src = p;
  const uint64_t* y = x;
  long long cur = n;
  int lvl = 0;
  for (;;) {
    const long long m = (cur + kEvalChunk - 1) / kEvalChunk;
    uint64_t* dst = m == 1 ? out : buf[lvl & 1];
    hipLaunchKernelGGL(eval_level_kernel<L>, dim3(grid_of(m)), dim3(256), 0, st, a.F, src, cur, y, dst);
    RG_TRY(check_launch("evaluate level"));
    if (m == 1) return RG_OK;
    hipLaunchKernelGGL(eval_pow_kernel<L>, dim3(1), dim3(64), 0, st, a.F, y, pw[lvl & 1]);
    RG_TRY(check_launch("evaluate power"));
    y = pw[lvl & 1];
    src = dst;
    cur = m;
    ++lvl;
  }
}

// ---- ModSwitchTo ---------------------------------------------------------------------------
// Per coefficient p (w words, two's complement; |p| < 2^(64w-1)), with c = p q:
//   cRem = c mod qBig (Euclidean); cRem -= qBig when cRem > floor(qBig/2); c = (c - cRem) / qBig
//   mod q (cyclotomic.go:111-121).
// With A = |p| q = Qa qBig + ra (0 <= ra < qBig) this is
//   p >= 0: M = Qa + [ra > floor(qBig/2)],   result M mod q
//   p <  0: M = Qa + [ra >= qBig - floor(qBig/2)],   result (-M) mod q
// (for p < 0, c mod qBig = qBig - ra unless ra = 0, and the rounding moves toward +inf).  Both
// divisions are Barrett with host-computed reciprocals of 2^(64 nx), nx = w + L the width of A:
// the estimate floor(x mu / 2^(64 nx)) is at most 2 below the quotient, fixed by at most two
// subtractions.  Arrays are sized for w <= kMsMaxW.
constexpr int kMsMaxW = 8;

template <int L>
struct MsArgs {
  FieldParams<L> F;
  uint64_t r2[L];                          // R^2 mod q (SetBigInt -> Montgomery form)
  const uint64_t* in;                      // [n][w]
  uint64_t* out;                           // [n][L]
  long long n;
  int w, nx, nmu1, nmu2;
  uint64_t qbig[kMsMaxW];
  uint64_t tpos[kMsMaxW], tneg[kMsMaxW];   // floor(qBig/2) + 1, qBig - floor(qBig/2)
  uint64_t mu1[kMsMaxW + 16];              // floor(2^(64 nx) / qBig)
  uint64_t mu2[kMsMaxW + 16];              // floor(2^(64 nx) / q)
};

// a >= b over n words (little-endian)
__device__ __forceinline__ bool mw_geq(const uint64_t* a, const uint64_t* b, int n) {
  for (int i = n - 1; i >= 0; --i)
    if (a[i] != b[i]) return a[i] > b[i];
  return true;
}
// a -= b over n words (a >= b)
__device__ __forceinline__ void mw_sub(uint64_t* a, const uint64_t* b, int n) {
  uint32_t br = 0;
  for (int i = 0; i < n; ++i) {
    const uint64_t x = a[i], y = b[i];
    const uint64_t d = x - y - br;
    br = (x < y || (x == y && br)) ? 1u : 0u;
    a[i] = d;
  }
}
// a (na words) >= b (nb words, nb <= na); a -= b with b zero-extended
__device__ __forceinline__ bool mw_geq_ext(const uint64_t* a, int na, const uint64_t* b, int nb) {
  for (int i = na - 1; i >= nb; --i)
    if (a[i] != 0) return true;
  return mw_geq(a, b, nb);
}
__device__ __forceinline__ void mw_sub_ext(uint64_t* a, int na, const uint64_t* b, int nb) {
  uint32_t br = 0;
  for (int i = 0; i < na; ++i) {
    const uint64_t x = a[i], y = i < nb ? b[i] : 0;
    a[i] = x - y - br;
    br = (x < y || (x == y && br)) ? 1u : 0u;
  }
}
// quo (nx words), rem (nm words) of x (nx words) by m (nm words, m > 0) with mu = floor(2^(64 nx) / m)
// (nmu words); x and the scratch live in the caller's arrays
template <int NX>
__device__ void ms_divmod(const uint64_t* x, int nx, const uint64_t* m, int nm, const uint64_t* mu, int nmu,
                          uint64_t* quo, uint64_t* rem) {
  uint64_t pr[2 * NX + 1];
  for (int i = 0; i < nx + nmu; ++i) pr[i] = 0;
  for (int i = 0; i < nx; ++i) {  // pr = x mu
    uint64_t carry = 0;
    for (int j = 0; j < nmu; ++j) {
      uint64_t lo, hi;
      mul_wide(x[i], mu[j], lo, hi);
      uint32_t c = 0;
      lo = addc(lo, pr[i + j], c);
      hi += c;
      c = 0;
      lo = addc(lo, carry, c);
      hi += c;
      pr[i + j] = lo;
      carry = hi;
    }
    pr[i + nmu] = carry;
  }
  for (int i = 0; i < nx; ++i) quo[i] = i < nmu ? pr[nx + i] : 0;  // floor(x mu / 2^(64 nx)) < 2^(64 nx)
  uint64_t r[NX + 1];  // x - quo m, exact in nx words
  for (int i = 0; i < nx; ++i) r[i] = x[i];
  for (int i = 0; i < nm; ++i) {  // r -= quo * m[i] << 64 i (low nx words)
    uint64_t carry = 0;
    uint32_t br = 0;
    for (int j = 0; i + j < nx; ++j) {
      uint64_t lo, hi;
      mul_wide(quo[j], m[i], lo, hi);
      uint32_t c = 0;
      lo = addc(lo, carry, c);
      hi += c;
      carry = hi;
      const uint64_t a = r[i + j];
      const uint64_t d = a - lo - br;
      br = (a < lo || (a == lo && br)) ? 1u : 0u;
      r[i + j] = d;
    }
  }
  for (int it = 0; it < 3 && mw_geq_ext(r, nx, m, nm); ++it) {  // at most two corrections
    mw_sub_ext(r, nx, m, nm);
    for (int i = 0; i < nx && ++quo[i] == 0; ++i) {
    }
  }
  for (int i = 0; i < nm; ++i) rem[i] = i < nx ? r[i] : 0;
}

template <int L>
__global__ __launch_bounds__(256) void modswitch_kernel(MsArgs<L> a) {
  constexpr int NX = kMsMaxW + L;
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= a.n) return;
  const int w = a.w, nx = a.nx;
  const uint64_t* pin = a.in + gid * w;
  uint64_t mag[kMsMaxW];
  const bool neg = (pin[w - 1] >> 63) != 0;
  {
    uint32_t c = neg ? 1u : 0u;  // |p| = (p ^ -neg) + neg
    for (int i = 0; i < w; ++i) {
      const uint64_t x = neg ? ~pin[i] : pin[i];
      mag[i] = x + c;
      c = (c && mag[i] == 0) ? 1u : 0u;
    }
  }
  uint64_t A[NX];
  for (int i = 0; i < nx; ++i) A[i] = 0;
  for (int i = 0; i < w; ++i) {  // A = |p| q
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      uint64_t lo, hi;
      mul_wide(mag[i], a.F.q[j], lo, hi);
      uint32_t c = 0;
      lo = addc(lo, A[i + j], c);
      hi += c;
      c = 0;
      lo = addc(lo, carry, c);
      hi += c;
      A[i + j] = lo;
      carry = hi;
    }
    A[i + L] = carry;
  }
  uint64_t Q[NX], ra[kMsMaxW];
  ms_divmod<NX>(A, nx, a.qbig, w, a.mu1, a.nmu1, Q, ra);
  if (mw_geq(ra, neg ? a.tneg : a.tpos, w))
    for (int i = 0; i < nx && ++Q[i] == 0; ++i) {
    }
  uint64_t Qq[NX], r[L];
  ms_divmod<NX>(Q, nx, a.F.q, L, a.mu2, a.nmu2, Qq, r);
  bool nz = false;
#pragma unroll
  for (int j = 0; j < L; ++j) nz |= r[j] != 0;
  if (neg && nz) {  // (-M) mod q = q - (M mod q)
    uint64_t t[L];
#pragma unroll
    for (int j = 0; j < L; ++j) t[j] = a.F.q[j];
    mw_sub(t, r, L);
#pragma unroll
    for (int j = 0; j < L; ++j) r[j] = t[j];
  }
  uint64_t o[L];
  f_mul<L>(o, r, a.r2, a.F);  // SetBigInt: r R mod q
  cp<L>(a.out + gid * L, o);
}

// host: floor(2^(64 nx) / m) by restoring binary division (m: nm words, result <= nx + 1 words)
static int host_recip(const uint64_t* m, int nm, int nx, uint64_t* mu, int cap) {
  const int nq = nx + 1;
  if (nq > cap) return -1;
  std::vector<uint64_t> r(nm + 1, 0);
  for (int i = 0; i < nq; ++i) mu[i] = 0;
  auto geq = [&](void) {
    if (r[nm] != 0) return true;
    for (int i = nm - 1; i >= 0; --i)
      if (r[i] != m[i]) return r[i] > m[i];
    return true;
  };
  for (int bit = 64 * nx; bit >= 0; --bit) {  // dividend 2^(64 nx): a single 1 bit at position 64 nx
    for (int i = nm; i > 0; --i) r[i] = (r[i] << 1) | (r[i - 1] >> 63);  // r = 2 r + bit
    r[0] = (r[0] << 1) | (bit == 64 * nx ? 1u : 0u);
    if (geq()) {
      uint64_t br = 0;
      for (int i = 0; i <= nm; ++i) {
        const uint64_t y = i < nm ? m[i] : 0;
        const uint64_t x = r[i];
        r[i] = x - y - br;
        br = (x < y || (x == y && br)) ? 1u : 0u;
      }
      mu[bit >> 6] |= 1ull << (bit & 63);
    }
  }
  int n = nq;
  while (n > 1 && mu[n - 1] == 0) --n;
  return n;
}

template <int L>
static rg_status modswitch_L(const rg_field* f, const uint64_t* pbig, int w, const uint64_t* qbig, uint64_t* out,
                             long long n, hipStream_t st) {
  MsArgs<L> a;
  memset(&a, 0, sizeof(a));
  memcpy(a.F.q, f->q, 8 * L);
  a.F.qinv = f->qinv;
  memcpy(a.r2, f->r2, 8 * L);
  a.in = pbig;
  a.out = out;
  a.n = n;
  a.w = w;
  a.nx = w + L;
  memcpy(a.qbig, qbig, 8 * w);
  // thresholds: h = floor(qBig / 2); tpos = h + 1, tneg = qBig - h
  uint64_t h[kMsMaxW];
  for (int i = 0; i < w; ++i) h[i] = (qbig[i] >> 1) | (i + 1 < w ? (qbig[i + 1] << 63) : 0);
  {
    uint32_t c = 1;
    for (int i = 0; i < w; ++i) {
      a.tpos[i] = h[i] + c;
      c = (c && a.tpos[i] == 0) ? 1u : 0u;
    }
    uint64_t br = 0;
    for (int i = 0; i < w; ++i) {
      const uint64_t x = qbig[i], y = h[i];
      a.tneg[i] = x - y - br;
      br = (x < y || (x == y && br)) ? 1u : 0u;
    }
  }
  int nqb = w;
  while (nqb > 1 && qbig[nqb - 1] == 0) --nqb;
  a.nmu1 = host_recip(qbig, nqb, a.nx, a.mu1, kMsMaxW + 16);
  a.nmu2 = host_recip(f->q, L, a.nx, a.mu2, kMsMaxW + 16);
  if (a.nmu1 < 0 || a.nmu2 < 0) return RG_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(modswitch_kernel<L>, dim3(grid_of(n)), dim3(256), 0, st, a);
  return check_launch("modswitch");
}

#define RG_DISPATCH_L(L_, CALL)                 \
  switch (L_) {                                 \
    case 1: return CALL(1);                     \
    case 2: return CALL(2);                     \
    case 4: return CALL(4);                     \
    case 7: return CALL(7);                     \
    case 14: return CALL(14);                   \
    default: return RG_ERR_UNSUPPORTED;         \
  }

static bool pow2(long long n) { return n > 0 && !(n & (n - 1)); }

}  // namespace rg

using namespace rg;

extern "C" {

rg_status rg_poly_quorem_vanishing_dev(const rg_field* f, size_t rank, long long n_vanish, uint64_t* d_quo,
                                       uint64_t* d_rem, const uint64_t* d_p, size_t batch, void* stream) {
  if (!f || n_vanish < 0 || (batch && (!d_quo || !d_rem || !d_p)) || d_quo == d_rem) return RG_ERR_INVALID;
  if (batch == 0 || rank == 0) return RG_OK;
  hipStream_t st = as_stream(stream);
  if (n_vanish == 0) {  // every coefficient moves to the quotient: quo = p, rem = 0
    RG_HIP(hipMemcpyAsync(d_quo, d_p, batch * rank * f->L * 8, hipMemcpyDeviceToDevice, st));
    RG_HIP(hipMemsetAsync(d_rem, 0, batch * rank * f->L * 8, st));
    return RG_OK;
  }
  if (d_quo == d_p) return RG_ERR_INVALID;  // rem may alias p (each lane reads its class first)
#define RG_QR(L) quorem_L<L>(f, (long long)rank, n_vanish, d_quo, d_rem, d_p, (long long)batch, st)
  RG_DISPATCH_L(f->L, RG_QR)
#undef RG_QR
}

rg_status rg_poly_aut_dev(const rg_field* f, size_t rank, long long idx, int ntt_domain, uint64_t* d_out,
                          const uint64_t* d_p, size_t batch, void* stream) {
  if (!f || (batch && (!d_out || !d_p)) || d_out == d_p) return RG_ERR_INVALID;
  if (!pow2((long long)rank)) return RG_ERR_INVALID;
  if ((idx & 1) == 0) return RG_ERR_INVALID;  // cyclotomic.go:34-36 "AutTo: idx must be odd"
  if (batch == 0) return RG_OK;
  const long long n2 = 2 * (long long)rank;
  long long k = idx % n2;  // cyclotomic.go:38-41
  if (k < 0) k += n2;
  hipStream_t st = as_stream(stream);
#define RG_AUT(L) aut_L<L>(f, (long long)rank, k, ntt_domain != 0, d_out, d_p, (long long)batch, st)
  RG_DISPATCH_L(f->L, RG_AUT)
#undef RG_AUT
}

rg_status rg_poly_evaluate_dev(const rg_field* f, const uint64_t* d_p, size_t n, const uint64_t* d_x, uint64_t* d_out,
                               uint64_t* d_scratch, void* stream) {
  if (!f || !d_x || !d_out || (n && (!d_p || !d_scratch))) return RG_ERR_INVALID;
  hipStream_t st = as_stream(stream);
  if (n == 0) {  // z stays 0
    RG_HIP(hipMemsetAsync(d_out, 0, f->L * 8, st));
    return RG_OK;
  }
#define RG_EV(L) eval_L<L>(f, d_p, (long long)n, d_x, d_out, d_scratch, st)
  RG_DISPATCH_L(f->L, RG_EV)
#undef RG_EV
}

rg_status rg_poly_modswitch_dev(const rg_field* f, size_t n, const uint64_t* d_pbig, size_t w, const uint64_t* qbig,
                                uint64_t* d_out, void* stream) {
  if (!f || !qbig || w == 0 || w > (size_t)kMsMaxW || (n && (!d_pbig || !d_out))) return RG_ERR_INVALID;
  bool qz = true;
  for (size_t i = 0; i < w; ++i) qz = qz && qbig[i] == 0;
  if (qz || (qbig[w - 1] >> 63)) return RG_ERR_INVALID;  // qBig > 0, as a w-word signed value
  if (n == 0) return RG_OK;
  hipStream_t st = as_stream(stream);
#define RG_MS(L) modswitch_L<L>(f, d_pbig, (int)w, qbig, d_out, (long long)n, st)
  RG_DISPATCH_L(f->L, RG_MS)
#undef RG_MS
}

size_t rg_poly_evaluate_scratch_bytes(const rg_field* f, size_t n) {
  return f ? (2 * ((n + kEvalChunk - 1) / kEvalChunk) + 2) * f->L * 8 : 0;
}

// host-pointer forms (cgo drop-in; stage through device buffers)
rg_status rg_poly_quorem_vanishing(const rg_field* f, size_t rank, long long n_vanish, uint64_t* quo, uint64_t* rem,
                                   const uint64_t* p) {
  if (!f || !quo || !rem || !p) return RG_ERR_INVALID;
  const size_t bytes = rank * f->L * 8;
  DevBuf dp, dq, dr;
  RG_TRY(dp.upload(p, bytes));
  RG_TRY(dq.alloc(bytes));
  RG_TRY(dr.alloc(bytes));
  RG_TRY(rg_poly_quorem_vanishing_dev(f, rank, n_vanish, dq.as<uint64_t>(), dr.as<uint64_t>(), dp.as<uint64_t>(), 1,
                                      nullptr));
  RG_HIP(hipMemcpy(quo, dq.p, bytes, hipMemcpyDeviceToHost));
  RG_HIP(hipMemcpy(rem, dr.p, bytes, hipMemcpyDeviceToHost));
  return RG_OK;
}

rg_status rg_poly_aut(const rg_field* f, size_t rank, long long idx, int ntt_domain, uint64_t* out, const uint64_t* p) {
  if (!f || !out || !p) return RG_ERR_INVALID;
  const size_t bytes = rank * f->L * 8;
  DevBuf dp, dq;
  RG_TRY(dp.upload(p, bytes));
  RG_TRY(dq.alloc(bytes));
  RG_TRY(rg_poly_aut_dev(f, rank, idx, ntt_domain, dq.as<uint64_t>(), dp.as<uint64_t>(), 1, nullptr));
  RG_HIP(hipMemcpy(out, dq.p, bytes, hipMemcpyDeviceToHost));
  return RG_OK;
}

rg_status rg_poly_modswitch(const rg_field* f, size_t n, const uint64_t* pbig, size_t w, const uint64_t* qbig,
                            uint64_t* out) {
  if (!f || !qbig || (n && (!pbig || !out)) || w == 0 || w > (size_t)kMsMaxW) return RG_ERR_INVALID;
  if (n == 0) return rg_poly_modswitch_dev(f, 0, nullptr, w, qbig, nullptr, nullptr);
  DevBuf dp, dq;
  RG_TRY(dp.upload(pbig, n * w * 8));
  RG_TRY(dq.alloc(n * f->L * 8));
  RG_TRY(rg_poly_modswitch_dev(f, n, dp.as<uint64_t>(), w, qbig, dq.as<uint64_t>(), nullptr));
  RG_HIP(hipMemcpy(out, dq.p, n * f->L * 8, hipMemcpyDeviceToHost));
  return RG_OK;
}

rg_status rg_poly_evaluate(const rg_field* f, const uint64_t* p, size_t n, const uint64_t* x, uint64_t* out) {
  if (!f || !x || !out || (n && !p)) return RG_ERR_INVALID;
  DevBuf dp, dx, dout, ds;
  if (n) RG_TRY(dp.upload(p, n * f->L * 8));
  RG_TRY(dx.upload(x, f->L * 8));
  RG_TRY(dout.alloc(f->L * 8));
  RG_TRY(ds.alloc(rg_poly_evaluate_scratch_bytes(f, n) + 8));
  RG_TRY(rg_poly_evaluate_dev(f, n ? dp.as<uint64_t>() : nullptr, n, dx.as<uint64_t>(), dout.as<uint64_t>(),
                              ds.as<uint64_t>(), nullptr));
  RG_HIP(hipMemcpy(out, dout.p, f->L * 8, hipMemcpyDeviceToHost));
  return RG_OK;
}

}  // extern "C"
