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
//     same field element as the reference's single Horner pass.
// All field arithmetic is the Montgomery form of field.hpp (gnark's representation), so every
// output limb equals the reference's.
#include <cstring>

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
