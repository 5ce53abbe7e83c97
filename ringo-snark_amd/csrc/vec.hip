// vec.hip -- pointwise ring ops of math/bigpoly (vec.go:9-121 through baseOperator,
// base_op.go:49-171) for gfx950.
//
// HBM-bound streaming kernels: element i of [n][L] is handled by one lane; loads/stores are
// 16 B per lane where L is even (two limbs) and 8 B otherwise, grid-strided over a capped
// grid (2048 workgroups).  The *Add/*Sub forms read-modify-write `out` in one pass instead of
// the reference's pooled temporary (base_op.go:105-110) -- same residues, one less HBM trip.
#include <cstring>

#include "common.hpp"
#include "field.hpp"

namespace rg {

template <int L>
struct VecArgs {
  uint64_t* out;
  const uint64_t* a;
  const uint64_t* b;
  long long n;
  FieldParams<L> F;
  int spare;  // q < 2^(64L-1)
};

template <int L>
__device__ __forceinline__ void ld(uint64_t* r, const uint64_t* p) {
  if constexpr (L % 2 == 0) {
#pragma unroll
    for (int l = 0; l < L; l += 2) {
      ulonglong2 v = *reinterpret_cast<const ulonglong2*>(p + l);
      r[l] = v.x;
      r[l + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int l = 0; l < L; ++l) r[l] = p[l];
  }
}
template <int L>
__device__ __forceinline__ void st(uint64_t* p, const uint64_t* r) {
  if constexpr (L % 2 == 0) {
#pragma unroll
    for (int l = 0; l < L; l += 2) {
      ulonglong2 v;
      v.x = r[l];
      v.y = r[l + 1];
      *reinterpret_cast<ulonglong2*>(p + l) = v;
    }
  } else {
#pragma unroll
    for (int l = 0; l < L; ++l) p[l] = r[l];
  }
}

template <int L>
__device__ __forceinline__ void fmul(uint64_t* z, const uint64_t* x, const uint64_t* y, const FieldParams<L>& F,
                                     int spare) {
  if constexpr (L == 1) {
    if (spare) {
      z[0] = mont_mul1(x[0], y[0], F.q[0], F.qinv);
      return;
    }
  }
  f_mul<L>(z, x, y, F);
}

template <int L, int OP>
__global__ __launch_bounds__(256) void vec_kernel(VecArgs<L> a) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  uint64_t c[L];  // scalar operand of the SMUL* ops (one element at a.b)
  if constexpr (OP == RG_VEC_SMUL || OP == RG_VEC_SMUL_ADD || OP == RG_VEC_SMUL_SUB) ld<L>(c, a.b);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    uint64_t x[L], y[L], z[L];
    ld<L>(x, a.a + i * L);
    if constexpr (OP == RG_VEC_ADD || OP == RG_VEC_SUB || OP == RG_VEC_MUL || OP == RG_VEC_MUL_ADD ||
                  OP == RG_VEC_MUL_SUB)
      ld<L>(y, a.b + i * L);
    if constexpr (OP == RG_VEC_ADD) f_add<L>(z, x, y, a.F);
    if constexpr (OP == RG_VEC_SUB) f_sub<L>(z, x, y, a.F);
    if constexpr (OP == RG_VEC_NEG) f_neg<L>(z, x, a.F);
    if constexpr (OP == RG_VEC_MUL) fmul<L>(z, x, y, a.F, a.spare);
    if constexpr (OP == RG_VEC_SMUL) fmul<L>(z, x, c, a.F, a.spare);
    if constexpr (OP == RG_VEC_MUL_ADD || OP == RG_VEC_MUL_SUB || OP == RG_VEC_SMUL_ADD || OP == RG_VEC_SMUL_SUB) {
      uint64_t t[L], o[L];
      if constexpr (OP == RG_VEC_MUL_ADD || OP == RG_VEC_MUL_SUB)
        fmul<L>(t, x, y, a.F, a.spare);
      else
        fmul<L>(t, x, c, a.F, a.spare);
      ld<L>(o, a.out + i * L);
      if constexpr (OP == RG_VEC_MUL_ADD || OP == RG_VEC_SMUL_ADD)
        f_add<L>(z, o, t, a.F);
      else
        f_sub<L>(z, o, t, a.F);
    }
    st<L>(a.out + i * L, z);
  }
}

template <int L, int OP>
static rg_status launch_vec(const VecArgs<L>& a, hipStream_t st) {
  long long blocks = (a.n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) return RG_OK;
  hipLaunchKernelGGL((vec_kernel<L, OP>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  return check_launch("vec");
}

template <int L>
static rg_status vec_L(const rg_field* f, int op, uint64_t* out, const uint64_t* a, const uint64_t* b, size_t n,
                       hipStream_t st) {
  VecArgs<L> v;
  memcpy(v.F.q, f->q, 8 * L);
  v.F.qinv = f->qinv;
  v.out = out;
  v.a = a;
  v.b = b;
  v.n = (long long)n;
  v.spare = f->spare_bit ? 1 : 0;
  switch (op) {
    case RG_VEC_ADD: return launch_vec<L, RG_VEC_ADD>(v, st);
    case RG_VEC_SUB: return launch_vec<L, RG_VEC_SUB>(v, st);
    case RG_VEC_NEG: return launch_vec<L, RG_VEC_NEG>(v, st);
    case RG_VEC_MUL: return launch_vec<L, RG_VEC_MUL>(v, st);
    case RG_VEC_SMUL: return launch_vec<L, RG_VEC_SMUL>(v, st);
    case RG_VEC_MUL_ADD: return launch_vec<L, RG_VEC_MUL_ADD>(v, st);
    case RG_VEC_MUL_SUB: return launch_vec<L, RG_VEC_MUL_SUB>(v, st);
    case RG_VEC_SMUL_ADD: return launch_vec<L, RG_VEC_SMUL_ADD>(v, st);
    case RG_VEC_SMUL_SUB: return launch_vec<L, RG_VEC_SMUL_SUB>(v, st);
    default: return RG_ERR_INVALID;
  }
}

}  // namespace rg

using namespace rg;

extern "C" {

rg_status rg_vec_dev(const rg_field* f, int op, uint64_t* d_out, const uint64_t* d_a, const uint64_t* d_b, size_t n,
                     void* stream) {
  if (!f || op < 0 || op > RG_VEC_SMUL_SUB) return RG_ERR_INVALID;
  if (n == 0) return RG_OK;
  if (!d_out || !d_a || (op != RG_VEC_NEG && !d_b)) return RG_ERR_INVALID;
  hipStream_t st = as_stream(stream);
  switch (f->L) {
    case 1: return vec_L<1>(f, op, d_out, d_a, d_b, n, st);
    case 2: return vec_L<2>(f, op, d_out, d_a, d_b, n, st);
    case 4: return vec_L<4>(f, op, d_out, d_a, d_b, n, st);
    case 7: return vec_L<7>(f, op, d_out, d_a, d_b, n, st);
    case 14: return vec_L<14>(f, op, d_out, d_a, d_b, n, st);
    default: return RG_ERR_UNSUPPORTED;
  }
}

rg_status rg_vec(const rg_field* f, int op, uint64_t* out, const uint64_t* a, const uint64_t* b, size_t n) {
  if (!f || op < 0 || op > RG_VEC_SMUL_SUB) return RG_ERR_INVALID;
  if (n == 0) return RG_OK;
  if (!out || !a || (op != RG_VEC_NEG && !b)) return RG_ERR_INVALID;
  const size_t bytes = n * f->L * 8;
  const bool scalar = op == RG_VEC_SMUL || op == RG_VEC_SMUL_ADD || op == RG_VEC_SMUL_SUB;
  const bool rmw = op == RG_VEC_MUL_ADD || op == RG_VEC_MUL_SUB || op == RG_VEC_SMUL_ADD || op == RG_VEC_SMUL_SUB;
  DevBuf da, db, dout;
  RG_TRY(da.upload(a, bytes));
  if (op != RG_VEC_NEG) RG_TRY(db.upload(b, scalar ? f->L * 8 : bytes));
  RG_TRY(dout.alloc(bytes));
  if (rmw) RG_HIP(hipMemcpy(dout.p, out, bytes, hipMemcpyHostToDevice));
  RG_TRY(rg_vec_dev(f, op, dout.as<uint64_t>(), da.as<uint64_t>(), op != RG_VEC_NEG ? db.as<uint64_t>() : da.as<uint64_t>(),
                    n, nullptr));
  RG_HIP(hipMemcpy(out, dout.p, bytes, hipMemcpyDeviceToHost));
  return RG_OK;
}

}  // extern "C"
