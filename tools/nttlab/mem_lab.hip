// Memory lab: the HBM access patterns of one ntt16_pass step (COL load/store, ROW-RP load/store,
// in place over batch x 2^16 u64) with NO arithmetic and NO LDS, to separate the patterns' own
// streaming rate from what the LDS exchanges / barriers / butterflies cost (pass_lab "neither").
// Build: hipcc -O3 --offload-arch=gfx950 -o mem_lab mem_lab.hip   Run: tools/nttlab/mem_lab [batch]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
template <int AUX> __device__ __forceinline__ uint64_t ld(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
  const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, AUX);
  return ((uint64_t)v.y << 32) | v.x;
}
template <int AUX> __device__ __forceinline__ void st(uint64_t x, __amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
  u32x2 v; v.x = (uint32_t)x; v.y = (uint32_t)(x >> 32);
  __builtin_amdgcn_raw_buffer_store_b64(v, r, vo, so, AUX);
}

// COL fwd: tile = 16 columns of one poly; load rows t + 32y, store rows 8t + r (ntt16_tile)
template <int AUX, bool INV>
__global__ __launch_bounds__(512) void col_pat(uint64_t* x) {
  const uint32_t tid = threadIdx.x, s = tid & 15u, t = tid >> 4, tile = blockIdx.x;
  const size_t tbase = ((size_t)(tile >> 4) << 16) + ((tile & 15u) << 4);
  const auto r = rsrc(x + tbase);
  uint64_t e[8];
  const uint32_t voH = ((t << 8) + s) * 8u, voL = ((t << 11) + s) * 8u;
  if (!INV) {
#pragma unroll
    for (int y = 0; y < 8; ++y) e[y] = ld<AUX>(r, voH, (uint32_t)y << 16);
#pragma unroll
    for (int y = 0; y < 8; ++y) st<AUX>(e[y] + 1, r, voL, (uint32_t)y << 11);
  } else {
#pragma unroll
    for (int y = 0; y < 8; ++y) e[y] = ld<AUX>(r, voL, (uint32_t)y << 11);
#pragma unroll
    for (int y = 0; y < 8; ++y) st<AUX>(e[y] + 1, r, voH, (uint32_t)y << 16);
  }
}
// ROW (RP): tile = row (tile & 255) of 16 consecutive polys; lane t, rows s: t + 32 y
template <int AUX>
__global__ __launch_bounds__(512) void row_pat(uint64_t* x) {
  const uint32_t tid = threadIdx.x, s = tid >> 5, t = tid & 31u, tile = blockIdx.x;
  const size_t tbase = ((size_t)(tile >> 8) << 20) + ((tile & 255u) << 8);
  const auto r = rsrc(x + tbase);
  const uint32_t vo = ((s << 16) + t) * 8u;
  uint64_t e[8];
#pragma unroll
  for (int y = 0; y < 8; ++y) e[y] = ld<AUX>(r, vo + 256u * y, 0);
#pragma unroll
  for (int y = 0; y < 8; ++y) st<AUX>(e[y] + 1, r, vo + 256u * y, 0);
}
// linear in-place read-modify-write, 16 B per lane (the streaming reference)
__global__ __launch_bounds__(512) void lin_pat(uint64_t* x, size_t n2) {
  u32x4* p = reinterpret_cast<u32x4*>(x);
  for (size_t i = (size_t)blockIdx.x * 512 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 512) {
    u32x4 v = __builtin_nontemporal_load(p + i);
    v.x += 1;
    __builtin_nontemporal_store(v, p + i);
  }
}
// COL with 32 columns per tile, 2 adjacent columns per lane as one 16-B access
template <int AUX>
__global__ __launch_bounds__(512) void col32_pat(uint64_t* x) {
  const uint32_t tid = threadIdx.x, s = tid & 15u, t = tid >> 4, tile = blockIdx.x;
  const size_t tbase = ((size_t)(tile >> 3) << 16) + ((tile & 7u) << 5);
  const auto r = rsrc(x + tbase);
  u32x4 e[8];
  const uint32_t voH = ((t << 8) + 2 * s) * 8u, voL = ((t << 11) + 2 * s) * 8u;
#pragma unroll
  for (int y = 0; y < 8; ++y) e[y] = __builtin_amdgcn_raw_buffer_load_b128(r, voH, (uint32_t)y << 16, AUX);
#pragma unroll
  for (int y = 0; y < 8; ++y) { e[y].x += 1; __builtin_amdgcn_raw_buffer_store_b128(e[y], r, voL, (uint32_t)y << 11, AUX); }
}

template <class F>
static float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); f();
  std::vector<float> v;
  for (int k = 0; k < reps; ++k) {
    CK(hipEventRecord(a)); f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); v.push_back(ms);
  }
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const size_t batch = argc > 1 ? atoi(argv[1]) : 1024, N = 1 << 16;
  uint64_t* x;
  CK(hipMalloc(&x, batch * N * 8));
  CK(hipMemset(x, 1, batch * N * 8));
  const unsigned tcol = (unsigned)(batch * 16), trow = (unsigned)(batch * 16);
  const double step_bytes = 4.0 * 2 * batch * N * 8;  // 4 passes, read + write
  auto rep = [&](const char* name, float ms, double bytes) {
    printf("%-34s %8.3f ms  %6.2f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12);
  };
  for (int k = 0; k < 2; ++k) {
    rep("lin rmw x4 (16B/lane, nt)", timeit([&] { for (int i = 0; i < 4; ++i) hipLaunchKernelGGL(lin_pat, dim3(8192), dim3(512), 0, 0, x, batch * N / 2); }, 7), step_bytes);
    rep("col fwd+inv x2, row x2 (aux 2)", timeit([&] {
      hipLaunchKernelGGL((col_pat<2, false>), dim3(tcol), dim3(512), 0, 0, x);
      hipLaunchKernelGGL((row_pat<2>), dim3(trow), dim3(512), 0, 0, x);
      hipLaunchKernelGGL((row_pat<2>), dim3(trow), dim3(512), 0, 0, x);
      hipLaunchKernelGGL((col_pat<2, true>), dim3(tcol), dim3(512), 0, 0, x); }, 7), step_bytes);
    rep("  col fwd only x4 (aux 2)", timeit([&] { for (int i = 0; i < 4; ++i) hipLaunchKernelGGL((col_pat<2, false>), dim3(tcol), dim3(512), 0, 0, x); }, 7), step_bytes);
    rep("  col inv only x4 (aux 2)", timeit([&] { for (int i = 0; i < 4; ++i) hipLaunchKernelGGL((col_pat<2, true>), dim3(tcol), dim3(512), 0, 0, x); }, 7), step_bytes);
    rep("  row only x4 (aux 2)", timeit([&] { for (int i = 0; i < 4; ++i) hipLaunchKernelGGL((row_pat<2>), dim3(trow), dim3(512), 0, 0, x); }, 7), step_bytes);
    rep("  row only x4 (aux 0)", timeit([&] { for (int i = 0; i < 4; ++i) hipLaunchKernelGGL((row_pat<0>), dim3(trow), dim3(512), 0, 0, x); }, 7), step_bytes);
    rep("  col fwd only x4 (aux 0)", timeit([&] { for (int i = 0; i < 4; ++i) hipLaunchKernelGGL((col_pat<0, false>), dim3(tcol), dim3(512), 0, 0, x); }, 7), step_bytes);
    rep("  col32 (16B lanes) x4 (aux 2)", timeit([&] { for (int i = 0; i < 4; ++i) hipLaunchKernelGGL((col32_pat<2>), dim3(tcol / 2), dim3(512), 0, 0, x); }, 7), step_bytes);
  }
  return 0;
}
