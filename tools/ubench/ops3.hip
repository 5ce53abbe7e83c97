// Microbenchmark: issue cost (cycles per wave64 instruction per SIMD) of the VALU ops in the
// sampler / prep / NTT kernels that ops2.hip and intmul.hip do not cover: v_perm_b32,
// v_bitop3_b32 (AES), 64-bit moves / shifts / compares, the f64 arithmetic of the Gaussian
// samplers, conversions, lane ops.  Same harness as ops2.hip: 8 independent chains per lane.
// Build: hipcc -O3 --offload-arch=gfx950 -o ops3 tools/ubench/ops3.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 2048
#define K32(ID, ASM, ...)                                                                       \
  __global__ void __launch_bounds__(256) k##ID(uint32_t* out, uint32_t seed) {                 \
    uint32_t a = seed * threadIdx.x | 1;                                                       \
    uint32_t x[8];                                                                             \
    for (int i = 0; i < 8; ++i) x[i] = a + i;                                                  \
    asm volatile("v_cmp_gt_u32 vcc, %0, %1" ::"v"(x[0]), "v"(x[1]));                           \
    for (int it = 0; it < ITERS; ++it) {                                                       \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(ASM : "+v"(x[i]) : "v"(a) __VA_ARGS__); \
    }                                                                                          \
    uint32_t s = 0;                                                                            \
    for (int i = 0; i < 8; ++i) s += x[i];                                                     \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                            \
  }
#define K64(ID, ASM, ...)                                                                       \
  __global__ void __launch_bounds__(256) k##ID(uint32_t* out, uint32_t seed) {                 \
    uint64_t a = (uint64_t)(seed * threadIdx.x | 1) * 0x9E3779B97F4A7C15ull;                   \
    uint64_t x[8];                                                                             \
    for (int i = 0; i < 8; ++i) x[i] = a + i;                                                  \
    for (int it = 0; it < ITERS; ++it) {                                                       \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(ASM : "+v"(x[i]) : "v"(a) __VA_ARGS__); \
    }                                                                                          \
    uint64_t s = 0;                                                                            \
    for (int i = 0; i < 8; ++i) s += x[i];                                                     \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);            \
  }
K32(0, "v_perm_b32 %0, %1, %0, %1", )
K32(1, "v_bitop3_b32 %0, %1, %0, %1 bitop3:0x96", )
K32(2, "v_cndmask_b32 %0, %1, %0, vcc", )
K64(3, "v_mov_b64 %0, %0", )
K64(4, "v_lshl_add_u64 %0, %0, 1, %1", )
K64(5, "v_lshlrev_b64 %0, 3, %0", )
K64(6, "v_add_f64 %0, %0, %1", )
K64(7, "v_mul_f64 %0, %0, %1", )
K64(8, "v_fma_f64 %0, %0, %1, %1", )
K32(9, "v_cvt_f32_u32 %0, %0", )
K32(10, "v_cmp_lt_u32 vcc, %0, %1", : "vcc")
K64(11, "v_cmp_lt_u64 vcc, %0, %1", : "vcc")
K32(12, "v_mul_hi_u32_u24 %0, %1, %0", )
K32(13, "v_mul_u32_u24 %0, %1, %0", )
K32(14, "v_readfirstlane_b32 s40, %0", : "s40")
K64(15, "v_floor_f64 %0, %0", )
K32(16, "v_lshl_or_b32 %0, %0, 3, %1", )
K32(17, "v_exp_f32 %0, %0", )
K64(18, "v_rcp_f64 %0, %0", )
K64(19, "v_ldexp_f64 %0, %0, 3", )
template <typename F>
void run(const char* name, F f, uint32_t* d, int blocks) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  f<<<blocks, 256>>>(d, 3);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) f<<<blocks, 256>>>(d, 3 + r);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  double ops = (double)blocks * 256 * ITERS * 8;
  printf("%-16s %8.3f ms  %.2f cyc/wave-instr/SIMD @2.4GHz\n", name, ms, (ms * 1e-3 * 2.4e9 * 1024) / (ops / 64));
}
int main() {
  int blocks = 256 * 8 * 2;
  uint32_t* d;
  (void)hipMalloc(&d, blocks * 256 * 4);
#define R(ID, N) run(N, k##ID, d, blocks);
  R(0, "perm") R(1, "bitop3") R(2, "cndmask vcc") R(3, "mov_b64") R(4, "lshl_add_u64") R(5, "lshlrev_b64")
  R(6, "add_f64") R(7, "mul_f64") R(8, "fma_f64") R(9, "cvt_f32_u32") R(10, "cmp_lt_u32") R(11, "cmp_lt_u64")
  R(12, "mul_hi_u32_u24") R(13, "mul_u32_u24") R(14, "readfirstlane") R(15, "floor_f64") R(16, "lshl_or") R(17, "exp_f32")
  R(18, "rcp_f64") R(19, "ldexp_f64")
  return 0;
}
