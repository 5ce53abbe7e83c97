// Microbenchmark: issue cost (cycles per wave64 instruction per SIMD) of the 32-bit VALU ops an
// integer butterfly can be built from (tools/ubench/intmul.hip covers multiplies / carries).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 2048
#define K(ID, ASM, ...)                                                                         \
  __global__ void __launch_bounds__(256) k##ID(uint32_t* out, uint32_t seed) {                 \
    uint32_t a = seed * threadIdx.x | 1;                                                       \
    uint32_t x[8];                                                                          \
    for (int i = 0; i < 8; ++i) x[i] = a + i;                                                  \
    asm volatile("v_cmp_gt_u32 vcc, %0, %1" ::"v"(x[0]), "v"(x[1]));                           \
    for (int it = 0; it < ITERS; ++it) {                                                       \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(ASM : "+v"(x[i]) : "v"(a) __VA_ARGS__); \
    }                                                                                          \
    uint32_t s = 0;                                                                            \
    for (int i = 0; i < 8; ++i) s += x[i];                                                     \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                            \
  }
K(0, "v_add_u32 %0, %1, %0", )
K(1, "v_sub_u32 %0, %1, %0", )
K(2, "v_xor_b32 %0, %1, %0", )
K(3, "v_and_b32 %0, %1, %0", )
K(4, "v_lshlrev_b32 %0, 3, %0", )
K(5, "v_mov_b32 %0, %1", )
K(6, "v_max_u32 %0, %1, %0", )
K(7, "v_min_u32 %0, %1, %0", )
K(8, "v_cndmask_b32 %0, %1, %0, vcc", )
K(9, "v_bfi_b32 %0, %1, %0, %1", )
K(10, "v_lshl_add_u32 %0, %0, 2, %1", )
K(11, "v_add_lshl_u32 %0, %0, %1, 2", )
K(12, "v_subrev_u32 %0, %1, %0", )
K(13, "v_alignbit_b32 %0, %1, %0, 7", )
K(14, "v_med3_u32 %0, %1, %0, %1", )
K(15, "v_ashrrev_i32 %0, 31, %0", )
K(16, "v_or3_b32 %0, %1, %0, %1", )
K(17, "v_lshrrev_b32 %0, 5, %0", )
K(18, "v_add_co_u32 %0, vcc, %1, %0", : "vcc")
K(19, "v_cndmask_b32_e64 %0, %1, %0, s[40:41]", : "s40")
K(20, "v_xad_u32 %0, %1, %0, %1", )
K(21, "v_mul_lo_u32 %0, %1, %0", )
K(22, "v_and_or_b32 %0, %1, %0, %1", )
K(23, "v_add3_u32 %0, %1, %0, %1", )
K(24, "v_add_co_u32 %0, vcc, %1, %0\n v_cndmask_b32 %0, %1, %0, vcc", : "vcc")
K(25, "v_cndmask_b32_e64 %0, %1, %0, vcc", : "vcc")
K(26, "v_add_co_u32 %0, s[40:41], %1, %0\n v_cndmask_b32_e64 %0, %1, %0, s[40:41]", : "s40", "s41")
K(27, "v_mul_hi_u32 %0, %1, %0", )
K(28, "v_add_co_u32 %0, vcc, %1, %0\n v_addc_co_u32 %0, vcc, %1, %0, vcc", : "vcc")
K(29, "v_sub_co_u32 %0, s[40:41], %1, %0\n v_subb_co_u32 %0, s[42:43], %1, %0, s[40:41]\n v_cndmask_b32_e64 %0, %1, %0, s[42:43]", : "s40", "s41", "s42", "s43")
K(30, "v_lshlrev_b32 %0, %1, %0", )
K(31, "v_not_b32 %0, %0", )
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
  R(0, "add_u32") R(1, "sub_u32") R(2, "xor") R(3, "and") R(4, "lshlrev") R(5, "mov") R(6, "max_u32")
  R(7, "min_u32") R(8, "cndmask vcc") R(9, "bfi") R(10, "lshl_add_u32") R(11, "add_lshl_u32") R(12, "subrev_u32")
  R(13, "alignbit") R(14, "med3_u32") R(15, "ashrrev") R(16, "or3") R(17, "lshrrev") R(18, "add_co vcc")
  R(19, "cndmask_e64 s") R(20, "xad_u32") R(21, "mul_lo_u32") R(22, "and_or") R(23, "add3") R(24, "add_co+cnd vcc(2)") R(25, "cnd_e64 vcc") R(26, "add_co+cnd s(2)") R(27, "mul_hi") R(28, "add_co+addc vcc(2)") R(29, "sub/subb/cnd s(3)") R(30, "lshlrev vreg") R(31, "not")
  return 0;
}
