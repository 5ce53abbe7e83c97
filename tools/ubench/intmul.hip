// Microbenchmark: per-instruction issue rates on gfx950 for the integer ops a modular
// multiply is built from. Inline asm pins the exact instruction; 8 independent chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 2048
template <int KIND>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1;
  uint32_t x[8]; uint64_t y[8]; double f[8];
  for (int i = 0; i < 8; ++i) { x[i] = a + i; y[i] = a * 3 + i; f[i] = (double)(a + i); }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (KIND == 0) asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(y[i]) : "v"(a) : "vcc");
      if (KIND == 1) asm volatile("v_mul_hi_u32 %0, %1, %0" : "+v"(x[i]) : "v"(a));
      if (KIND == 2) asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(x[i]) : "v"(a));
      if (KIND == 3) asm volatile("v_add_u32 %0, %1, %0" : "+v"(x[i]) : "v"(a));
      if (KIND == 4) asm volatile("v_mad_u32_u24 %0, %1, %0, %1" : "+v"(x[i]) : "v"(a));
      if (KIND == 5) asm volatile("v_fma_f64 %0, %1, %0, %1" : "+v"(f[i]) : "v"((double)a));
      if (KIND == 6) asm volatile("v_lshl_add_u64 %0, %0, 1, %0" : "+v"(y[i]));
      if (KIND == 7) asm volatile("v_mul_u32_u24 %0, %1, %0" : "+v"(x[i]) : "v"(a));
      if (KIND == 8) asm volatile("v_mul_f64 %0, %1, %0" : "+v"(f[i]) : "v"((double)a));
      if (KIND == 9) asm volatile("v_add_co_u32 %0, vcc, %1, %0" : "+v"(x[i]) : "v"(a) : "vcc");
      if (KIND == 10) asm volatile("v_addc_co_u32 %0, vcc, %1, %0, vcc" : "+v"(x[i]) : "v"(a) : "vcc");
      if (KIND == 11) asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(x[i]) : "v"(a) : "vcc");
      if (KIND == 12) asm volatile("v_add_co_u32 %0, s[40:41], %1, %0" : "+v"(x[i]) : "v"(a) : "s40", "s41");
      if (KIND == 13) asm volatile("v_add3_u32 %0, %1, %0, %1" : "+v"(x[i]) : "v"(a));
      if (KIND == 14) asm volatile("v_cmp_gt_u64 vcc, %0, %1" : : "v"(y[i]), "v"(y[(i + 1) & 7]) : "vcc");
      if (KIND == 15) asm volatile("v_alignbit_b32 %0, %1, %0, 12" : "+v"(x[i]) : "v"(a));
      if (KIND == 16) asm volatile("v_mul_hi_u32_u24 %0, %1, %0" : "+v"(x[i]) : "v"(a));
      if (KIND == 17) asm volatile("v_sub_co_u32 %0, s[40:41], %1, %0\n v_subb_co_u32 %0, s[40:41], %1, %0, s[40:41]" : "+v"(x[i]) : "v"(a) : "s40", "s41");
      if (KIND == 18) asm volatile("v_pk_add_u16 %0, %1, %0" : "+v"(x[i]) : "v"(a));
      if (KIND == 19) asm volatile("v_cndmask_b32 %0, %1, %0, s[40:41]" : "+v"(x[i]) : "v"(a) : "s40", "s41");
    }
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x[i] + (uint32_t)y[i] + (uint32_t)(y[i] >> 32) + (uint32_t)f[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int KIND> void run(const char* name, uint32_t* d, int blocks) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  k<KIND><<<blocks, 256>>>(d, 3); (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0); for (int r = 0; r < 5; ++r) k<KIND><<<blocks, 256>>>(d, 3 + r);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1); ms /= 5;
  double ops = (double)blocks * 256 * ITERS * 8;
  printf("%-16s %8.3f ms  %8.2f T lane-ops/s  (%.2f cyc/wave-instr/SIMD @2.4GHz)\n", name, ms, ops / ms / 1e9,
         (ms * 1e-3 * 2.4e9 * 1024) / (ops / 64));
}
int main() {
  int blocks = 256 * 8 * 2; uint32_t* d; (void)hipMalloc(&d, blocks * 256 * 4);
  run<0>("v_mad_u64_u32", d, blocks); run<1>("v_mul_hi_u32", d, blocks); run<2>("v_mul_lo_u32", d, blocks);
  run<3>("v_add_u32", d, blocks); run<4>("v_mad_u32_u24", d, blocks); run<5>("v_fma_f64", d, blocks);
  run<6>("v_lshl_add_u64", d, blocks); run<7>("v_mul_u32_u24", d, blocks); run<8>("v_mul_f64", d, blocks);
  run<9>("v_add_co_u32", d, blocks); run<10>("v_addc_co_u32", d, blocks); run<11>("v_cndmask vcc", d, blocks);
  run<12>("v_add_co sgpr", d, blocks); run<13>("v_add3_u32", d, blocks); run<14>("v_cmp_gt_u64", d, blocks);
  run<15>("v_alignbit", d, blocks); run<16>("v_mul_hi_u24", d, blocks); run<17>("sub_co+subb(2)", d, blocks);
  run<18>("v_pk_add_u16", d, blocks); run<19>("v_cndmask sgpr", d, blocks);
  return 0;
}
