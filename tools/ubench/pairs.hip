#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 1024
__global__ void __launch_bounds__(256) k0(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %1, %0" : "+v"(y0[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k1(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(x0[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k2(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_hi_u32 %0, %1, %0" : "+v"(x0[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k3(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_co_u32 %0, s[42:43], %1, %0" : "+v"(x0[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k4(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_addc_co_u32 %0, s[44:45], %1, %0, s[46:47]" : "+v"(x0[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k5(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_cndmask_b32_e64 %0, %1, %0, s[48:49]" : "+v"(x0[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k6(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add3_u32 %0, %1, %0, %1" : "+v"(x0[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k7(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_lshl_add_u64 %0, %0, 1, %0" : "+v"(y0[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k8(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_u32 %0, %1, %0" : "+v"(x0[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k9(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_bfi_b32 %0, %1, %0, %1" : "+v"(x0[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k10(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_cmp_gt_u64 s[50:51], %0, %0" : "+v"(y0[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k11(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_sub_co_u32 %0, s[52:53], %1, %0" : "+v"(x0[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k12(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %2, %0\n v_mad_u64_u32 %1, s[40:41], %2, %2, %1" : "+v"(y0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k13(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %2, %0\n v_mul_lo_u32 %1, %2, %1" : "+v"(y0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k14(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %2, %0\n v_mul_hi_u32 %1, %2, %1" : "+v"(y0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k15(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %2, %0\n v_add_co_u32 %1, s[42:43], %2, %1" : "+v"(y0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k16(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %2, %0\n v_addc_co_u32 %1, s[44:45], %2, %1, s[46:47]" : "+v"(y0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k17(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %2, %0\n v_cndmask_b32_e64 %1, %2, %1, s[48:49]" : "+v"(y0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k18(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %2, %0\n v_add3_u32 %1, %2, %1, %2" : "+v"(y0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k19(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %2, %0\n v_lshl_add_u64 %1, %1, 1, %1" : "+v"(y0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k20(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %2, %0\n v_add_u32 %1, %2, %1" : "+v"(y0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k21(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %2, %0\n v_bfi_b32 %1, %2, %1, %2" : "+v"(y0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k22(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %2, %0\n v_cmp_gt_u64 s[50:51], %1, %1" : "+v"(y0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k23(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mad_u64_u32 %0, s[40:41], %2, %2, %0\n v_sub_co_u32 %1, s[52:53], %2, %1" : "+v"(y0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k24(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_lo_u32 %0, %2, %0\n v_mul_lo_u32 %1, %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k25(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_lo_u32 %0, %2, %0\n v_mul_hi_u32 %1, %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k26(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_lo_u32 %0, %2, %0\n v_add_co_u32 %1, s[42:43], %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k27(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_lo_u32 %0, %2, %0\n v_addc_co_u32 %1, s[44:45], %2, %1, s[46:47]" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k28(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_lo_u32 %0, %2, %0\n v_cndmask_b32_e64 %1, %2, %1, s[48:49]" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k29(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_lo_u32 %0, %2, %0\n v_add3_u32 %1, %2, %1, %2" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k30(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_lo_u32 %0, %2, %0\n v_lshl_add_u64 %1, %1, 1, %1" : "+v"(x0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k31(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_lo_u32 %0, %2, %0\n v_add_u32 %1, %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k32(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_lo_u32 %0, %2, %0\n v_bfi_b32 %1, %2, %1, %2" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k33(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_lo_u32 %0, %2, %0\n v_cmp_gt_u64 s[50:51], %1, %1" : "+v"(x0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k34(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_lo_u32 %0, %2, %0\n v_sub_co_u32 %1, s[52:53], %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k35(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_hi_u32 %0, %2, %0\n v_mul_hi_u32 %1, %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k36(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_hi_u32 %0, %2, %0\n v_add_co_u32 %1, s[42:43], %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k37(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_hi_u32 %0, %2, %0\n v_addc_co_u32 %1, s[44:45], %2, %1, s[46:47]" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k38(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_hi_u32 %0, %2, %0\n v_cndmask_b32_e64 %1, %2, %1, s[48:49]" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k39(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_hi_u32 %0, %2, %0\n v_add3_u32 %1, %2, %1, %2" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k40(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_hi_u32 %0, %2, %0\n v_lshl_add_u64 %1, %1, 1, %1" : "+v"(x0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k41(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_hi_u32 %0, %2, %0\n v_add_u32 %1, %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k42(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_hi_u32 %0, %2, %0\n v_bfi_b32 %1, %2, %1, %2" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k43(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_hi_u32 %0, %2, %0\n v_cmp_gt_u64 s[50:51], %1, %1" : "+v"(x0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k44(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_hi_u32 %0, %2, %0\n v_sub_co_u32 %1, s[52:53], %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k45(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_co_u32 %0, s[42:43], %2, %0\n v_add_co_u32 %1, s[42:43], %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k46(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_co_u32 %0, s[42:43], %2, %0\n v_addc_co_u32 %1, s[44:45], %2, %1, s[46:47]" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k47(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_co_u32 %0, s[42:43], %2, %0\n v_cndmask_b32_e64 %1, %2, %1, s[48:49]" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k48(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_co_u32 %0, s[42:43], %2, %0\n v_add3_u32 %1, %2, %1, %2" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k49(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_co_u32 %0, s[42:43], %2, %0\n v_lshl_add_u64 %1, %1, 1, %1" : "+v"(x0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k50(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_co_u32 %0, s[42:43], %2, %0\n v_add_u32 %1, %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k51(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_co_u32 %0, s[42:43], %2, %0\n v_bfi_b32 %1, %2, %1, %2" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k52(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_co_u32 %0, s[42:43], %2, %0\n v_cmp_gt_u64 s[50:51], %1, %1" : "+v"(x0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k53(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_co_u32 %0, s[42:43], %2, %0\n v_sub_co_u32 %1, s[52:53], %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k54(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_addc_co_u32 %0, s[44:45], %2, %0, s[46:47]\n v_addc_co_u32 %1, s[44:45], %2, %1, s[46:47]" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k55(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_addc_co_u32 %0, s[44:45], %2, %0, s[46:47]\n v_cndmask_b32_e64 %1, %2, %1, s[48:49]" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k56(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_addc_co_u32 %0, s[44:45], %2, %0, s[46:47]\n v_add3_u32 %1, %2, %1, %2" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k57(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_addc_co_u32 %0, s[44:45], %2, %0, s[46:47]\n v_lshl_add_u64 %1, %1, 1, %1" : "+v"(x0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k58(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_addc_co_u32 %0, s[44:45], %2, %0, s[46:47]\n v_add_u32 %1, %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k59(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_addc_co_u32 %0, s[44:45], %2, %0, s[46:47]\n v_bfi_b32 %1, %2, %1, %2" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k60(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_addc_co_u32 %0, s[44:45], %2, %0, s[46:47]\n v_cmp_gt_u64 s[50:51], %1, %1" : "+v"(x0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k61(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_addc_co_u32 %0, s[44:45], %2, %0, s[46:47]\n v_sub_co_u32 %1, s[52:53], %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k62(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_cndmask_b32_e64 %0, %2, %0, s[48:49]\n v_cndmask_b32_e64 %1, %2, %1, s[48:49]" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k63(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_cndmask_b32_e64 %0, %2, %0, s[48:49]\n v_add3_u32 %1, %2, %1, %2" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k64(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_cndmask_b32_e64 %0, %2, %0, s[48:49]\n v_lshl_add_u64 %1, %1, 1, %1" : "+v"(x0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k65(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_cndmask_b32_e64 %0, %2, %0, s[48:49]\n v_add_u32 %1, %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k66(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_cndmask_b32_e64 %0, %2, %0, s[48:49]\n v_bfi_b32 %1, %2, %1, %2" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k67(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_cndmask_b32_e64 %0, %2, %0, s[48:49]\n v_cmp_gt_u64 s[50:51], %1, %1" : "+v"(x0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k68(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_cndmask_b32_e64 %0, %2, %0, s[48:49]\n v_sub_co_u32 %1, s[52:53], %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k69(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add3_u32 %0, %2, %0, %2\n v_add3_u32 %1, %2, %1, %2" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k70(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add3_u32 %0, %2, %0, %2\n v_lshl_add_u64 %1, %1, 1, %1" : "+v"(x0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k71(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add3_u32 %0, %2, %0, %2\n v_add_u32 %1, %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k72(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add3_u32 %0, %2, %0, %2\n v_bfi_b32 %1, %2, %1, %2" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k73(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add3_u32 %0, %2, %0, %2\n v_cmp_gt_u64 s[50:51], %1, %1" : "+v"(x0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k74(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add3_u32 %0, %2, %0, %2\n v_sub_co_u32 %1, s[52:53], %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k75(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_lshl_add_u64 %0, %0, 1, %0\n v_lshl_add_u64 %1, %1, 1, %1" : "+v"(y0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k76(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_lshl_add_u64 %0, %0, 1, %0\n v_add_u32 %1, %2, %1" : "+v"(y0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k77(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_lshl_add_u64 %0, %0, 1, %0\n v_bfi_b32 %1, %2, %1, %2" : "+v"(y0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k78(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_lshl_add_u64 %0, %0, 1, %0\n v_cmp_gt_u64 s[50:51], %1, %1" : "+v"(y0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k79(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_lshl_add_u64 %0, %0, 1, %0\n v_sub_co_u32 %1, s[52:53], %2, %1" : "+v"(y0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k80(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_u32 %0, %2, %0\n v_add_u32 %1, %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k81(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_u32 %0, %2, %0\n v_bfi_b32 %1, %2, %1, %2" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k82(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_u32 %0, %2, %0\n v_cmp_gt_u64 s[50:51], %1, %1" : "+v"(x0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k83(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_u32 %0, %2, %0\n v_sub_co_u32 %1, s[52:53], %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k84(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_bfi_b32 %0, %2, %0, %2\n v_bfi_b32 %1, %2, %1, %2" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k85(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_bfi_b32 %0, %2, %0, %2\n v_cmp_gt_u64 s[50:51], %1, %1" : "+v"(x0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k86(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_bfi_b32 %0, %2, %0, %2\n v_sub_co_u32 %1, s[52:53], %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k87(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_cmp_gt_u64 s[50:51], %0, %0\n v_cmp_gt_u64 s[50:51], %1, %1" : "+v"(y0[i]), "+v"(y1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k88(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_cmp_gt_u64 s[50:51], %0, %0\n v_sub_co_u32 %1, s[52:53], %2, %1" : "+v"(y0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k89(uint32_t* out, uint32_t seed) {
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) { x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_sub_co_u32 %0, s[52:53], %2, %0\n v_sub_co_u32 %1, s[52:53], %2, %1" : "+v"(x0[i]), "+v"(x1[i]) : "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53");
  }
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <typename F> float run(F f, uint32_t* d, int blocks) {
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  f<<<blocks, 256>>>(d, 3); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) f<<<blocks, 256>>>(d, 3 + r);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 3; double blk = (double)blocks * 256 * ITERS * 8 / 64;  // wave-iterations
  return (ms * 1e-3 * 2.4e9 * 1024) / blk; }
int main() { int blocks = 256 * 8 * 2; uint32_t* d; (void)hipMalloc(&d, blocks * 256 * 4);
  printf("%-16s %6.2f cyc\n", "mad64", run(k0, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_lo", run(k1, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_hi", run(k2, d, blocks));
  printf("%-16s %6.2f cyc\n", "add_co", run(k3, d, blocks));
  printf("%-16s %6.2f cyc\n", "addc", run(k4, d, blocks));
  printf("%-16s %6.2f cyc\n", "cnd", run(k5, d, blocks));
  printf("%-16s %6.2f cyc\n", "add3", run(k6, d, blocks));
  printf("%-16s %6.2f cyc\n", "lsh64", run(k7, d, blocks));
  printf("%-16s %6.2f cyc\n", "add", run(k8, d, blocks));
  printf("%-16s %6.2f cyc\n", "bfi", run(k9, d, blocks));
  printf("%-16s %6.2f cyc\n", "cmp64", run(k10, d, blocks));
  printf("%-16s %6.2f cyc\n", "sub64", run(k11, d, blocks));
  printf("%-16s %6.2f cyc\n", "mad64+mad64", run(k12, d, blocks));
  printf("%-16s %6.2f cyc\n", "mad64+mul_lo", run(k13, d, blocks));
  printf("%-16s %6.2f cyc\n", "mad64+mul_hi", run(k14, d, blocks));
  printf("%-16s %6.2f cyc\n", "mad64+add_co", run(k15, d, blocks));
  printf("%-16s %6.2f cyc\n", "mad64+addc", run(k16, d, blocks));
  printf("%-16s %6.2f cyc\n", "mad64+cnd", run(k17, d, blocks));
  printf("%-16s %6.2f cyc\n", "mad64+add3", run(k18, d, blocks));
  printf("%-16s %6.2f cyc\n", "mad64+lsh64", run(k19, d, blocks));
  printf("%-16s %6.2f cyc\n", "mad64+add", run(k20, d, blocks));
  printf("%-16s %6.2f cyc\n", "mad64+bfi", run(k21, d, blocks));
  printf("%-16s %6.2f cyc\n", "mad64+cmp64", run(k22, d, blocks));
  printf("%-16s %6.2f cyc\n", "mad64+sub64", run(k23, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_lo+mul_lo", run(k24, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_lo+mul_hi", run(k25, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_lo+add_co", run(k26, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_lo+addc", run(k27, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_lo+cnd", run(k28, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_lo+add3", run(k29, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_lo+lsh64", run(k30, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_lo+add", run(k31, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_lo+bfi", run(k32, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_lo+cmp64", run(k33, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_lo+sub64", run(k34, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_hi+mul_hi", run(k35, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_hi+add_co", run(k36, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_hi+addc", run(k37, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_hi+cnd", run(k38, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_hi+add3", run(k39, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_hi+lsh64", run(k40, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_hi+add", run(k41, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_hi+bfi", run(k42, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_hi+cmp64", run(k43, d, blocks));
  printf("%-16s %6.2f cyc\n", "mul_hi+sub64", run(k44, d, blocks));
  printf("%-16s %6.2f cyc\n", "add_co+add_co", run(k45, d, blocks));
  printf("%-16s %6.2f cyc\n", "add_co+addc", run(k46, d, blocks));
  printf("%-16s %6.2f cyc\n", "add_co+cnd", run(k47, d, blocks));
  printf("%-16s %6.2f cyc\n", "add_co+add3", run(k48, d, blocks));
  printf("%-16s %6.2f cyc\n", "add_co+lsh64", run(k49, d, blocks));
  printf("%-16s %6.2f cyc\n", "add_co+add", run(k50, d, blocks));
  printf("%-16s %6.2f cyc\n", "add_co+bfi", run(k51, d, blocks));
  printf("%-16s %6.2f cyc\n", "add_co+cmp64", run(k52, d, blocks));
  printf("%-16s %6.2f cyc\n", "add_co+sub64", run(k53, d, blocks));
  printf("%-16s %6.2f cyc\n", "addc+addc", run(k54, d, blocks));
  printf("%-16s %6.2f cyc\n", "addc+cnd", run(k55, d, blocks));
  printf("%-16s %6.2f cyc\n", "addc+add3", run(k56, d, blocks));
  printf("%-16s %6.2f cyc\n", "addc+lsh64", run(k57, d, blocks));
  printf("%-16s %6.2f cyc\n", "addc+add", run(k58, d, blocks));
  printf("%-16s %6.2f cyc\n", "addc+bfi", run(k59, d, blocks));
  printf("%-16s %6.2f cyc\n", "addc+cmp64", run(k60, d, blocks));
  printf("%-16s %6.2f cyc\n", "addc+sub64", run(k61, d, blocks));
  printf("%-16s %6.2f cyc\n", "cnd+cnd", run(k62, d, blocks));
  printf("%-16s %6.2f cyc\n", "cnd+add3", run(k63, d, blocks));
  printf("%-16s %6.2f cyc\n", "cnd+lsh64", run(k64, d, blocks));
  printf("%-16s %6.2f cyc\n", "cnd+add", run(k65, d, blocks));
  printf("%-16s %6.2f cyc\n", "cnd+bfi", run(k66, d, blocks));
  printf("%-16s %6.2f cyc\n", "cnd+cmp64", run(k67, d, blocks));
  printf("%-16s %6.2f cyc\n", "cnd+sub64", run(k68, d, blocks));
  printf("%-16s %6.2f cyc\n", "add3+add3", run(k69, d, blocks));
  printf("%-16s %6.2f cyc\n", "add3+lsh64", run(k70, d, blocks));
  printf("%-16s %6.2f cyc\n", "add3+add", run(k71, d, blocks));
  printf("%-16s %6.2f cyc\n", "add3+bfi", run(k72, d, blocks));
  printf("%-16s %6.2f cyc\n", "add3+cmp64", run(k73, d, blocks));
  printf("%-16s %6.2f cyc\n", "add3+sub64", run(k74, d, blocks));
  printf("%-16s %6.2f cyc\n", "lsh64+lsh64", run(k75, d, blocks));
  printf("%-16s %6.2f cyc\n", "lsh64+add", run(k76, d, blocks));
  printf("%-16s %6.2f cyc\n", "lsh64+bfi", run(k77, d, blocks));
  printf("%-16s %6.2f cyc\n", "lsh64+cmp64", run(k78, d, blocks));
  printf("%-16s %6.2f cyc\n", "lsh64+sub64", run(k79, d, blocks));
  printf("%-16s %6.2f cyc\n", "add+add", run(k80, d, blocks));
  printf("%-16s %6.2f cyc\n", "add+bfi", run(k81, d, blocks));
  printf("%-16s %6.2f cyc\n", "add+cmp64", run(k82, d, blocks));
  printf("%-16s %6.2f cyc\n", "add+sub64", run(k83, d, blocks));
  printf("%-16s %6.2f cyc\n", "bfi+bfi", run(k84, d, blocks));
  printf("%-16s %6.2f cyc\n", "bfi+cmp64", run(k85, d, blocks));
  printf("%-16s %6.2f cyc\n", "bfi+sub64", run(k86, d, blocks));
  printf("%-16s %6.2f cyc\n", "cmp64+cmp64", run(k87, d, blocks));
  printf("%-16s %6.2f cyc\n", "cmp64+sub64", run(k88, d, blocks));
  printf("%-16s %6.2f cyc\n", "sub64+sub64", run(k89, d, blocks));
  return 0; }
