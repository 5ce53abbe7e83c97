// Check of the v_mfma_i32_16x16x64_i8 operand maps used by mac_mfma.hip: lane l supplies
// A[row l&15][k 16(l>>4) + i] and B[k 16(l>>4) + i][col l&15] as byte i of its 16-byte operand,
// and receives D[row 4(l>>4) + r][col l&15] in accumulator r.  Exact integer data, asymmetric.
// Also times back-to-back independent MFMAs (cycles per instruction per SIMD).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void map_kernel(const int8_t* A, const int8_t* B, int* D) {
  const int l = threadIdx.x;
  int8_t a[16], b[16];
  for (int i = 0; i < 16; ++i) {
    a[i] = A[(l & 15) * 64 + 16 * (l >> 4) + i];
    b[i] = B[(16 * (l >> 4) + i) * 16 + (l & 15)];
  }
  v4i av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  v4i c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

__global__ void rate_kernel(int iters, int* out) {
  v4i a = {(int)threadIdx.x, 3, 5, 7}, b = {11, (int)threadIdx.x, 13, 17};
  v4i c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c3, 0, 0, 0);
  }
  const v4i s = c0 + c1 + c2 + c3;
  if (s[0] == 12345) out[0] = s[1];
}

int main() {
  int8_t hA[16 * 64], hB[64 * 16];
  for (int i = 0; i < 16; ++i)
    for (int k = 0; k < 64; ++k) hA[i * 64 + k] = (int8_t)((i * 7 + k * 3 + (i * k) % 11) % 256 - 128);
  for (int k = 0; k < 64; ++k)
    for (int j = 0; j < 16; ++j) hB[k * 16 + j] = (int8_t)((k * 5 + j * 13 + (k ^ j)) % 256 - 128);
  int8_t *dA, *dB;
  int* dD;
  hipMalloc(&dA, sizeof hA);
  hipMalloc(&dB, sizeof hB);
  hipMalloc(&dD, 256 * 4);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  map_kernel<<<1, 64>>>(dA, dB, dD);
  int hD[256];
  hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      int s = 0;
      for (int k = 0; k < 64; ++k) s += hA[i * 64 + k] * hB[k * 16 + j];
      if (s != hD[i * 16 + j]) ++bad;
    }
  printf("mfma_i32_16x16x64_i8 operand/result map: %d of 256 wrong\n", bad);
  int* dO;
  hipMalloc(&dO, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000, blocks = 256 * 4 * 4;  // 4 waves per SIMD
  rate_kernel<<<blocks, 64>>>(100, dO);
  hipEventRecord(e0);
  rate_kernel<<<blocks, 64>>>(iters, dO);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double inst = (double)blocks * iters * 4;
  printf("16x16x64 i8: %.3f ms, %.2f cycles per MFMA per SIMD at 2.4 GHz, %.0f TOPS\n", ms,
         ms * 1e-3 * 2.4e9 * 1024 / inst, inst * 32768 / (ms * 1e-3) / 1e12);
  return bad != 0;
}
