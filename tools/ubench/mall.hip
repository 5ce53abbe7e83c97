// Microbenchmark: streaming copy bandwidth, and whether data written by one kernel is re-read
// from the Infinity Cache (MALL) by the next: copy X->Y then Y->Z at working sets 16..1024 MiB.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ __launch_bounds__(256) void copy(const ulonglong2* __restrict__ in, ulonglong2* __restrict__ out, size_t n) {
  size_t i = (size_t)blockIdx.x * 256 * 4 + threadIdx.x;
  ulonglong2 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = in[i + 256 * k];
#pragma unroll
  for (int k = 0; k < 4; ++k) out[i + 256 * k] = v[k];
}
int main() {
  const size_t maxb = (size_t)1024 << 20;
  char *x, *y, *z;
  (void)hipMalloc(&x, maxb); (void)hipMalloc(&y, maxb); (void)hipMalloc(&z, maxb);
  (void)hipMemset(x, 1, maxb); (void)hipMemset(y, 2, maxb); (void)hipMemset(z, 3, maxb);
  hipEvent_t e[3];
  for (auto& v : e) (void)hipEventCreate(&v);
  for (size_t mb : {8, 16, 32, 64, 96, 128, 192, 256, 512, 1024}) {
    const size_t b = mb << 20, n = b / 16;
    const int grid = (int)(n / 1024);
    float t1 = 0, t2 = 0;
    for (int r = 0; r < 6; ++r) {
      (void)hipMemset(z + (r & 1) * 0, 0, 1);  // perturb
      // evict: stream an unrelated 512 MiB region
      copy<<<(int)(((size_t)512 << 20) / 16 / 1024), 256>>>((ulonglong2*)(x + 0), (ulonglong2*)(z), ((size_t)512 << 20) / 16);
      (void)hipEventRecord(e[0]);
      copy<<<grid, 256>>>((ulonglong2*)x, (ulonglong2*)y, n);
      (void)hipEventRecord(e[1]);
      copy<<<grid, 256>>>((ulonglong2*)y, (ulonglong2*)z, n);
      (void)hipEventRecord(e[2]);
      (void)hipEventSynchronize(e[2]);
      float a, c;
      (void)hipEventElapsedTime(&a, e[0], e[1]);
      (void)hipEventElapsedTime(&c, e[1], e[2]);
      if (r >= 2) { t1 += a; t2 += c; }
    }
    t1 /= 4; t2 /= 4;
    printf("%5zu MiB: copy X->Y %7.1f us %6.2f TB/s (R+W) | then Y->Z %7.1f us %6.2f TB/s\n", mb, t1 * 1e3,
           2.0 * b / (t1 * 1e-3) / 1e12, t2 * 1e3, 2.0 * b / (t2 * 1e-3) / 1e12);
  }
  return 0;
}
