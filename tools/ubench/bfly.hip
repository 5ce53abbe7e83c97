// Microbenchmark: ceiling of the L=1 Shoup butterfly code (ntt_kernels.hpp stage8_fwd) with
// data and twiddles in registers -- no memory, no LDS, full occupancy.  Reports butterflies/s,
// to compare with the NTT pass kernels' butterfly rate (tools note in DESIGN.md).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../ringo-snark_amd/csrc/ntt_kernels.hpp"
using namespace rg;
template <bool QLO1>
__global__ __launch_bounds__(256) void k(uint64_t* out, uint64_t q, uint64_t w0, uint64_t wp0, int iters) {
  uint64_t e[16][1];
  for (int i = 0; i < 16; ++i) e[i][0] = (threadIdx.x * 7919u + i * 104729u) % q;
  uint64_t w[8], wp[8];
  for (int i = 0; i < 8; ++i) { w[i] = (w0 + i * 3) % q; wp[i] = wp0 + i; }
  for (int it = 0; it < iters; ++it) {
    stage8_fwd<8, QLO1>(e, w, wp, q);
    stage8_fwd<4, QLO1>(e, w, wp, q);
    stage8_fwd<2, QLO1>(e, w, wp, q);
    stage8_fwd<1, QLO1>(e, w, wp, q);
  }
  uint64_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= e[i][0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
int main() {
  const uint64_t q = 47104ull * 47104ull * 47104ull * 47104ull + 1;
  const uint64_t w0 = 123456789012345ull % q;
  const uint64_t wp0 = (uint64_t)(((unsigned __int128)w0 << 64) / q);
  int blocks = 256 * 8 * 4, iters = 200;
  uint64_t* d; (void)hipMalloc(&d, (size_t)blocks * 256 * 8);
  for (int rep = 0; rep < 2; ++rep) {
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    k<true><<<blocks, 256>>>(d, q, w0, wp0, iters); (void)hipDeviceSynchronize();
    (void)hipEventRecord(a); k<true><<<blocks, 256>>>(d, q, w0, wp0, iters); (void)hipEventRecord(b); (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    double bf = (double)blocks * 256 * iters * 32;
    printf("qlo1 butterflies/s = %.3e  (%.1f ms)  -> per NTT-step(1.07e9 bfly) %.3f ms\n", bf / ms * 1e3, ms, 1.07e9 / (bf / ms));
    k<false><<<blocks, 256>>>(d, q, w0, wp0, iters); (void)hipDeviceSynchronize();
    (void)hipEventRecord(a); k<false><<<blocks, 256>>>(d, q, w0, wp0, iters); (void)hipEventRecord(b); (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
    printf("generic butterflies/s = %.3e  (%.1f ms)  -> per NTT-step %.3f ms\n", bf / ms * 1e3, ms, 1.07e9 / (bf / ms));
  }
  return 0;
}
