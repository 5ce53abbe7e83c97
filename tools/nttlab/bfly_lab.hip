// Butterfly-arithmetic lab: ALU-only ceiling (data + twiddles in registers) of candidate L = 1
// butterfly formulations for q = 47104^4 + 1 (q mod 2^32 == 1, 2^62 < q < 2^64/3).
// Prints butterflies/s and checks every variant against __int128 arithmetic on the host.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../ringo-snark_amd/csrc/ntt_kernels.hpp"
#include "../../ringo-snark_amd/csrc/ntt64.hpp"
using namespace rg;

template <int V>
__device__ __forceinline__ void bfly(uint64_t& x, uint64_t& y, uint64_t w, uint64_t wp, const Q64& Q) {
  if constexpr (V == 0) {  // current: canonical in/out
    uint64_t r = reduce2q(shoup_lazy<true>(y, w, wp, Q.q), Q.q);
    uint64_t a = x;
    x = addmod63(a, r, Q.q);
    y = submod63(a, r, Q.q);
  } else if constexpr (V == 1) {
    fwd_bfly_lazy(x, y, w, wp, Q);
  } else if constexpr (V == 2) {
    fwd_bfly_x(x, y, w, wp, Q.q2, 0u - Q.qhi);
  }
}

template <int V, int NB>
__global__ __launch_bounds__(256) void k(uint64_t* out, const uint64_t* in, const uint64_t* tws, Q64 Q, int iters) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t e[2 * NB];
  for (int i = 0; i < 2 * NB; ++i) e[i] = in[(g * 2 * NB + i) & 4095];
  uint64_t w[NB], wp[NB];
  for (int i = 0; i < NB; ++i) { w[i] = tws[2 * ((g + i) & 255)]; wp[i] = tws[2 * ((g + i) & 255) + 1]; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NB; ++i) bfly<V>(e[i], e[i + NB], w[i], wp[i], Q);
#pragma unroll
    for (int i = 0; i < NB; ++i) bfly<V>(e[2 * i], e[2 * i + 1], w[(i + 1) % NB], wp[(i + 1) % NB], Q);
  }
  for (int i = 0; i < 2 * NB; ++i) out[(size_t)g * 2 * NB + i] = e[i];
}

static uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) { return (unsigned __int128)a * b % q; }

template <int V, int NB>
void run(const char* name, uint64_t* d_out, uint64_t* d_in, uint64_t* d_tw, const uint64_t* h_in, const uint64_t* h_tw,
         Q64 Q, int canon_out) {
  const int blocks = 256 * 16, iters = 64;
  k<V, NB><<<blocks, 256>>>(d_out, d_in, d_tw, Q, iters);
  (void)hipDeviceSynchronize();
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  k<V, NB><<<blocks, 256>>>(d_out, d_in, d_tw, Q, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  const double nb = (double)blocks * 256 * iters * 2 * NB;
  // check the first 64 threads against the host
  const int T = 64;
  static uint64_t got[64 * 64];
  (void)hipMemcpy(got, d_out, sizeof(uint64_t) * T * 2 * NB, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int g = 0; g < T; ++g) {
    uint64_t e[2 * NB], w[NB];
    for (int i = 0; i < 2 * NB; ++i) e[i] = h_in[(g * 2 * NB + i) & 4095];
    for (int i = 0; i < NB; ++i) w[i] = h_tw[2 * ((g + i) & 255)];
    for (int it = 0; it < iters; ++it) {
      for (int i = 0; i < NB; ++i) {
        uint64_t t = mulmod(e[i + NB], w[i], Q.q), x = e[i];
        e[i] = (x + t) % Q.q;
        e[i + NB] = (x + Q.q - t) % Q.q;
      }
      for (int i = 0; i < NB; ++i) {
        uint64_t t = mulmod(e[2 * i + 1], w[(i + 1) % NB], Q.q), x = e[2 * i];
        e[2 * i] = (x + t) % Q.q;
        e[2 * i + 1] = (x + Q.q - t) % Q.q;
      }
    }
    for (int i = 0; i < 2 * NB; ++i) {
      uint64_t gv = got[g * 2 * NB + i];
      if (!canon_out) gv = gv % Q.q;
      bad += gv != e[i];
    }
  }
  printf("%-28s NB=%d  %.3e bfly/s  (%.1f cyc per wave-bfly)  %s\n", name, NB, nb / ms * 1e3,
         ms * 1e-3 * 2.4e9 * 1024 / (nb / 64), bad ? "MISMATCH" : "ok");
}

int main() {
  const uint64_t q = 47104ull * 47104ull * 47104ull * 47104ull + 1;
  Q64 Q = make_q64(q);
  static uint64_t h_in[4096], h_tw[512];
  uint64_t s = 0x1234567;
  for (int i = 0; i < 4096; ++i) { s = s * 6364136223846793005ull + 1442695040888963407ull; h_in[i] = (s >> 1) % q; }
  for (int i = 0; i < 256; ++i) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    h_tw[2 * i] = (s >> 1) % q;
    h_tw[2 * i + 1] = (uint64_t)(((unsigned __int128)h_tw[2 * i] << 64) / q);
  }
  uint64_t *d_in, *d_tw, *d_out;
  (void)hipMalloc(&d_in, sizeof(h_in));
  (void)hipMalloc(&d_tw, sizeof(h_tw));
  (void)hipMalloc(&d_out, (size_t)256 * 16 * 256 * 64 * 8);
  (void)hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice);
  (void)hipMemcpy(d_tw, h_tw, sizeof(h_tw), hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep) {
    run<0, 4>("current canonical", d_out, d_in, d_tw, h_in, h_tw, Q, 1);
    run<0, 8>("current canonical", d_out, d_in, d_tw, h_in, h_tw, Q, 1);
    run<1, 4>("lazy harvey (ntt64.hpp)", d_out, d_in, d_tw, h_in, h_tw, Q, 0);
    run<1, 8>("lazy harvey (ntt64.hpp)", d_out, d_in, d_tw, h_in, h_tw, Q, 0);
    run<2, 4>("lazy asm-carry", d_out, d_in, d_tw, h_in, h_tw, Q, 0);
    run<2, 8>("lazy asm-carry", d_out, d_in, d_tw, h_in, h_tw, Q, 0);
  }
  return 0;
}
