// Standalone check of mac_mfma.hip: random key A [J][T][per_col] and opening B [ncols][T][per_col]
// against (sum_t A B) 2^-64 mod q on the host, per (col, j, lk).  Build:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../ringo-snark_amd/csrc -o mac_mfma_check mac_mfma_check.hip
//         ../../ringo-snark_amd/csrc/mac_mfma.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#include "mac_mfma.hpp"

namespace rg {
void set_last_error(const std::string& m) { fprintf(stderr, "error: %s\n", m.c_str()); }
}  // namespace rg

using u64 = uint64_t;
using u128 = unsigned __int128;

static u64 powmod(u64 b, u64 e, u64 q) {
  u64 r = 1;
  while (e) {
    if (e & 1) r = (u128)r * b % q;
    b = (u128)b * b % q;
    e >>= 1;
  }
  return r;
}

__global__ void fill_kernel(u64* p, long long n, u64 q, u64 seed) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    u64 z = seed + (u64)i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = (z ^ (z >> 31)) % q;
  }
}

// timing mode (configs[4] half batch: q 288230376151748609, T1 513, T2 32, J 16, ncols 2304,
// per_col 512): the opening filled on the device, the kernel timed with events
static int timing(u64 q, int T1, int T2, int J, long long ncols, long long per_col, int iters) {
  const int d = 256, T = T1 + T2;
  const int NB = rg::mac_mfma_nb(&q, 1, J, T, d);
  if (!NB) return 1;
  u64 *dA1, *dA2, *dB1, *dB2, *dOut;
  const long long nA1 = (long long)J * T1 * per_col, nA2 = (long long)J * T2 * per_col, nB1 = ncols * T1 * per_col,
                  nB2 = ncols * T2 * per_col;
  hipMalloc(&dA1, nA1 * 8);
  hipMalloc(&dA2, nA2 * 8 + 8);
  hipMalloc(&dB1, nB1 * 8);
  hipMalloc(&dB2, nB2 * 8 + 8);
  hipMalloc(&dOut, ncols * J * per_col * 8);
  fill_kernel<<<4096, 256>>>(dA1, nA1, q, 1);
  fill_kernel<<<4096, 256>>>(dA2, nA2, q, 2);
  fill_kernel<<<4096, 256>>>(dB1, nB1, q, 3);
  fill_kernel<<<4096, 256>>>(dB2, nB2, q, 4);
  rg::MfmaPrime P{};
  P.q = q;
  P.rinv = powmod(powmod(2, 64 % (q - 1), q), q - 2, q);
  P.rinv_sh = (u64)(((u128)P.rinv << 64) / q);
  P.one_sh = (u64)(((u128)1 << 64) / q);
  rg::DevBuf key;
  if (rg::mac_mfma_key_dev(dA1, T1, dA2, T2, J, per_col, d, NB, &P, 1, key, 0) != RG_OK) return 2;
  rg::MfmaMacArgs a{};
  a.per_col = per_col;
  a.ncols = ncols;
  a.J = J;
  a.T1 = T1;
  a.T2 = T2;
  a.Tc = (T + 7) / 8;
  rg::mac_mfma_key_ptrs(key, per_col, T, &a.Ak, &a.corr);
  a.B1 = dB1;
  a.b1_col = (long long)T1 * per_col;
  a.b1_term = per_col;
  a.B2 = dB2;
  a.b2_col = (long long)T2 * per_col;
  a.b2_term = per_col;
  a.out = dOut;
  a.d = d;
  for (int l = 0; l < 4; ++l) a.P[l] = P;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) rg::launch_mac_mfma(a, NB, 0);
  hipEventRecord(e0);
  for (int i = 0; i < iters; ++i) rg::launch_mac_mfma(a, NB, 0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= iters;
  const double gb = (double)(nB1 + nB2) * 8 / 1e9;
  printf("NB=%d T=%d J=%d ncols=%lld per_col=%lld: %.3f ms per launch, opening %.2f GB -> %.2f TB/s\n", NB, T, J,
         ncols, per_col, ms, gb, gb / ms);
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 7)
    return timing(strtoull(argv[1], 0, 0), atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), atoll(argv[5]), atoll(argv[6]),
                  atoi(argv[7]));
  const u64 q = argc > 1 ? strtoull(argv[1], 0, 0) : 288230376151736833ull;
  const int T1 = argc > 2 ? atoi(argv[2]) : 33, T2 = argc > 3 ? atoi(argv[3]) : 32, J = argc > 4 ? atoi(argv[4]) : 10;
  const long long ncols = argc > 5 ? atoll(argv[5]) : 19;
  const int d = 256, nl = 1;
  const long long per_col = (long long)nl * d;
  const int T = T1 + T2;
  std::mt19937_64 rng(42);
  std::vector<u64> A1((size_t)J * T1 * per_col), A2((size_t)J * T2 * per_col), B1((size_t)ncols * T1 * per_col),
      B2((size_t)ncols * T2 * per_col);
  auto r = [&](void) -> u64 {
    const u64 k = rng() % 8;
    return k == 0 ? 0 : k == 1 ? q - 1 : rng() % q;
  };
  for (auto& x : A1) x = r();
  for (auto& x : A2) x = r();
  for (auto& x : B1) x = r();
  for (auto& x : B2) x = r();
  const int NB = rg::mac_mfma_nb(&q, 1, J, T, d);
  printf("q=%llu T=%d J=%d ncols=%lld NB=%d\n", (unsigned long long)q, T, J, ncols, NB);
  if (!NB) return 1;
  u64 *dA1, *dA2, *dB1, *dB2, *dOut;
  hipMalloc(&dA1, A1.size() * 8);
  hipMalloc(&dA2, A2.size() * 8 + 8);
  hipMalloc(&dB1, B1.size() * 8);
  hipMalloc(&dB2, B2.size() * 8 + 8);
  hipMalloc(&dOut, (size_t)ncols * J * per_col * 8);
  hipMemcpy(dA1, A1.data(), A1.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dA2, A2.data(), A2.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dB1, B1.data(), B1.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dB2, B2.data(), B2.size() * 8, hipMemcpyHostToDevice);
  rg::MfmaPrime P{};
  P.q = q;
  P.rinv = powmod(powmod(2, 64 % (q - 1), q), q - 2, q);  // 2^-64
  P.rinv_sh = (u64)(((u128)P.rinv << 64) / q);
  P.one_sh = (u64)(((u128)1 << 64) / q);
  rg::DevBuf key;
  if (rg::mac_mfma_key_dev(dA1, T1, dA2, T2, J, per_col, d, NB, &P, 1, key, 0) != RG_OK) return 2;
  rg::MfmaMacArgs a{};
  a.per_col = per_col;
  a.ncols = ncols;
  a.J = J;
  a.T1 = T1;
  a.T2 = T2;
  a.Tc = (T + 7) / 8;
  rg::mac_mfma_key_ptrs(key, per_col, T, &a.Ak, &a.corr);
  a.B1 = dB1;
  a.b1_col = (long long)T1 * per_col;
  a.b1_term = per_col;
  a.B2 = dB2;
  a.b2_col = (long long)T2 * per_col;
  a.b2_term = per_col;
  a.out = dOut;
  a.d = d;
  a.bxor = rg::mac_mfma_bxor(NB);
  a.P[0] = P;
  if (rg::launch_mac_mfma(a, NB, 0) != RG_OK) return 3;
  std::vector<u64> out((size_t)ncols * J * per_col);
  hipMemcpy(out.data(), dOut, out.size() * 8, hipMemcpyDeviceToHost);
  long bad = 0;
  for (long long c = 0; c < ncols; ++c)
    for (int j = 0; j < J; ++j)
      for (long long lk = 0; lk < per_col; ++lk) {
        u128 s = 0;
        u64 m = 0;
        for (int t = 0; t < T; ++t) {
          const u64 av = t < T1 ? A1[((size_t)j * T1 + t) * per_col + lk] : A2[((size_t)j * T2 + t - T1) * per_col + lk];
          const u64 bv = t < T1 ? B1[((size_t)c * T1 + t) * per_col + lk] : B2[((size_t)c * T2 + t - T1) * per_col + lk];
          m = (m + (u64)((u128)av * bv % q)) % q;
        }
        (void)s;
        const u64 want = (u128)m * P.rinv % q, got = out[((size_t)c * J + j) * per_col + lk];
        if (want != got && bad++ < 8)
          printf("col %lld j %d lk %lld: got %llu want %llu\n", c, j, lk, (unsigned long long)got,
                 (unsigned long long)want);
      }
  printf("%ld of %lld wrong\n", bad, (long long)out.size());
  return bad != 0;
}
