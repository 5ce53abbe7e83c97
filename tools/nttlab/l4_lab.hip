// L = 4 lab: ntt256_pass (ntt256.hpp) at N = 2^16, q255, vs libringo's generic multi-limb path:
// bit-exact check of fwd and inv, and timing.  Run (GPU box): tools/nttlab/l4_lab [batch]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/ringo.h"
#include "../../ringo-snark_amd/csrc/ntt256.hpp"
using namespace rg;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define RK(x) do { if ((x) != 0) { printf("ringo error %s at %d\n", rg_last_error(), __LINE__); exit(1); } } while (0)

template <class F>
static float time_min(F fn, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  fn();
  float best = 1e30f;
  for (int k = 0; k < reps; ++k) {
    CK(hipEventRecord(a)); fn(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); best = std::min(best, ms);
  }
  return best;
}

int main(int argc, char** argv) {
  const size_t batch = argc > 1 ? atoi(argv[1]) : 64;
  const int N = 1 << 16;
  const uint64_t q[4] = {1ull, 0xd65643d9e6fb6555ull ^ 0ull, 0ull, 0ull};
  // q255 = 0x430d45996b62afc2 d65643d9e6fb6555 8e9630dc8c373281 0000000000000001
  const uint64_t qq[4] = {0x0000000000000001ull, 0x8e9630dc8c373281ull, 0xd65643d9e6fb6555ull, 0x430d45996b62afc2ull};
  (void)q;
  rg_field* F;
  RK(rg_field_create(4, qq, &F));
  rg_ntt* T;
  RK(rg_ntt_create(F, N, 1, &T));
  std::vector<uint64_t> tw(4 * N), twi(4 * N), ninv(4), w1n(4);
  RK(rg_ntt_tables(T, tw.data(), twi.data(), ninv.data()));
  RK(rg_vec(F, RG_VEC_MUL, w1n.data(), &twi[4], ninv.data(), 1));
  Ntt256Args base{};
  for (int i = 0; i < 4; ++i) {
    base.q[2 * i] = (uint32_t)qq[i]; base.q[2 * i + 1] = (uint32_t)(qq[i] >> 32);
    const unsigned __int128 two = (unsigned __int128)qq[i] * 2;  // per-limb doubling with carry below
    (void)two;
    base.w1n[2 * i] = (uint32_t)w1n[i]; base.w1n[2 * i + 1] = (uint32_t)(w1n[i] >> 32);
  }
  uint32_t c = 0;
  for (int i = 0; i < 8; ++i) { uint64_t v = 2ull * base.q[i] + c; base.q2[i] = (uint32_t)v; c = (uint32_t)(v >> 32); }
  uint64_t *d_tw, *d_twi, *d_src, *d_ref, *d_x;
  const size_t bytes = batch * N * 32;
  CK(hipMalloc(&d_tw, 32 * N)); CK(hipMalloc(&d_twi, 32 * N));
  CK(hipMalloc(&d_src, bytes)); CK(hipMalloc(&d_ref, bytes)); CK(hipMalloc(&d_x, bytes));
  CK(hipMemcpy(d_tw, tw.data(), 32 * N, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_twi, twi.data(), 32 * N, hipMemcpyHostToDevice));
  std::vector<uint64_t> h(batch * N * 4);
  uint64_t s = 0x1234;
  for (size_t i = 0; i < h.size(); ++i) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    h[i] = (i % 4 == 3) ? ((s >> 1) & 0x3fffffffffffffffull) : s;  // top limb < 2^62 < q's
  }
  CK(hipMemcpy(d_src, h.data(), bytes, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ref, d_src, bytes, hipMemcpyDeviceToDevice));
  RK(rg_ntt_fwd_dev(T, d_ref, d_ref, batch, nullptr));
  CK(hipDeviceSynchronize());
  const float tprod = time_min([&]() { RK(rg_ntt_fwd_dev(T, d_x, d_x, batch, nullptr)); RK(rg_ntt_inv_dev(T, d_x, d_x, batch, nullptr)); }, 5);
  printf("libringo L=4 (generic)  fwd+inv %8.1f us  %.1f K NTT/s\n", tprod * 1e3, 2.0 * batch / (tprod * 1e-3) / 1e3);
  const bool rp = batch % 4 == 0;
  auto launch = [&](bool inv, bool col, Ntt256Args a) {
    const unsigned grid = (unsigned)(batch * 64);
    if (!inv && col) hipLaunchKernelGGL((ntt256_pass<false, true, false, false, false>), dim3(grid), dim3(128), 0, 0, a);
    if (!inv && !col) {
      if (rp) hipLaunchKernelGGL((ntt256_pass<false, false, false, true, true>), dim3(grid), dim3(128), 0, 0, a);
      else hipLaunchKernelGGL((ntt256_pass<false, false, false, true, false>), dim3(grid), dim3(128), 0, 0, a);
    }
    if (inv && !col) {
      if (rp) hipLaunchKernelGGL((ntt256_pass<true, false, false, false, true>), dim3(grid), dim3(128), 0, 0, a);
      else hipLaunchKernelGGL((ntt256_pass<true, false, false, false, false>), dim3(grid), dim3(128), 0, 0, a);
    }
    if (inv && col) hipLaunchKernelGGL((ntt256_pass<true, true, true, true, false>), dim3(grid), dim3(128), 0, 0, a);
  };
  Ntt256Args f = base, r = base;
  f.tw = d_tw; r.tw = d_twi;
  f.in = r.in = d_x;
  f.out = r.out = d_x;
  f.total_sub = r.total_sub = (long long)batch * 256;
  auto fwd = [&]() { launch(false, true, f); launch(false, false, f); };
  auto inv = [&]() { launch(true, false, r); launch(true, true, r); };
  CK(hipMemcpy(d_x, d_src, bytes, hipMemcpyDeviceToDevice));
  fwd();
  CK(hipDeviceSynchronize());
  std::vector<uint64_t> got(h.size()), want(h.size());
  CK(hipMemcpy(got.data(), d_x, bytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(want.data(), d_ref, bytes, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < got.size(); ++i) bad += got[i] != want[i];
  inv();
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(got.data(), d_x, bytes, hipMemcpyDeviceToHost));
  size_t badi = 0;
  for (size_t i = 0; i < got.size(); ++i) badi += got[i] != h[i];
  printf("ntt256 fwd %s (%zu bad)  inv roundtrip %s (%zu bad)\n", bad ? "MISMATCH" : "ok", bad, badi ? "MISMATCH" : "ok", badi);
  hipEvent_t e[5];
  for (auto& x : e) CK(hipEventCreate(&x));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e[0])); launch(false, true, f);
    CK(hipEventRecord(e[1])); launch(false, false, f);
    CK(hipEventRecord(e[2])); launch(true, false, r);
    CK(hipEventRecord(e[3])); launch(true, true, r);
    CK(hipEventRecord(e[4])); CK(hipEventSynchronize(e[4]));
    float t[4];
    for (int i = 0; i < 4; ++i) CK(hipEventElapsedTime(&t[i], e[i], e[i + 1]));
    printf("ntt256 passes us: fwd col %.1f row %.1f | inv row %.1f col %.1f\n", t[0] * 1e3, t[1] * 1e3, t[2] * 1e3, t[3] * 1e3);
  }
  const float tn = time_min([&]() { fwd(); inv(); }, 5);
  printf("ntt256                  fwd+inv %8.1f us  %.1f K NTT/s  (%.2f TB/s algorithmic)\n", tn * 1e3,
         2.0 * batch / (tn * 1e-3) / 1e3, 2.0 * batch * 2 * N * 32 / (tn * 1e-3) / 1e12);
  return 0;
}
