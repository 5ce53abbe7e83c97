// Pass-kernel lab: times candidate N = 2^16, L = 1 pass kernels against libringo's production
// transform on the same device buffers and checks them bit-exactly against it.
// Build: make -C tools/nttlab   Run (GPU box): tools/nttlab/pass_lab [batch]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#include "../../include/ringo.h"
#include "../../ringo-snark_amd/csrc/ntt64.hpp"
using namespace rg;

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      exit(1);                                                           \
    }                                                                    \
  } while (0)
#define RK(x)                                                         \
  do {                                                                \
    if ((x) != 0) {                                                   \
      printf("ringo error %s at %d\n", rg_last_error(), __LINE__); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)


// min and median over `reps` timed repetitions of fn (one event pair per repetition)
template <class F>
static void time_reps(F fn, int reps, float& tmin, float& tmed) {
  std::vector<float> v;
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  fn();
  for (int k = 0; k < reps; ++k) {
    CK(hipEventRecord(a));
    fn();
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    v.push_back(ms);
  }
  std::sort(v.begin(), v.end());
  tmin = v[0];
  tmed = v[v.size() / 2];
}

static uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) { return (unsigned __int128)a * b % q; }
static uint64_t powmod(uint64_t a, uint64_t e, uint64_t q) {
  uint64_t r = 1;
  while (e) {
    if (e & 1) r = mulmod(r, a, q);
    a = mulmod(a, a, q);
    e >>= 1;
  }
  return r;
}

template <bool INV, bool COL, bool SCALE, bool CANON, int MINW, int PROBE>
static void launch(const Ntt64Args& a, int grid) {
  (void)grid;
  hipLaunchKernelGGL((ntt16_pass<INV, COL, SCALE, CANON, (PROBE & 512) != 0, MINW, (PROBE & 255)>), dim3((unsigned)(a.total_sub / 16)), dim3(512), 0, 0, a);
}

template <int MINW, int PROBE = 0>
static void run_variant(const char* name, Ntt64Args base, const uint64_t* d_tw, const uint64_t* d_twi, uint64_t* d_x,
                        const uint64_t* d_src, const uint64_t* d_ref_fwd, size_t batch, int N, int grid_cap) {
  const size_t bytes = batch * N * 8;
  const long long tsub = (long long)batch * (N >> 8);
  const int grid = (int)std::min<long long>(tsub / 16, grid_cap);
  Ntt64Args f = base, r = base;
  f.tw = d_tw;
  f.total_sub = tsub;
  r.tw = d_twi;
  r.total_sub = tsub;
  auto fwd = [&]() {
    f.in = d_x; f.out = d_x; f.G0 = 0;
    launch<false, true, false, false, MINW, PROBE>(f, grid);
    f.G0 = 8;
    launch<false, false, false, true, MINW, PROBE>(f, grid);
  };
  auto inv = [&]() {
    r.in = d_x; r.out = d_x; r.G0 = 8;
    launch<true, false, false, false, MINW, PROBE>(r, grid);
    r.G0 = 0;
    launch<true, true, true, true, MINW, PROBE>(r, grid);
  };
  CK(hipMemcpy(d_x, d_src, bytes, hipMemcpyDeviceToDevice));
  fwd();
  CK(hipDeviceSynchronize());
  std::vector<uint64_t> got(batch * N), want(batch * N), src(batch * N);
  CK(hipMemcpy(got.data(), d_x, bytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(want.data(), d_ref_fwd, bytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(src.data(), d_src, bytes, hipMemcpyDeviceToHost));
  size_t badf = 0;
  for (size_t i = 0; i < got.size(); ++i) badf += got[i] != want[i];
  inv();
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(got.data(), d_x, bytes, hipMemcpyDeviceToHost));
  size_t badi = 0;
  for (size_t i = 0; i < got.size(); ++i) badi += got[i] != src[i];
  hipEvent_t e[5];
  for (auto& x : e) CK(hipEventCreate(&x));
  const int reps = 5;
  float tc = 0, tr = 0, tic = 0, tir = 0;
  for (int k = 0; k < reps; ++k) {
    float ms;
    f.in = d_x; f.out = d_x;
    r.in = d_x; r.out = d_x;
    CK(hipEventRecord(e[0]));
    f.G0 = 0; launch<false, true, false, false, MINW, PROBE>(f, grid);
    CK(hipEventRecord(e[1]));
    f.G0 = 8; launch<false, false, false, true, MINW, PROBE>(f, grid);
    CK(hipEventRecord(e[2]));
    r.G0 = 8; launch<true, false, false, false, MINW, PROBE>(r, grid);
    CK(hipEventRecord(e[3]));
    r.G0 = 0; launch<true, true, true, true, MINW, PROBE>(r, grid);
    CK(hipEventRecord(e[4]));
    CK(hipEventSynchronize(e[4]));
    CK(hipEventElapsedTime(&ms, e[0], e[1])); tc += ms;
    CK(hipEventElapsedTime(&ms, e[1], e[2])); tr += ms;
    CK(hipEventElapsedTime(&ms, e[2], e[3])); tir += ms;
    CK(hipEventElapsedTime(&ms, e[3], e[4])); tic += ms;
  }
  tc /= reps; tr /= reps; tic /= reps; tir /= reps;
  const double tot = tc + tr + tic + tir;
  printf("%-26s grid %5d  fwd col %7.1f row %7.1f | inv row %7.1f col %7.1f us | %.3f M NTT/s (%.1f%% HBM)  fwd %s inv %s\n",
         name, grid, tc * 1e3, tr * 1e3, tir * 1e3, tic * 1e3, 2.0 * batch / (tot * 1e-3) / 1e6,
         100.0 * 2 * batch * 2.0 * N * 8 / (tot * 1e-3) / 8e12, badf ? "MISMATCH" : "ok", badi ? "MISMATCH" : "ok");
  if (badf) printf("   fwd mismatches: %zu\n", badf);
  if (badi) printf("   inv mismatches: %zu\n", badi);
}

// fwd+inv over the whole batch in chunks of `chunk` polys (col+row per chunk), full kernels
template <int PROBE = 0, int MINW = 1>
static void run_chunked(const char* name, Ntt64Args base, const uint64_t* d_tw, const uint64_t* d_twi, uint64_t* d_x,
                        size_t batch, int N, size_t chunk) {
  Ntt64Args f = base, r = base;
  f.tw = d_tw;
  r.tw = d_twi;
  auto step = [&]() {
    for (size_t b0 = 0; b0 < batch; b0 += chunk) {
      const size_t nb = std::min(chunk, batch - b0);
      const long long tsub = (long long)nb * (N >> 8);
      const int grid = (int)(tsub / 16);
      f.in = f.out = d_x + b0 * N;
      f.total_sub = tsub;
      f.G0 = 0; launch<false, true, false, false, MINW, PROBE>(f, grid);
      f.G0 = 8; launch<false, false, false, true, MINW, PROBE>(f, grid);
    }
    for (size_t b0 = 0; b0 < batch; b0 += chunk) {
      const size_t nb = std::min(chunk, batch - b0);
      const long long tsub = (long long)nb * (N >> 8);
      const int grid = (int)(tsub / 16);
      r.in = r.out = d_x + b0 * N;
      r.total_sub = tsub;
      r.G0 = 8; launch<true, false, false, false, MINW, PROBE>(r, grid);
      r.G0 = 0; launch<true, true, true, true, MINW, PROBE>(r, grid);
    }
  };
  float ms, med;
  time_reps(step, 8, ms, med);
  printf("%-26s chunk %4zu  fwd+inv min %7.1f med %7.1f us | %.3f M NTT/s (%.1f%% HBM)\n", name, chunk, ms * 1e3,
         med * 1e3, 2.0 * batch / (ms * 1e-3) / 1e6, 100.0 * 2 * batch * 2.0 * N * 8 / (ms * 1e-3) / 8e12);
}

int main(int argc, char** argv) {
  const size_t batch = argc > 1 ? atoi(argv[1]) : 384;
  const int logN = 16, N = 1 << logN;
  const uint64_t q = 47104ull * 47104ull * 47104ull * 47104ull + 1;
  rg_field* F;
  RK(rg_field_create(1, &q, &F));
  rg_ntt* T;
  RK(rg_ntt_create(F, N, 1, &T));
  std::vector<uint64_t> tw(N), twi(N);
  uint64_t ninv_m;
  RK(rg_ntt_tables(T, tw.data(), twi.data(), &ninv_m));
  // Montgomery (x 2^64) -> plain, plus Shoup quotients
  const uint64_t rinv = powmod(powmod(2, 64, q) == 0 ? 1 : (uint64_t)(((unsigned __int128)1 << 64) % q), q - 2, q);
  std::vector<uint64_t> htw(2 * N), htwi(2 * N);
  auto shp = [&](uint64_t w) { return (uint64_t)(((unsigned __int128)w << 64) / q); };
  for (int i = 0; i < N; ++i) {
    uint64_t w = mulmod(tw[i], rinv, q), wi = mulmod(twi[i], rinv, q);
    htw[2 * i] = w; htw[2 * i + 1] = shp(w);
    htwi[2 * i] = wi; htwi[2 * i + 1] = shp(wi);
  }
  for (auto* v : {&htw, &htwi}) {  // lane-ordered ROW last-round copy (as ntt.hip finalize)
    const size_t base = v->size();
    v->resize(base + (size_t)2 * 256 * 192);
    for (int r = 0; r < 256; ++r)
      for (int tt = 0; tt < 32; ++tt) {
        for (int g = 0; g < 2; ++g) {
          const size_t src = (size_t)(1 << 14) + 64 * r + 2 * tt + g, dst = (size_t)r * 192 + 32 * g + tt;
          (*v)[base + 2 * dst] = (*v)[2 * src]; (*v)[base + 2 * dst + 1] = (*v)[2 * src + 1];
        }
        for (int j = 0; j < 4; ++j) {
          const size_t src = (size_t)(1 << 15) + 128 * r + 4 * tt + j, dst = (size_t)r * 192 + 64 + 32 * j + tt;
          (*v)[base + 2 * dst] = (*v)[2 * src]; (*v)[base + 2 * dst + 1] = (*v)[2 * src + 1];
        }
      }
  }
  const uint64_t ninv = mulmod(ninv_m, rinv, q);
  const uint64_t w1n = mulmod(htwi[2], ninv, q);
  Ntt64Args base{};
  base.q = q; base.q2 = 2 * q; base.nqhi = 0u - (uint32_t)(q >> 32);
  base.ninv = ninv; base.ninv_p = shp(ninv); base.w1n = w1n; base.w1n_p = shp(w1n);
  base.logN = logN;
  uint64_t *d_tw, *d_twi, *d_src, *d_ref, *d_x;
  const size_t bytes = batch * N * 8;
  CK(hipMalloc(&d_tw, 8 * htw.size())); CK(hipMalloc(&d_twi, 8 * htwi.size()));
  CK(hipMalloc(&d_src, bytes)); CK(hipMalloc(&d_ref, bytes)); CK(hipMalloc(&d_x, bytes));
  CK(hipMemcpy(d_tw, htw.data(), 8 * htw.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_twi, htwi.data(), 8 * htwi.size(), hipMemcpyHostToDevice));
  std::vector<uint64_t> h(batch * N);
  uint64_t s = 0x52494E47;
  for (auto& v : h) { s = s * 6364136223846793005ull + 1442695040888963407ull; v = (s >> 1) % q; }
  CK(hipMemcpy(d_src, h.data(), bytes, hipMemcpyHostToDevice));
  // production reference (+ its timing)
  CK(hipMemcpy(d_ref, d_src, bytes, hipMemcpyDeviceToDevice));
  RK(rg_ntt_fwd_dev(T, d_ref, d_ref, batch, nullptr));
  CK(hipDeviceSynchronize());
  {
    CK(hipMemcpy(d_x, d_src, bytes, hipMemcpyDeviceToDevice));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float ms, med;
    // clock ramp: per-repetition times of the first 40 production steps
    {
      hipEvent_t c0, c1;
      CK(hipEventCreate(&c0)); CK(hipEventCreate(&c1));
      printf("ramp (us):");
      for (int k = 0; k < 40; ++k) {
        CK(hipEventRecord(c0));
        RK(rg_ntt_fwd_dev(T, d_x, d_x, batch, nullptr)); RK(rg_ntt_inv_dev(T, d_x, d_x, batch, nullptr));
        CK(hipEventRecord(c1)); CK(hipEventSynchronize(c1));
        float t; CK(hipEventElapsedTime(&t, c0, c1));
        printf(" %.0f", t * 1e3);
      }
      printf("\n");
    }
    time_reps([&]() { RK(rg_ntt_fwd_dev(T, d_x, d_x, batch, nullptr)); RK(rg_ntt_inv_dev(T, d_x, d_x, batch, nullptr)); }, 8, ms, med);
    printf("%-26s fwd+inv %.1f us  | %.3f M NTT/s (%.1f%% HBM)\n", "libringo (production)", ms * 1e3,
           2.0 * batch / (ms * 1e-3) / 1e6, 100.0 * 2 * batch * 2.0 * N * 8 / (ms * 1e-3) / 8e12);
  }
  int dev = 0, cus = 256;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  (void)cus;
  for (int rep = 0; rep < 2; ++rep) {
    run_chunked<256 + 512>("ntt16 RP", base, d_tw, d_twi, d_x, batch, N, 1 << 20);
    run_chunked<256 + 512 + 4>("ntt16 RP no-HBM (compute)", base, d_tw, d_twi, d_x, batch, N, 1 << 20);
    run_variant<1, 256>("ntt16 per-pass", base, d_tw, d_twi, d_x, d_src, d_ref, batch, N, 1 << 30);
    run_variant<1, 256 + 512>("ntt16 RP per-pass", base, d_tw, d_twi, d_x, d_src, d_ref, batch, N, 1 << 30);
    run_variant<1, 256 + 512 + 1>("RP no-tw per-pass", base, d_tw, d_twi, d_x, d_src, d_ref, batch, N, 1 << 30);
    run_chunked<256>("ntt16", base, d_tw, d_twi, d_x, batch, N, 1 << 20);
    run_chunked<256 + 512>("ntt16 RP", base, d_tw, d_twi, d_x, batch, N, 1 << 20);
  }
  return 0;
}
