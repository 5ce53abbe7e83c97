// ntt_lwide.hip -- wide buckler fields (zp440: 7 limbs, zp880: 14 limbs): the LDS-tiled pass
// kernel of ntt_wide.hpp for N <= 2^16 (two passes: COL then ROW; one pass for N <= 2^8), the
// per-stage kernels of ntt_kernels.hpp for larger ranks or a modulus without a spare top bit.
#include "ntt_kernels.hpp"
#include "ntt_wide.hpp"

namespace rg {

template <int L>
static rg_status wide_run(const NttLaunch& p, hipStream_t st) {
  const int logN = p.logN;
  const bool spare = (p.q[L - 1] >> 63) == 0;
  const char* k = knob(Knob::NttKernel);  // experiments build: RINGO_NTT_KERNEL=stage (A/B)
  if (logN < 1 || logN > 16 || !spare || (p.inv && !p.halving) || (k && k[0] == 's')) return run_stages<L, false>(p, st);
  WideArgs a;
  memset(&a, 0, sizeof(a));
  // inverse: the halved copy of twInv that ntt.hip's finalize() appends to the table
  a.tw = p.inv ? p.tw + ((size_t)1 << logN) * L : p.tw;
  for (int l = 0; l < L; ++l) {
    a.q[2 * l] = (uint32_t)p.q[l];
    a.q[2 * l + 1] = (uint32_t)(p.q[l] >> 32);
  }
  a.qinv28 = (uint32_t)p.qinv & 0x0FFFFFFFu;  // -q^-1 mod 2^64, so its low 28 bits are -q^-1 mod 2^28
  for (int k = 0; k < 64 * L / 28; ++k) {  // q in 28-bit digits
    const int bit = 28 * k, l = bit >> 6, sh = bit & 63;
    uint64_t v = p.q[l] >> sh;
    if (sh > 36 && l + 1 < L) v |= p.q[l + 1] << (64 - sh);
    a.q28[k] = (uint32_t)v & 0x0FFFFFFFu;
  }
  a.logN = logN;
  // passes in forward order: (G0, P)
  int G0s[2], Ps[2], np;
  if (logN <= 8) {
    np = 1;
    G0s[0] = 0;
    Ps[0] = logN;
  } else {
    np = 2;
    G0s[0] = 0;
    Ps[0] = logN / 2;
    G0s[1] = logN / 2;
    Ps[1] = logN - logN / 2;
  }
  const int base_cpt = 1;  // one 256-point sub-transform per workgroup at P = 8: 14 / 28 KiB of LDS, so LDS does not cap occupancy below the VGPRs
  for (int k = 0; k < np; ++k) {
    const int i = p.inv ? np - 1 - k : k;
    a.G0 = G0s[i];
    a.P = Ps[i];
    a.logS = logN - a.G0 - a.P;
    a.cpt = std::max(base_cpt, 256 >> a.P);
    if (a.logS > 0) a.cpt = std::min(a.cpt, 1 << a.logS);  // a COL tile stays inside one row of columns
    a.nsub = (long long)p.batch << (logN - a.P);
    a.in = k == 0 ? p.in : p.out;
    a.out = p.out;
    const size_t lds = (size_t)a.cpt * ((size_t)1 << a.P) * L * 8;
    const long long grid = (a.nsub + a.cpt - 1) / a.cpt;
    if (p.inv)
      hipLaunchKernelGGL((ntt_wide_pass<L, true>), dim3((unsigned)grid), dim3(kWideThreads), lds, st, a);
    else
      hipLaunchKernelGGL((ntt_wide_pass<L, false>), dim3((unsigned)grid), dim3(kWideThreads), lds, st, a);
    RG_TRY(check_launch("ntt_wide_pass"));
  }
  return RG_OK;
}

rg_status ntt_run_L7(const NttLaunch& p, hipStream_t st) { return wide_run<7>(p, st); }
rg_status ntt_run_L14(const NttLaunch& p, hipStream_t st) { return wide_run<14>(p, st); }
}  // namespace rg
