// ntt_l4_fast.hip -- dispatch of the 4-limb degree-2^16 / 2^15 kernels (ntt256.hpp) for q = 1 mod 2^64,
// q < 2^255 (the Jindo default prime q255).  Other 4-limb shapes keep the generic CIOS kernels
// of ntt_kernels.hpp.  RINGO_NTT_KERNEL=r... forces the generic path (A/B switch; experiments
// build only, common.hpp).
#include "ntt256.hpp"
#include "ntt_plan.hpp"

namespace rg {

template <bool INV, bool COL, bool SCALE, bool CANON, int LOGN>
static rg_status launch256(const Ntt256Args& a, size_t polys, hipStream_t st) {
  const unsigned grid = (unsigned)(polys << (LOGN - 10));  // 1024 points (32 KiB) per workgroup
  if (LOGN == 16 && measure_probe() == 5) {  // bench.py's L = 4 compute floor (experiments build)
    if (!COL && polys % 4 == 0)
      hipLaunchKernelGGL((ntt256_pass<INV, COL, SCALE, CANON, true, LOGN, 1>), dim3(grid), dim3(128), 0, st, a);
    else
      hipLaunchKernelGGL((ntt256_pass<INV, COL, SCALE, CANON, false, LOGN, 1>), dim3(grid), dim3(128), 0, st, a);
    return check_launch("ntt256_pass (probe)");
  }
  if (!COL && polys % 4 == 0)
    hipLaunchKernelGGL((ntt256_pass<INV, COL, SCALE, CANON, true, LOGN>), dim3(grid), dim3(128), 0, st, a);
  else
    hipLaunchKernelGGL((ntt256_pass<INV, COL, SCALE, CANON, false, LOGN>), dim3(grid), dim3(128), 0, st, a);
  return check_launch("ntt256_pass");
}

template <int LOGN>
static rg_status run_passes(Ntt256Args a, const NttLaunch& p, hipStream_t st) {
  if (!p.inv) {
    RG_TRY((launch256<false, true, false, false, LOGN>(a, p.batch, st)));
    a.in = a.out;
    RG_TRY((launch256<false, false, false, true, LOGN>(a, p.batch, st)));
  } else {
    RG_TRY((launch256<true, false, false, false, LOGN>(a, p.batch, st)));
    a.in = a.out;
    RG_TRY((launch256<true, true, true, true, LOGN>(a, p.batch, st)));
  }
  return RG_OK;
}

// N = 2^16 (passes 8 + 8) and N = 2^15 (7 + 8: the Buckler witness rank of the bench)
rg_status ntt256_run(const NttLaunch& p, hipStream_t st, bool* handled) {
  *handled = false;
  if (p.npasses != 2 || p.passes[1].P != 8 || !((p.logN == 16 && p.passes[0].P == 8) || (p.logN == 15 && p.passes[0].P == 7)))
    return RG_OK;
  if (p.q[0] != 1 || (p.q[3] >> 63) != 0) return RG_OK;
  const char* e = knob(Knob::NttKernel);
  if (e && e[0] == 'r') return RG_OK;
  *handled = true;
  const size_t N = (size_t)1 << p.logN;
  Ntt256Args a{};
  a.tw = p.tw;
  uint32_t c = 0;
  for (int i = 0; i < 4; ++i) {
    a.q[2 * i] = (uint32_t)p.q[i];
    a.q[2 * i + 1] = (uint32_t)(p.q[i] >> 32);
    a.w1n[2 * i] = (uint32_t)p.w1n[i];
    a.w1n[2 * i + 1] = (uint32_t)(p.w1n[i] >> 32);
  }
  for (int i = 0; i < 8; ++i) {
    const uint64_t v = 2ull * a.q[i] + c;
    a.q2[i] = (uint32_t)v;
    c = (uint32_t)(v >> 32);
  }
  a.total_sub = (long long)(p.batch * (N >> 8));
  a.in = p.in;
  a.out = p.out;
  return p.logN == 16 ? run_passes<16>(a, p, st) : run_passes<15>(a, p, st);
}

}  // namespace rg
