// ntt_l4_fast.hip -- dispatch of the 4-limb degree-2^16 kernels (ntt256.hpp) for q = 1 mod 2^64,
// q < 2^255 (the Jindo default prime q255).  Other 4-limb shapes keep the generic CIOS kernels
// of ntt_kernels.hpp.  RINGO_NTT_KERNEL=r... forces the generic path (A/B switch).
#include <cstdlib>

#include "ntt256.hpp"
#include "ntt_plan.hpp"

namespace rg {

template <bool INV, bool COL, bool SCALE, bool CANON>
static rg_status launch256(const Ntt256Args& a, size_t polys, hipStream_t st) {
  const unsigned grid = (unsigned)(polys * 64);  // 4 sub-transforms x 256 points per workgroup
  if (!COL && polys % 4 == 0)
    hipLaunchKernelGGL((ntt256_pass<INV, COL, SCALE, CANON, true>), dim3(grid), dim3(128), 0, st, a);
  else
    hipLaunchKernelGGL((ntt256_pass<INV, COL, SCALE, CANON, false>), dim3(grid), dim3(128), 0, st, a);
  return check_launch("ntt256_pass");
}

rg_status ntt256_run(const NttLaunch& p, hipStream_t st, bool* handled) {
  *handled = false;
  if (p.logN != 16 || p.npasses != 2 || p.passes[0].P != 8 || p.passes[1].P != 8) return RG_OK;
  if (p.q[0] != 1 || (p.q[3] >> 63) != 0) return RG_OK;
  const char* e = getenv("RINGO_NTT_KERNEL");
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
  if (!p.inv) {
    RG_TRY((launch256<false, true, false, false>(a, p.batch, st)));
    a.in = a.out;
    RG_TRY((launch256<false, false, false, true>(a, p.batch, st)));
  } else {
    RG_TRY((launch256<true, false, false, false>(a, p.batch, st)));
    a.in = a.out;
    RG_TRY((launch256<true, true, true, true>(a, p.batch, st)));
  }
  return RG_OK;
}

}  // namespace rg
