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
static rg_status run_passes(Ntt256Args a, const NttLaunch& p, size_t polys, hipStream_t st) {
  if (!p.inv) {
    RG_TRY((launch256<false, true, false, false, LOGN>(a, polys, st)));
    a.in = a.out;
    RG_TRY((launch256<false, false, false, true, LOGN>(a, polys, st)));
  } else {
    RG_TRY((launch256<true, false, false, false, LOGN>(a, polys, st)));
    a.in = a.out;
    RG_TRY((launch256<true, true, true, true, LOGN>(a, polys, st)));
  }
  return RG_OK;
}

// The batch as two halves, the first on the caller's stream and the second on the plan's helper
// stream: each pass is ~2.7 rounds of workgroups (3 per SIMD resident), and the halves' passes
// fill each other's last round (configs[3] fwd+inv: 182.5 -> 187.3 K NTT/s; four quarters
// alternating measured 160 K, the headline ntt16_pass split lost 1.5%: profiles/r06r_ntt_split.txt)
template <int LOGN>
static rg_status run_split(Ntt256Args a, const NttLaunch& p, hipStream_t st) {
  Aux* x = p.aux;
  if (!x || p.batch < 8 || measure_probe() == 5) return run_passes<LOGN>(a, p, p.batch, st);
  const size_t N = (size_t)1 << LOGN;
  const size_t h = (p.batch / 2 + 3) & ~(size_t)3;  // the ROW passes' RP tiles take 4 polys
  Ntt256Args b = a;
  a.total_sub = (long long)(h * (N >> 8));
  b.total_sub = (long long)((p.batch - h) * (N >> 8));
  b.in += h * N * 4;
  b.out += h * N * 4;
  std::lock_guard<std::mutex> lk(x->mu);
  RG_HIP(hipEventRecord(x->fork, st));
  RG_HIP(hipStreamWaitEvent(x->s, x->fork, 0));
  rg_status s = run_passes<LOGN>(a, p, h, st);
  if (s == RG_OK) s = run_passes<LOGN>(b, p, p.batch - h, x->s);
  // joined on every path, so the caller's stream orders whatever was queued on the helper
  const hipError_t j[2] = {hipEventRecord(x->join, x->s), hipStreamWaitEvent(st, x->join, 0)};
  for (hipError_t e : j)
    if (e != hipSuccess && s == RG_OK) {
      set_last_error(std::string("ntt256: joining the helper stream: ") + hipGetErrorString(e));
      s = RG_ERR_DEVICE;
    }
  return s;
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
  return p.logN == 16 ? run_split<16>(a, p, st) : run_split<15>(a, p, st);
}

}  // namespace rg
