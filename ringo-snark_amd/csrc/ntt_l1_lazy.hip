// ntt_l1_lazy.hip -- dispatch of the lazy single-word pass kernels (ntt64.hpp) for the shapes
// they cover: N = 2^16 as two 8-stage passes, q < 2^63 with q mod 2^32 == 1 (the config-2
// jindo-modulus prime 47104^4 + 1 and every other p - 1 = b^(2^e) with b even).  Other shapes
// keep the generic kernels of ntt_kernels.hpp.  RINGO_NTT_KERNEL=r* forces the generic path
// (experiments build only, common.hpp).
#include "ntt64.hpp"
#include "ntt_plan.hpp"

namespace rg {

static bool lazy_disabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = knob(Knob::NttKernel);
    v = (e && e[0] == 'r') ? 1 : 0;
  }
  return v == 1;
}

// ROW passes tile the same row of 16 polynomials when the chunk allows it (RP, twiddles
// shared by the whole tile); otherwise 16 consecutive rows of one polynomial
template <bool INV, bool COL, bool SCALE, bool CANON>
static rg_status launch64(const Ntt64Args& a, size_t polys, hipStream_t st) {
  const long long tiles = a.total_sub / 16;
  if (measure_probe() == 4) {  // bench.py's compute floor (rg_set_probe, experiments build): no HBM data movement
    if (!COL && polys % 16 == 0)
      hipLaunchKernelGGL((ntt16_pass<INV, COL, SCALE, CANON, true, 1, 4>), dim3((unsigned)tiles), dim3(512), 0, st, a);
    else
      hipLaunchKernelGGL((ntt16_pass<INV, COL, SCALE, CANON, false, 1, 4>), dim3((unsigned)tiles), dim3(512), 0, st, a);
    return check_launch("ntt16_pass (probe)");
  }
  if (!COL && polys % 16 == 0)
    hipLaunchKernelGGL((ntt16_pass<INV, COL, SCALE, CANON, true>), dim3((unsigned)tiles), dim3(512), 0, st, a);
  else
    hipLaunchKernelGGL((ntt16_pass<INV, COL, SCALE, CANON, false>), dim3((unsigned)tiles), dim3(512), 0, st, a);
  return check_launch("ntt16_pass");
}

rg_status ntt64_run(const NttLaunch& p, hipStream_t st, bool* handled) {
  *handled = false;
  if (!p.shoup || p.logN != 16 || p.npasses != 2 || p.passes[0].P != 8 || p.passes[1].P != 8) return RG_OK;
  const uint64_t q = p.q[0];
  if ((uint32_t)q != 1u || (q >> 63) != 0 || lazy_disabled()) return RG_OK;
  *handled = true;
  const size_t N = (size_t)1 << p.logN;
  Ntt64Args a{};
  a.tw = p.tw;
  a.q = q;
  a.q2 = 2 * q;
  a.nqhi = 0u - (uint32_t)(q >> 32);
  a.ninv = p.nsc[0];
  a.ninv_p = p.nsc_sh;
  a.w1n = p.w1n[0];
  a.w1n_p = p.w1n_sh;
  a.logN = p.logN;
  static size_t chunk_polys = 0;
  if (!chunk_polys) {  // RINGO_NTT_CHUNK_MB bounds the polys per pass pair (default: whole batch)
    const char* e = knob(Knob::NttChunkMb);
    chunk_polys = e ? std::max<size_t>(1, ((size_t)atoi(e) << 20) / (N * 8)) : ~(size_t)0 >> 1;
  }
  for (size_t b0 = 0; b0 < p.batch; b0 += chunk_polys) {
    const size_t nb = std::min(chunk_polys, p.batch - b0);
    a.total_sub = (long long)(nb * (N >> 8));
    if (!p.inv) {
      a.in = p.in + b0 * N;
      a.out = p.out + b0 * N;
      a.G0 = 0;
      a.rev = 0;
      RG_TRY((launch64<false, true, false, false>(a, nb, st)));
      a.in = a.out;
      a.G0 = 8;
      a.rev = 1;  // reverse tile order: reads what the first pass wrote last first (ntt64.hpp)
      RG_TRY((launch64<false, false, false, true>(a, nb, st)));
    } else {
      a.in = p.in + b0 * N;
      a.out = p.out + b0 * N;
      a.G0 = 8;
      a.rev = 0;
      RG_TRY((launch64<true, false, false, false>(a, nb, st)));
      a.in = a.out;
      a.G0 = 0;
      a.rev = 1;  // reverse tile order: reads what the first pass wrote last first (ntt64.hpp)
      RG_TRY((launch64<true, true, true, true>(a, nb, st)));
    }
  }
  return RG_OK;
}

}  // namespace rg
