// ntt_l2.hip -- two-limb fields (buckler zp110, examples/mult 128-bit).
#include "ntt_kernels.hpp"
namespace rg {
rg_status ntt_run_L2(const NttLaunch& p, hipStream_t st) {
  return p.tiled ? run_tiled<2, false>(p, st) : run_stages<2, false>(p, st);
}
}  // namespace rg
