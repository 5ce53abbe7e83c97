// ntt_l1.hip -- single-word fields (the config-2 63-bit prime): Shoup twiddle products.
#include "ntt_kernels.hpp"
namespace rg {
rg_status ntt_run_L1(const NttLaunch& p, hipStream_t st) {
  if (p.shoup) return p.tiled ? run_tiled<1, true>(p, st) : run_stages<1, true>(p, st);
  return p.tiled ? run_tiled<1, false>(p, st) : run_stages<1, false>(p, st);
}
}  // namespace rg
