// ntt_l4.hip -- four-limb fields (the Jindo default 255-bit prime, zp220, bfv 240-bit).
#include "ntt_kernels.hpp"
namespace rg {
rg_status ntt_run_L4(const NttLaunch& p, hipStream_t st) {
  return p.tiled ? run_tiled<4, false>(p, st) : run_stages<4, false>(p, st);
}
}  // namespace rg
