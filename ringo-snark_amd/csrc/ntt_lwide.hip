// ntt_lwide.hip -- wide buckler fields (zp440: 7 limbs, zp880: 14 limbs): per-stage kernels.
#include "ntt_kernels.hpp"
namespace rg {
rg_status ntt_run_L7(const NttLaunch& p, hipStream_t st) { return run_stages<7, false>(p, st); }
rg_status ntt_run_L14(const NttLaunch& p, hipStream_t st) { return run_stages<14, false>(p, st); }
}  // namespace rg
