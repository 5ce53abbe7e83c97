// knobs_env.hip -- the experiments build's knob table (libringo_exp.so only; see
// ringo-snark_amd/csrc/common.hpp).  Knobs come from the RINGO_* environment, read once; the
// probe is per calling thread, so a probe window opened by bench.py's compute-floor leg cannot
// change launches issued from another thread.
#include <cstdlib>

#include "../../ringo-snark_amd/csrc/common.hpp"

namespace rg {
static thread_local int t_probe = 0;

const char* knob(Knob k) {
  // (round 6 removed the knobs whose kernels only an A/B run reached: RINGO_NTT_PREFETCH,
  // RINGO_NTT_WG_PER_CU, RINGO_NTT_R8_PF, RINGO_JINDO_PREP, RINGO_JINDO_PREP_W, RINGO_JINDO_EVAL and
  // RINGO_JINDO_MAC=h; tools/experiments/jindo_knob_kernels.patch, ntt_knob_kernels.patch)
  static const char* names[] = {"RINGO_NTT_KERNEL", "RINGO_NTT_CHUNK_MB", "RINGO_JINDO_MAC", "RINGO_JINDO_SPLIT",
                                "RINGO_JINDO_UNI_TRIES"};
  static_assert(sizeof(names) / sizeof(names[0]) == (size_t)Knob::Count, "knob names");
  const int i = (int)k;
  if (i < 0 || i >= (int)Knob::Count) return nullptr;
  const char* v = getenv(names[i]);
  return (v && v[0]) ? v : nullptr;
}

int measure_probe() { return t_probe; }
}  // namespace rg

// 4: ntt16_pass without HBM data loads / stores (bench.py's compute_floor_ms_per_step);
// 5: ntt256_pass likewise (the L = 4 line's floor).  0 restores the production kernels.
extern "C" rg_status rg_set_probe(int probe) {
  if (probe != 0 && probe != 4 && probe != 5) return RG_ERR_INVALID;
  rg::t_probe = probe;
  return RG_OK;
}
