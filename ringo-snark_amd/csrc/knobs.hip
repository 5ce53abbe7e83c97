// knobs.hip -- the production library's knob table: every kernel choice is the default one and
// the measurement probe is refused.  The experiments build (libringo_exp.so) links
// tools/experiments/knobs_env.hip in place of this file.
#include "common.hpp"

namespace rg {
const char* knob(Knob) { return nullptr; }
int measure_probe() { return 0; }
}  // namespace rg

extern "C" rg_status rg_set_probe(int probe) { return probe == 0 ? RG_OK : RG_ERR_INVALID; }
