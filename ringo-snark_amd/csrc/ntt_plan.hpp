// ntt_plan.hpp -- what ntt.hip hands to the per-limb-count kernel translation units.
#pragma once
#include <mutex>

#include "common.hpp"

namespace rg {

struct PassDesc {
  int G0, P;
};

// Everything a per-L translation unit needs from the host plan.
struct NttLaunch {
  const uint64_t* in;
  uint64_t* out;
  const uint64_t* tw;
  const uint64_t* q;
  uint64_t qinv;
  const uint64_t* nsc;
  uint64_t nsc_sh;
  const uint64_t* w1n;
  uint64_t w1n_sh;
  int logN;
  bool shoup, inv, tiled;
  bool halving;  // rank_inv == N^-1: the wide pass's per-stage halving scales the inverse correctly
  const PassDesc* passes;  // forward order
  int npasses;
  size_t batch;
  // the plan's helper stream for ntt256_run's two-half split (null: single stream); the mutex
  // serialises the fork/join enqueue of concurrent callers, which share the events
  struct Aux* aux = nullptr;
};

// a helper stream and the two events that fork it from and join it back to the caller's stream
struct Aux {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  std::mutex mu;
  ~Aux() {
    if (s) (void)hipStreamDestroy(s);
    if (fork) (void)hipEventDestroy(fork);
    if (join) (void)hipEventDestroy(join);
  }
};

// the field and kind of a plan (for the operators built on it: buckler.hip)
const rg_field* ntt_field(const rg_ntt* t);
bool ntt_negacyclic(const rg_ntt* t);

rg_status ntt_run_L1(const NttLaunch& p, hipStream_t st);
// lazy single-word pass kernels (ntt_l1_lazy.hip); sets *handled when the shape is covered
rg_status ntt64_run(const NttLaunch& p, hipStream_t st, bool* handled);
// 4-limb degree-2^16 kernels for q = 1 mod 2^64 (ntt_l4_fast.hip)
rg_status ntt256_run(const NttLaunch& p, hipStream_t st, bool* handled);
rg_status ntt_run_L2(const NttLaunch& p, hipStream_t st);
rg_status ntt_run_L4(const NttLaunch& p, hipStream_t st);
rg_status ntt_run_L7(const NttLaunch& p, hipStream_t st);
rg_status ntt_run_L14(const NttLaunch& p, hipStream_t st);

}  // namespace rg
