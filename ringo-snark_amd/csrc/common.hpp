// common.hpp -- shared host-side plumbing of libringo: status codes, HIP error capture,
// device buffers, and the opaque handle definitions behind include/ringo.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../include/ringo.h"

namespace rg {

void set_last_error(const std::string& msg);

// Measurement / A-B switches.  libringo.so links knobs.hip, where every knob is unset (nullptr:
// the production choice) and the probe is 0.  Only the experiments build, libringo_exp.so
// (tools/experiments/knobs_env.hip), reads them from the RINGO_* environment and honours
// rg_set_probe; the production library has no environment access at all.
enum class Knob : int {
  NttKernel,   // RINGO_NTT_KERNEL   r*: generic single-word / q255 pass kernels; stage: wide fields per stage
  NttChunkMb,  // RINGO_NTT_CHUNK_MB polys per pass pair bounded to this many MiB
  JindoMac,    // RINGO_JINDO_MAC    l: mac_kernel instead of the MFMA MAC
  JindoSplit,  // RINGO_JINDO_SPLIT  0: commit_sampled on the caller's stream only
  JindoUniTries,  // RINGO_JINDO_UNI_TRIES n: uniform_whole_kernel gives up after n tries (tests the fix-up path)
  Count
};
const char* knob(Knob k);
// rg_set_probe's value on the calling thread (always 0 in libringo.so)
int measure_probe();

#define RG_HIP(call)                                                                            \
  do {                                                                                          \
    hipError_t e_ = (call);                                                                     \
    if (e_ != hipSuccess) {                                                                     \
      ::rg::set_last_error(std::string(#call) + ": " + hipGetErrorString(e_) + " @" + __FILE__ + \
                           ":" + std::to_string(__LINE__));                                     \
      return RG_ERR_DEVICE;                                                                     \
    }                                                                                           \
  } while (0)

#define RG_TRY(expr)          \
  do {                        \
    rg_status s_ = (expr);    \
    if (s_ != RG_OK) return s_; \
  } while (0)

inline rg_status check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_last_error(std::string("launch ") + what + ": " + hipGetErrorString(e));
    return RG_ERR_DEVICE;
  }
  return RG_OK;
}

// RAII device buffer
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  rg_status alloc(size_t n) {
    if (p && bytes >= n) return RG_OK;
    if (p) {
      (void)hipFree(p);
      p = nullptr;
      bytes = 0;
    }
    if (n == 0) return RG_OK;
    hipError_t e = hipMalloc(&p, n);
    if (e != hipSuccess) {
      set_last_error(std::string("hipMalloc ") + std::to_string(n) + ": " + hipGetErrorString(e));
      p = nullptr;
      return RG_ERR_NOMEM;
    }
    bytes = n;
    return RG_OK;
  }
  rg_status upload(const void* src, size_t n) {
    RG_TRY(alloc(n));
    RG_HIP(hipMemcpy(p, src, n, hipMemcpyHostToDevice));
    return RG_OK;
  }
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
};

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Compile-time loop: f(std::integral_constant<int, i>) for i in [0, N), so a body indexes its
// register arrays with constants (a rolled loop the unroller leaves alone indexes them dynamically)
template <class F, int... I>
__host__ __device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__host__ __device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// Division of a 32-bit index by a launch-constant divisor through the double unit: q = floor(n / d)
// as trunc((n + 1/2) / d); (n + 1/2) / d keeps 1 / (2 d) from both neighbouring integers, far more
// than the few-ulp error of one fma on n < 2^32.  3 VALU against ~100 for a 64-bit integer division.
struct IdxDiv {
  uint32_t d;
  double inv, half_inv;  // 1 / d and (1 / d) / 2
};
inline IdxDiv make_idxdiv(uint32_t d) {
  IdxDiv f;
  f.d = d;
  f.inv = 1.0 / (double)d;
  f.half_inv = 0.5 * f.inv;
  return f;
}
__host__ __device__ __forceinline__ uint32_t idx_div(uint32_t n, const IdxDiv& f) {
  return (uint32_t)fma((double)n, f.inv, f.half_inv);
}

}  // namespace rg

// ------------------------------------------------------------------------------------------
// handle definitions
// ------------------------------------------------------------------------------------------
struct rg_field {
  int L;
  uint64_t q[16];
  uint64_t qinv;
  uint64_t r2[16];
  uint64_t one[16];
  bool spare_bit;  // q < 2^(64L-1)
};
