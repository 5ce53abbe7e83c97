// common.hpp -- shared host-side plumbing of libringo: status codes, HIP error capture,
// device buffers, and the opaque handle definitions behind include/ringo.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../include/ringo.h"

namespace rg {

void set_last_error(const std::string& msg);
// rg_set_probe: process-wide measurement probe (0 = production kernels)
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
