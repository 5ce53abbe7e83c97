// capi.hip -- C-ABI entry points that are not kernel-specific: status strings, field
// handles, device memory helpers.
#include <string>

#include "common.hpp"
#include "host_field.hpp"

namespace rg {
static thread_local std::string g_last_error;
void set_last_error(const std::string& msg) { g_last_error = msg; }
}  // namespace rg

using namespace rg;

extern "C" {

const char* rg_status_string(int s) {
  switch (s) {
    case RG_OK: return "ok";
    case RG_ERR_INVALID: return "inconsistent input(s)";
    case RG_ERR_NOT_POW2: return "rank must be a power of two";
    case RG_ERR_UNSUPPORTED: return "NTT not supported";
    case RG_ERR_DEVICE: return "device error";
    case RG_ERR_NOMEM: return "out of device memory";
    case RG_ERR_RANK: return "len(v) > params.rank";
    default: return "unknown status";
  }
}

const char* rg_last_error(void) { return g_last_error.c_str(); }

#define RG_STR2(x) #x
#define RG_STR(x) RG_STR2(x)
const char* rg_version(void) {
  return "libringo 0.2 gfx950 (ntt, vec, jindo) sampler-layout " RG_STR(RG_SAMPLER_LAYOUT);
}

rg_status rg_field_create(int limbs, const uint64_t* q_le, rg_field** out) {
  if (!out || !q_le) return RG_ERR_INVALID;
  *out = nullptr;
  rg_field* f = new rg_field();
  if (!init_field(f, limbs, q_le)) {
    delete f;
    return RG_ERR_INVALID;
  }
  *out = f;
  return RG_OK;
}

void rg_field_destroy(rg_field* f) { delete f; }
int rg_field_limbs(const rg_field* f) { return f ? f->L : 0; }

rg_status rg_field_constants(const rg_field* f, uint64_t* qinv_neg, uint64_t* r2_le, uint64_t* one_le) {
  if (!f) return RG_ERR_INVALID;
  if (qinv_neg) *qinv_neg = f->qinv;
  if (r2_le) memcpy(r2_le, f->r2, 8 * f->L);
  if (one_le) memcpy(one_le, f->one, 8 * f->L);
  return RG_OK;
}

rg_status rg_malloc(void** d_ptr, size_t bytes) {
  if (!d_ptr) return RG_ERR_INVALID;
  hipError_t e = hipMalloc(d_ptr, bytes);
  if (e != hipSuccess) {
    set_last_error(std::string("hipMalloc: ") + hipGetErrorString(e));
    return RG_ERR_NOMEM;
  }
  return RG_OK;
}
rg_status rg_free(void* d_ptr) {
  RG_HIP(hipFree(d_ptr));
  return RG_OK;
}
rg_status rg_memcpy_h2d(void* d_dst, const void* src, size_t bytes, void* stream) {
  RG_HIP(hipMemcpyAsync(d_dst, src, bytes, hipMemcpyHostToDevice, as_stream(stream)));
  return RG_OK;
}
rg_status rg_memcpy_d2h(void* dst, const void* d_src, size_t bytes, void* stream) {
  RG_HIP(hipMemcpyAsync(dst, d_src, bytes, hipMemcpyDeviceToHost, as_stream(stream)));
  return RG_OK;
}
rg_status rg_memcpy_d2d(void* d_dst, const void* d_src, size_t bytes, void* stream) {
  RG_HIP(hipMemcpyAsync(d_dst, d_src, bytes, hipMemcpyDeviceToDevice, as_stream(stream)));
  return RG_OK;
}
rg_status rg_stream_sync(void* stream) {
  RG_HIP(hipStreamSynchronize(as_stream(stream)));
  return RG_OK;
}
rg_status rg_set_device(int device) {
  RG_HIP(hipSetDevice(device));
  return RG_OK;
}

rg_status rg_get_device(int* device) {
  if (!device) return RG_ERR_INVALID;
  RG_HIP(hipGetDevice(device));
  return RG_OK;
}

rg_status rg_device_count(int* n) {
  if (!n) return RG_ERR_INVALID;
  RG_HIP(hipGetDeviceCount(n));
  return RG_OK;
}

}  // extern "C"
