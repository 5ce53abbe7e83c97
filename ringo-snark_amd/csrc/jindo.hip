// jindo.hip -- placeholder (commit pipeline lands next)
#include "common.hpp"
extern "C" {
rg_status rg_jindo_create(const rg_jindo_params*, const uint64_t*, const uint64_t*, const uint64_t*, rg_jindo**) { return RG_ERR_UNSUPPORTED; }
rg_status rg_jindo_create_from_crs(const rg_jindo_params*, const uint8_t*, size_t, rg_jindo**) { return RG_ERR_UNSUPPORTED; }
void rg_jindo_destroy(rg_jindo*) {}
rg_status rg_jindo_commit_key(const rg_jindo*, uint64_t*, uint64_t*, uint64_t*) { return RG_ERR_UNSUPPORTED; }
rg_status rg_jindo_commit(const rg_jindo*, const uint64_t*, size_t, const uint64_t*, const uint64_t*, const int64_t*, const int64_t*, uint64_t*, uint64_t*, uint64_t*, uint64_t*) { return RG_ERR_UNSUPPORTED; }
rg_status rg_jindo_commit_dev(const rg_jindo*, size_t, const uint64_t*, size_t, const uint64_t*, const uint64_t*, const int64_t*, const int64_t*, uint64_t*, uint64_t*, uint64_t*, uint64_t*, void*) { return RG_ERR_UNSUPPORTED; }
size_t rg_jindo_scratch_bytes(const rg_jindo*, size_t) { return 0; }
}
