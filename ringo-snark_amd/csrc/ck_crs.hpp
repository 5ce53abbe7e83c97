// ck_crs.hpp -- commit-key derivation from the CRS, exactly as jindo.NewCommitKey does
// (jindo/entities.go:21-73) on top of math/csprng.UniformSampler (uniform.go:38-95):
//   key = SHA-384(crs)[0:32], iv = SHA-384(crs)[32:48], AES-256-CTR keystream (128-bit
//   big-endian counter, Go's cipher.NewCTR), little-endian u64 words out of an 8192-byte
//   buffer that each refill XORs the next keystream chunk INTO (`XORKeyStream(buf, buf)`,
//   uniform.go:64-70: chunk c holds KS_0 ^ ... ^ KS_c), SampleN(q) by rejection below
//   2^64-1 - (2^64-1) mod q.
// SHA-384 and AES come from the system libcrypto, loaded at run time (no OpenSSL headers
// needed to build; the GPU image ships libcrypto.so.3).  Setup-only, host-side.
#pragma once
#include <dlfcn.h>
#include <stdint.h>
#include <string.h>

#include <vector>

namespace rg {

// SHA-384 from the system libcrypto (NewUniformSamplerWithSeed's key derivation, uniform.go:47)
inline bool sha384(const uint8_t* m, size_t n, uint8_t out[48]) {
  void* h = dlopen("libcrypto.so.3", RTLD_NOW | RTLD_LOCAL);
  if (!h) h = dlopen("libcrypto.so", RTLD_NOW | RTLD_LOCAL);
  if (!h) return false;
  auto f = (unsigned char* (*)(const unsigned char*, size_t, unsigned char*))dlsym(h, "SHA384");
  const bool ok = f && f(m, n, out);
  dlclose(h);
  return ok;
}

class CtrStream {
 public:
  bool ok = false;
  CtrStream(const uint8_t* seed, size_t n) {
    void* h = dlopen("libcrypto.so.3", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("libcrypto.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    lib_ = h;
    auto sha384 = (unsigned char* (*)(const unsigned char*, size_t, unsigned char*))dlsym(h, "SHA384");
    ctx_new_ = (void* (*)())dlsym(h, "EVP_CIPHER_CTX_new");
    ctx_free_ = (void (*)(void*))dlsym(h, "EVP_CIPHER_CTX_free");
    auto aes = (const void* (*)())dlsym(h, "EVP_aes_256_ctr");
    auto init = (int (*)(void*, const void*, void*, const unsigned char*, const unsigned char*))dlsym(
        h, "EVP_EncryptInit_ex");
    update_ = (int (*)(void*, unsigned char*, int*, const unsigned char*, int))dlsym(h, "EVP_EncryptUpdate");
    if (!sha384 || !ctx_new_ || !ctx_free_ || !aes || !init || !update_) return;
    unsigned char r[48];
    sha384(seed, n, r);
    ctx_ = ctx_new_();
    if (!ctx_ || init(ctx_, aes(), nullptr, r, r + 32) != 1) return;
    ok = true;
  }
  ~CtrStream() {
    if (ctx_) ctx_free_(ctx_);
    if (lib_) dlclose(lib_);
  }
  uint64_t next() {  // Sample() (uniform.go:64-82)
    if (pos_ == buf_.size()) refill();
    uint64_t v;
    memcpy(&v, &buf_[pos_], 8);  // little-endian host
    pos_ += 8;
    return v;
  }
  uint64_t sample_n(uint64_t n) {  // SampleN (uniform.go:85-93)
    const uint64_t bound = UINT64_MAX - UINT64_MAX % n;
    for (;;) {
      uint64_t r = next();
      if (r < bound) return r % n;
    }
  }

 private:
  // uniform.go:66-67: s.prng.XORKeyStream(s.buf[:], s.buf[:]) -- the buffer (zero at first)
  // is encrypted in place, i.e. XORed with the next 8192 keystream bytes
  void refill() {
    buf_.resize(kBuf, 0);
    std::vector<unsigned char> in(buf_);
    int outl = 0;
    update_(ctx_, buf_.data(), &outl, in.data(), (int)kBuf);
    pos_ = 0;
  }
  static constexpr size_t kBuf = 8192;
  void* lib_ = nullptr;
  void* ctx_ = nullptr;
  void* (*ctx_new_)() = nullptr;
  void (*ctx_free_)(void*) = nullptr;
  int (*update_)(void*, unsigned char*, int*, const unsigned char*, int) = nullptr;
  std::vector<unsigned char> buf_;
  size_t pos_ = 0;
};

}  // namespace rg
