// host_field.hpp -- runtime-L Montgomery arithmetic on the host, used only for setup work
// inside the library (twiddle tables, root search, constants).  Same semantics as the device
// code in field.hpp (gnark Montgomery, R = 2^(64L), canonical results).
#pragma once
#include <stdint.h>
#include <string.h>

#include <vector>

#include "common.hpp"

namespace rg {

typedef unsigned __int128 u128;

struct HostField {
  int L;
  const uint64_t* q;
  uint64_t qinv;
  const uint64_t* one;
  const uint64_t* r2;
  explicit HostField(const rg_field* f) : L(f->L), q(f->q), qinv(f->qinv), one(f->one), r2(f->r2) {}

  static bool geq(const uint64_t* a, const uint64_t* b, int L) {
    for (int i = L - 1; i >= 0; --i)
      if (a[i] != b[i]) return a[i] > b[i];
    return true;
  }
  static uint64_t add_n(uint64_t* z, const uint64_t* a, const uint64_t* b, int L) {
    uint64_t c = 0;
    for (int i = 0; i < L; ++i) {
      u128 s = (u128)a[i] + b[i] + c;
      z[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    return c;
  }
  static uint64_t sub_n(uint64_t* z, const uint64_t* a, const uint64_t* b, int L) {
    uint64_t br = 0;
    for (int i = 0; i < L; ++i) {
      u128 d = (u128)a[i] - b[i] - br;
      z[i] = (uint64_t)d;
      br = (uint64_t)(d >> 64) & 1;
    }
    return br;
  }
  void add(uint64_t* z, const uint64_t* x, const uint64_t* y) const {
    uint64_t t[16];
    uint64_t c = add_n(t, x, y, L);
    if (c || geq(t, q, L)) sub_n(t, t, q, L);
    memcpy(z, t, 8 * L);
  }
  void mul(uint64_t* z, const uint64_t* x, const uint64_t* y) const {
    uint64_t t[18] = {0};
    for (int i = 0; i < L; ++i) {
      uint64_t c = 0;
      for (int j = 0; j < L; ++j) {
        u128 s = (u128)x[i] * y[j] + t[j] + c;
        t[j] = (uint64_t)s;
        c = (uint64_t)(s >> 64);
      }
      u128 s = (u128)t[L] + c;
      t[L] = (uint64_t)s;
      t[L + 1] = (uint64_t)(s >> 64);
      uint64_t m = t[0] * qinv;
      s = (u128)m * q[0] + t[0];
      c = (uint64_t)(s >> 64);
      for (int j = 1; j < L; ++j) {
        s = (u128)m * q[j] + t[j] + c;
        t[j - 1] = (uint64_t)s;
        c = (uint64_t)(s >> 64);
      }
      s = (u128)t[L] + c;
      t[L - 1] = (uint64_t)s;
      t[L] = t[L + 1] + (uint64_t)(s >> 64);
    }
    if (t[L] || geq(t, q, L)) sub_n(t, t, q, L);
    memcpy(z, t, 8 * L);
  }
  void pow(uint64_t* z, const uint64_t* x, const uint64_t* e, int ne) const {
    uint64_t r[16], b[16];
    memcpy(r, one, 8 * L);
    memcpy(b, x, 8 * L);
    for (int w = 0; w < ne; ++w)
      for (int k = 0; k < 64; ++k) {
        if ((e[w] >> k) & 1) mul(r, r, b);
        mul(b, b, b);
      }
    memcpy(z, r, 8 * L);
  }
  void from_u64(uint64_t* z, uint64_t v) const {  // SetUint64 (element.go:93-97)
    uint64_t t[16] = {0};
    t[0] = v;
    mul(z, t, r2);
  }
  void from_mont(uint64_t* z, const uint64_t* x) const {  // fromMont
    uint64_t o[16] = {0};
    o[0] = 1;
    mul(z, x, o);
  }
  void inverse(uint64_t* z, const uint64_t* x) const {  // Fermat: x^(q-2)
    uint64_t e[16], two[16] = {0};
    two[0] = 2;
    sub_n(e, q, two, L);
    pow(z, x, e, L);
  }
  bool eq(const uint64_t* a, const uint64_t* b) const { return memcmp(a, b, 8 * L) == 0; }
};

// Fill f's derived constants from q (limbs 1..16).  Returns false if q is even or zero.
inline bool init_field(rg_field* f, int L, const uint64_t* q_le) {
  if (L < 1 || L > 16 || !(q_le[0] & 1)) return false;
  memset(f, 0, sizeof(*f));
  f->L = L;
  memcpy(f->q, q_le, 8 * L);
  if (L == 1 && q_le[0] < 3) return false;
  uint64_t inv = 1;
  for (int i = 0; i < 7; ++i) inv *= 2 - q_le[0] * inv;
  f->qinv = 0 - inv;
  uint64_t r[16] = {1};
  for (int i = 0; i < 128 * L; ++i) {  // R mod q after 64L doublings, R^2 after 128L
    uint64_t t[16];
    uint64_t c = HostField::add_n(t, r, r, L);
    if (c || HostField::geq(t, f->q, L)) HostField::sub_n(t, t, f->q, L);
    memcpy(r, t, 8 * L);
    if (i == 64 * L - 1) memcpy(f->one, r, 8 * L);
  }
  memcpy(f->r2, r, 8 * L);
  f->spare_bit = (f->q[L - 1] >> 63) == 0;
  return true;
}

}  // namespace rg
