/* oracle.c -- CPU restatement of the ringo-snark hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This file is the checker (and bench.py's timed "port" CPU baseline), never the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load liboracle.so.
 * It is a plain-C restatement of the reference's algorithms, cross-checked against the
 * big-int restatement oracle/pyref.py and the reference's generated field constants
 * (tests/golden/fields.json).  File:line citations are into sp301415/ringo-snark.
 *
 *   field      jindo/internal/zp/element.go:397-466 (Add/Sub/Neg), element_purego.go:46-213 (Mul)
 *   bigpoly    math/bigpoly/ntt.go:153-203 (tables), :246-466 (transforms), vec.go:9-121
 *   jindo      jindo/encoder.go:120-201, jindo/prover.go:45-202, jindo/rns.go:76-114
 *   lattigo    ring NTT/INTT/MForm/IMForm/MulCoeffsMontgomeryThenAdd (v6.1.0, source absent:
 *              restated from its published algorithm -- PARITY UNPINNED at that boundary)
 *
 * Layouts are identical to the C-ABI in include/ringo.h so tests compare buffers bytewise.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
#define MAXL 16

typedef struct {
  int L;
  uint64_t q[MAXL];
  uint64_t qinv; /* -q^-1 mod 2^64  (element.go:70-72) */
  uint64_t r2[MAXL];
  uint64_t one[MAXL]; /* R mod q */
} of_field;

/* ------------------------------------------------------------------------------------------ */
/* multi-limb helpers                                                                          */
/* ------------------------------------------------------------------------------------------ */
static inline int geq(const uint64_t* a, const uint64_t* b, int L) {
  for (int i = L - 1; i >= 0; --i) {
    if (a[i] != b[i]) return a[i] > b[i];
  }
  return 1;
}
static inline uint64_t add_n(uint64_t* z, const uint64_t* a, const uint64_t* b, int L) {
  uint64_t c = 0;
  for (int i = 0; i < L; ++i) {
    u128 s = (u128)a[i] + b[i] + c;
    z[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  return c;
}
static inline uint64_t sub_n(uint64_t* z, const uint64_t* a, const uint64_t* b, int L) {
  uint64_t br = 0;
  for (int i = 0; i < L; ++i) {
    u128 d = (u128)a[i] - b[i] - br;
    z[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  return br;
}

/* Add: z = x + y, conditional -q (element.go:397-413) */
static inline void f_add(const of_field* F, uint64_t* z, const uint64_t* x, const uint64_t* y, int L) {
  uint64_t t[MAXL];
  uint64_t c = add_n(t, x, y, L);
  if (c || geq(t, F->q, L)) sub_n(t, t, F->q, L);
  memcpy(z, t, 8 * L);
}
/* Sub: z = x - y, conditional +q (element.go:437-451) */
static inline void f_sub(const of_field* F, uint64_t* z, const uint64_t* x, const uint64_t* y, int L) {
  uint64_t t[MAXL];
  if (sub_n(t, x, y, L)) add_n(t, t, F->q, L);
  memcpy(z, t, 8 * L);
}
/* Neg: 0 -> 0, else q - x (element.go:454-466) */
static inline void f_neg(const of_field* F, uint64_t* z, const uint64_t* x, int L) {
  int zero = 1;
  for (int i = 0; i < L; ++i) zero &= x[i] == 0;
  if (zero) {
    memset(z, 0, 8 * L);
    return;
  }
  sub_n(z, F->q, x, L);
}
/* Montgomery CIOS z = x*y*R^-1 mod q, fully reduced (element_purego.go:46-213). */
static inline void f_mul(const of_field* F, uint64_t* z, const uint64_t* x, const uint64_t* y, int L) {
  uint64_t t[MAXL + 2];
  memset(t, 0, sizeof(uint64_t) * (L + 2));
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
    uint64_t m = t[0] * F->qinv;
    s = (u128)m * F->q[0] + t[0];
    c = (uint64_t)(s >> 64);
    for (int j = 1; j < L; ++j) {
      s = (u128)m * F->q[j] + t[j] + c;
      t[j - 1] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    s = (u128)t[L] + c;
    t[L - 1] = (uint64_t)s;
    t[L] = t[L + 1] + (uint64_t)(s >> 64);
  }
  if (t[L] || geq(t, F->q, L)) sub_n(t, t, F->q, L);
  memcpy(z, t, 8 * L);
}

int of_field_init(of_field* F, int L, const uint64_t* q) {
  if (L < 1 || L > MAXL || !(q[0] & 1)) return -1;
  memset(F, 0, sizeof(*F));
  F->L = L;
  memcpy(F->q, q, 8 * L);
  uint64_t inv = 1; /* Newton: q^-1 mod 2^64 */
  for (int i = 0; i < 7; ++i) inv *= 2 - q[0] * inv;
  F->qinv = 0 - inv;
  /* R mod q by doubling 1 (64L times); R^2 by doubling (128L times). */
  uint64_t r[MAXL] = {1};
  for (int i = 0; i < 128 * L; ++i) {
    f_add(F, r, r, r, L);
    if (i == 64 * L - 1) memcpy(F->one, r, 8 * L);
  }
  memcpy(F->r2, r, 8 * L);
  return 0;
}
void of_field_consts(const of_field* F, uint64_t* qinv, uint64_t* r2, uint64_t* one) {
  *qinv = F->qinv;
  memcpy(r2, F->r2, 8 * F->L);
  memcpy(one, F->one, 8 * F->L);
}
size_t of_field_size(void) { return sizeof(of_field); }

/* exported element ops (for tests) */
void of_f_mul(const of_field* F, uint64_t* z, const uint64_t* x, const uint64_t* y) { f_mul(F, z, x, y, F->L); }
void of_f_add(const of_field* F, uint64_t* z, const uint64_t* x, const uint64_t* y) { f_add(F, z, x, y, F->L); }
void of_f_sub(const of_field* F, uint64_t* z, const uint64_t* x, const uint64_t* y) { f_sub(F, z, x, y, F->L); }
void of_f_neg(const of_field* F, uint64_t* z, const uint64_t* x) { f_neg(F, z, x, F->L); }

/* z = x^e (Montgomery), e given as little-endian limbs (ne words) */
static void f_pow(const of_field* F, uint64_t* z, const uint64_t* x, const uint64_t* e, int ne) {
  int L = F->L;
  uint64_t r[MAXL], b[MAXL];
  memcpy(r, F->one, 8 * L);
  memcpy(b, x, 8 * L);
  for (int w = 0; w < ne; ++w)
    for (int k = 0; k < 64; ++k) {
      if ((e[w] >> k) & 1) f_mul(F, r, r, b, L);
      f_mul(F, b, b, b, L);
    }
  memcpy(z, r, 8 * L);
}
static void f_from_u64(const of_field* F, uint64_t* z, uint64_t v) { /* SetUint64 (element.go:93-97) */
  uint64_t t[MAXL] = {0};
  t[0] = v;
  f_mul(F, z, t, F->r2, F->L);
}
static void shr_n(uint64_t* z, const uint64_t* a, int L, int s) { /* s < 64 */
  for (int i = 0; i < L; ++i) z[i] = (a[i] >> s) | (s && i + 1 < L ? a[i + 1] << (64 - s) : 0);
}
static void bitrev_perm(uint64_t* v, int N, int L) { /* vec.go:123-137 */
  int j = 0;
  uint64_t tmp[MAXL];
  for (int i = 1; i < N; ++i) {
    int bit = N >> 1;
    for (; j >= bit; bit >>= 1) j -= bit;
    j += bit;
    if (i < j) {
      memcpy(tmp, v + (size_t)i * L, 8 * L);
      memcpy(v + (size_t)i * L, v + (size_t)j * L, 8 * L);
      memcpy(v + (size_t)j * L, tmp, 8 * L);
    }
  }
}

/* Generator search (ntt.go:46-53 / :173-180): first x=2,3,.. with (x^t1)^t2 != 1; t1 =
 * (p-1)/root_order via a right shift (root_order is a power of two dividing p-1). */
static int find_root(const of_field* F, int log_order, uint64_t t2, uint64_t* g) {
  int L = F->L;
  uint64_t pm1[MAXL], t1[MAXL], x[MAXL], gp[MAXL], e2[1] = {t2};
  memcpy(pm1, F->q, 8 * L);
  pm1[0] -= 1;
  memcpy(t1, pm1, 8 * L);
  for (int s = log_order; s > 0; s -= (s > 63 ? 63 : s)) shr_n(t1, t1, L, s > 63 ? 63 : s);
  for (uint64_t xv = 2; xv < 1000000; ++xv) {
    f_from_u64(F, x, xv);
    f_pow(F, g, x, t1, L);
    f_pow(F, gp, g, e2, 1);
    if (memcmp(gp, F->one, 8 * L) != 0) return 0;
  }
  return -1;
}
static int log2i(uint64_t n) {
  int k = 0;
  while ((1ull << k) < n) ++k;
  return k;
}
static int check_support(const of_field* F, int N) {
  if (N <= 0 || (N & (N - 1))) return -1; /* "rank must be a power of two" */
  uint64_t pm1 = F->q[0] - 1;           /* 2N | p-1 ("NTT not supported", ntt.go:162-164) */
  int tz = pm1 ? __builtin_ctzll(pm1) : 64;
  return (tz >= log2i((uint64_t)N) + 1) ? 0 : -2;
}

/* NewCyclotomicTransformer (ntt.go:153-203): tw[k] = psi^brv(k), twinv[k] = psi^-brv(k). */
int of_cyclotomic_tables(const of_field* F, int N, uint64_t* tw, uint64_t* twinv, uint64_t* ninv) {
  int rc = check_support(F, N), L = F->L;
  if (rc) return rc;
  uint64_t g[MAXL], gi[MAXL], pm2[MAXL];
  if (find_root(F, log2i(N) + 1, (uint64_t)N, g)) return -3;
  uint64_t two[MAXL] = {2};
  sub_n(pm2, F->q, two, L);
  f_pow(F, gi, g, pm2, L);
  memcpy(tw, F->one, 8 * L);
  memcpy(twinv, F->one, 8 * L);
  for (int i = 1; i < N; ++i) {
    f_mul(F, tw + (size_t)i * L, tw + (size_t)(i - 1) * L, g, L);
    f_mul(F, twinv + (size_t)i * L, twinv + (size_t)(i - 1) * L, gi, L);
  }
  bitrev_perm(tw, N, L);
  bitrev_perm(twinv, N, L);
  uint64_t n[MAXL];
  f_from_u64(F, n, (uint64_t)N);
  f_pow(F, ninv, n, pm2, L);
  return 0;
}

/* NewCyclicTransformer (ntt.go:26-95): per-stage table tw[m+i] = brv_{N/2}(w^j)[i]. */
int of_cyclic_tables(const of_field* F, int N, uint64_t* tw, uint64_t* twinv, uint64_t* ninv) {
  int rc = check_support(F, N), L = F->L;
  if (rc) return rc;
  uint64_t g[MAXL], gi[MAXL], pm2[MAXL];
  if (find_root(F, log2i(N), (uint64_t)(N >> 1), g)) return -3;
  uint64_t two[MAXL] = {2};
  sub_n(pm2, F->q, two, L);
  f_pow(F, gi, g, pm2, L);
  int h = N / 2 > 0 ? N / 2 : 1;
  uint64_t* ref = (uint64_t*)calloc((size_t)h * L, 8);
  uint64_t* refi = (uint64_t*)calloc((size_t)h * L, 8);
  memcpy(ref, F->one, 8 * L);
  memcpy(refi, F->one, 8 * L);
  for (int i = 1; i < N / 2; ++i) {
    f_mul(F, ref + (size_t)i * L, ref + (size_t)(i - 1) * L, g, L);
    f_mul(F, refi + (size_t)i * L, refi + (size_t)(i - 1) * L, gi, L);
  }
  if (N >= 2) {
    bitrev_perm(ref, N / 2, L);
    bitrev_perm(refi, N / 2, L);
  }
  memset(tw, 0, (size_t)N * L * 8);
  memset(twinv, 0, (size_t)N * L * 8);
  for (int m = 1; m <= N / 2; m <<= 1)
    for (int i = 0; i < m; ++i) {
      memcpy(tw + (size_t)(m + i) * L, ref + (size_t)i * L, 8 * L);
      memcpy(twinv + (size_t)(m + i) * L, refi + (size_t)i * L, 8 * L);
    }
  free(ref);
  free(refi);
  uint64_t n[MAXL];
  f_from_u64(F, n, (uint64_t)N);
  f_pow(F, ninv, n, pm2, L);
  return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* bigpoly transforms: nttInPlaceRef / inttInPlaceRef (ntt.go:254-275, 365-386) -- the
 * unrolled variants (:277-355, :388-466) perform the identical butterflies in another order.  */
/* ------------------------------------------------------------------------------------------ */
static inline void ntt_one(const of_field* F, uint64_t* p, const uint64_t* tw, int N, int L) {
  uint64_t v[MAXL];
  int t = N;
  for (int m = 1; m <= N / 2; m <<= 1) {
    t >>= 1;
    for (int i = 0; i < m; ++i) {
      const uint64_t* w = tw + (size_t)(m + i) * L;
      for (int j = 2 * i * t; j < 2 * i * t + t; ++j) {
        uint64_t* u = p + (size_t)j * L;
        uint64_t* x = p + (size_t)(j + t) * L;
        f_mul(F, v, x, w, L); /* butterfly: v*=w; u+=v; v = u-2v  == (u+v, u-v) */
        f_sub(F, x, u, v, L);
        f_add(F, u, u, v, L);
      }
    }
  }
}
static inline void intt_one(const of_field* F, uint64_t* p, const uint64_t* twinv, const uint64_t* ninv,
                            int N, int L) {
  uint64_t d[MAXL];
  int t = 1;
  for (int m = N / 2; m >= 1; m >>= 1) {
    for (int i = 0; i < m; ++i) {
      const uint64_t* w = twinv + (size_t)(m + i) * L;
      for (int j = 2 * i * t; j < 2 * i * t + t; ++j) {
        uint64_t* u = p + (size_t)j * L;
        uint64_t* x = p + (size_t)(j + t) * L;
        f_sub(F, d, u, x, L);
        f_add(F, u, u, x, L);
        f_mul(F, x, d, w, L);
      }
    }
    t <<= 1;
  }
  for (int j = 0; j < N; ++j) f_mul(F, p + (size_t)j * L, p + (size_t)j * L, ninv, L);
}

#define DISPATCH_L(L, CALL)   \
  switch (L) {                \
    case 1: { enum { LL = 1 }; CALL; } break;  \
    case 2: { enum { LL = 2 }; CALL; } break;  \
    case 4: { enum { LL = 4 }; CALL; } break;  \
    case 7: { enum { LL = 7 }; CALL; } break;  \
    case 14: { enum { LL = 14 }; CALL; } break; \
    default: { const int LL = L; CALL; } break; \
  }

/* in/out: [batch][N][L]; out may alias in (the Go side copies first, ntt.go:206-222). */
void of_ntt_fwd(const of_field* F, uint64_t* out, const uint64_t* in, const uint64_t* tw, int N, long batch) {
  if (out != in) memcpy(out, in, (size_t)batch * N * F->L * 8);
#pragma omp parallel for schedule(static)
  for (long b = 0; b < batch; ++b) DISPATCH_L(F->L, ntt_one(F, out + (size_t)b * N * LL, tw, N, LL));
}
void of_ntt_inv(const of_field* F, uint64_t* out, const uint64_t* in, const uint64_t* twinv,
                const uint64_t* ninv, int N, long batch) {
  if (out != in) memcpy(out, in, (size_t)batch * N * F->L * 8);
#pragma omp parallel for schedule(static)
  for (long b = 0; b < batch; ++b) DISPATCH_L(F->L, intt_one(F, out + (size_t)b * N * LL, twinv, ninv, N, LL));
}

/* pointwise ops (vec.go:9-121, base_op.go:49-171).  op codes match include/ringo.h rg_vec_op. */
enum { OV_ADD = 0, OV_SUB, OV_NEG, OV_MUL, OV_SMUL, OV_MUL_ADD, OV_MUL_SUB, OV_SMUL_ADD, OV_SMUL_SUB };
void of_vec(const of_field* F, int op, uint64_t* out, const uint64_t* a, const uint64_t* b, long n) {
  int L = F->L;
  uint64_t t[MAXL];
  for (long i = 0; i < n; ++i) {
    uint64_t* z = out + (size_t)i * L;
    const uint64_t* x = a + (size_t)i * L;
    const uint64_t* y = (op == OV_SMUL || op == OV_SMUL_ADD || op == OV_SMUL_SUB) ? b : (b ? b + (size_t)i * L : 0);
    switch (op) {
      case OV_ADD: f_add(F, z, x, y, L); break;
      case OV_SUB: f_sub(F, z, x, y, L); break;
      case OV_NEG: f_neg(F, z, x, L); break;
      case OV_MUL: case OV_SMUL: f_mul(F, z, x, y, L); break;
      case OV_MUL_ADD: case OV_SMUL_ADD: f_mul(F, t, x, y, L); f_add(F, z, z, t, L); break;
      case OV_MUL_SUB: case OV_SMUL_SUB: f_mul(F, t, x, y, L); f_sub(F, z, z, t, L); break;
    }
  }
}

/* ------------------------------------------------------------------------------------------ */
/* Lattigo-convention word ring (d-point negacyclic, per prime)                                 */
/* ------------------------------------------------------------------------------------------ */
static inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) { return (uint64_t)((u128)a * b % q); }
static uint64_t powmod(uint64_t a, uint64_t e, uint64_t q) {
  uint64_t r = 1 % q;
  a %= q;
  while (e) {
    if (e & 1) r = mulmod(r, a, q);
    a = mulmod(a, a, q);
    e >>= 1;
  }
  return r;
}
static int is_prime_u64(uint64_t n) {
  if (n < 2) return 0;
  static const uint64_t sp[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
  for (int i = 0; i < 12; ++i)
    if (n % sp[i] == 0) return n == sp[i];
  uint64_t d = n - 1;
  int r = 0;
  while (!(d & 1)) d >>= 1, ++r;
  for (int i = 0; i < 12; ++i) {
    uint64_t x = powmod(sp[i], d, n);
    if (x == 1 || x == n - 1) continue;
    int ok = 0;
    for (int k = 1; k < r; ++k) {
      x = mulmod(x, x, n);
      if (x == n - 1) { ok = 1; break; }
    }
    if (!ok) return 0;
  }
  return 1;
}
static uint64_t gcd_u64(uint64_t a, uint64_t b) {
  while (b) { uint64_t t = a % b; a = b; b = t; }
  return a;
}
static uint64_t rho(uint64_t n) {
  if (!(n & 1)) return 2;
  for (uint64_t c = 1;; ++c) {
    uint64_t x = 2, y = 2, d = 1;
    while (d == 1) {
      x = (mulmod(x, x, n) + c) % n;
      y = (mulmod(y, y, n) + c) % n;
      y = (mulmod(y, y, n) + c) % n;
      d = gcd_u64(x > y ? x - y : y - x, n);
    }
    if (d != n) return d;
  }
}
static int factor_rec(uint64_t n, uint64_t* f, int nf) {
  if (n == 1) return nf;
  if (is_prime_u64(n)) {
    for (int i = 0; i < nf; ++i) if (f[i] == n) return nf;
    f[nf] = n;
    return nf + 1;
  }
  uint64_t d = rho(n);
  nf = factor_rec(d, f, nf);
  return factor_rec(n / d, f, nf);
}
/* ring.PrimitiveRoot: smallest g >= 3 that is a primitive root mod q. */
uint64_t of_primitive_root(uint64_t q) {
  uint64_t f[64];
  int nf = factor_rec(q - 1, f, 0);
  for (uint64_t g = 3;; ++g) {
    int ok = 1;
    for (int i = 0; i < nf && ok; ++i) ok = powmod(g, (q - 1) / f[i], q) != 1;
    if (ok) return g;
  }
}
static uint64_t brv(uint64_t x, int logn) {
  uint64_t r = 0;
  for (int i = 0; i < logn; ++i) r = (r << 1) | ((x >> i) & 1);
  return r;
}
typedef struct {
  uint64_t q;
  int d, logd;
  uint64_t* roots;   /* plain residues, roots[brv(j)] = psi^j */
  uint64_t* iroots;
  uint64_t ninv, m, minv; /* 2^64 mod q, 2^-64 mod q */
} of_subring;
static void subring_init(of_subring* S, int d, uint64_t q) {
  S->q = q;
  S->d = d;
  S->logd = log2i((uint64_t)d);
  uint64_t g = of_primitive_root(q);
  uint64_t psi = powmod(g, (q - 1) / (2 * (uint64_t)d), q), psii = powmod(psi, q - 2, q);
  S->roots = (uint64_t*)malloc(8 * (size_t)d);
  S->iroots = (uint64_t*)malloc(8 * (size_t)d);
  uint64_t a = 1, b = 1;
  for (int j = 0; j < d; ++j) {
    S->roots[brv((uint64_t)j, S->logd)] = a;
    S->iroots[brv((uint64_t)j, S->logd)] = b;
    a = mulmod(a, psi, q);
    b = mulmod(b, psii, q);
  }
  S->ninv = powmod((uint64_t)d, q - 2, q);
  S->m = (uint64_t)(((u128)1 << 64) % q);
  S->minv = powmod(S->m, q - 2, q);
}
static void subring_free(of_subring* S) {
  free(S->roots);
  free(S->iroots);
}
uint64_t of_lattigo_psi(uint64_t q, int d) {
  return powmod(of_primitive_root(q), (q - 1) / (2 * (uint64_t)d), q);
}
static void r_ntt(const of_subring* S, uint64_t* p) {
  uint64_t q = S->q;
  int N = S->d, t = N;
  for (int m = 1; m < N; m <<= 1) {
    t >>= 1;
    for (int i = 0; i < m; ++i) {
      uint64_t w = S->roots[m + i];
      for (int j = 2 * i * t; j < 2 * i * t + t; ++j) {
        uint64_t u = p[j], v = mulmod(p[j + t], w, q);
        p[j] = u + v >= q ? u + v - q : u + v;
        p[j + t] = u >= v ? u - v : u + q - v;
      }
    }
  }
}
static void r_intt(const of_subring* S, uint64_t* p) {
  uint64_t q = S->q;
  int N = S->d, t = 1;
  for (int m = N / 2; m >= 1; m >>= 1) {
    for (int i = 0; i < m; ++i) {
      uint64_t w = S->iroots[m + i];
      for (int j = 2 * i * t; j < 2 * i * t + t; ++j) {
        uint64_t u = p[j], v = p[j + t];
        p[j] = u + v >= q ? u + v - q : u + v;
        p[j + t] = mulmod(u >= v ? u - v : u + q - v, w, q);
      }
    }
    t <<= 1;
  }
  for (int j = 0; j < N; ++j) p[j] = mulmod(p[j], S->ninv, q);
}
static inline uint64_t signed_res(int64_t c, uint64_t q) { /* setCoeffSigned (utils.go:49-61) */
  if (c >= 0) return (uint64_t)c;
  uint64_t a = (uint64_t)(-(c + 1)) + 1; /* |c| */
  return q - a % q;                      /* Go: c%q + q  (== q when q | c) */
}

/* ------------------------------------------------------------------------------------------ */
/* Jindo commit with injected randomness (layouts: include/ringo.h rg_jindo_commit)            */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  int rank, rows, cols, slots, exp, d, in_msis, out_msis, mlwe, dcmp, log_in_cut, log_out_cut;
  uint64_t base;
  int nq, nqo;
  uint64_t q[4], qo[4];
  int field_limbs;
  uint64_t field_q[MAXL];
} of_jindo_params;

typedef struct {
  of_jindo_params P;
  of_field F;
  of_subring rq[4], ro[4];
} of_jindo;

of_jindo* of_jindo_create(const of_jindo_params* P) {
  if (P->nq < 1 || P->nq > 4 || P->nqo < 1 || P->nqo > 4 || P->nqo > P->nq) return 0;
  of_jindo* J = (of_jindo*)calloc(1, sizeof(of_jindo));
  J->P = *P;
  if (of_field_init(&J->F, P->field_limbs, P->field_q)) { free(J); return 0; }
  for (int l = 0; l < P->nq; ++l) subring_init(&J->rq[l], P->d, P->q[l]);
  for (int l = 0; l < P->nqo; ++l) subring_init(&J->ro[l], P->d, P->qo[l]);
  return J;
}
void of_jindo_destroy(of_jindo* J) {
  for (int l = 0; l < J->P.nq; ++l) subring_free(&J->rq[l]);
  for (int l = 0; l < J->P.nqo; ++l) subring_free(&J->ro[l]);
  free(J);
}

/* baseEncodeTo (encoder.go:120-146): digits[d] from n<=slots Montgomery elements. */
static void base_encode(const of_jindo* J, uint64_t* digits, const uint64_t* v, int n) {
  const of_jindo_params* P = &J->P;
  int L = J->F.L;
  memset(digits, 0, 8 * (size_t)P->d);
  uint64_t one[MAXL] = {1}, c[MAXL];
  for (int i = 0; i < n; ++i) {
    f_mul(&J->F, c, v + (size_t)i * L, one, L); /* Slice = fromMont (element.go:1769-1773) */
    for (int j = 0; j < P->exp - 1; ++j) {       /* divMod64 (utils.go:12-19) */
      uint64_t r = 0;
      for (int k = L - 1; k >= 0; --k) {
        u128 num = ((u128)r << 64) | c[k];
        c[k] = (uint64_t)(num / P->base);
        r = (uint64_t)(num % P->base);
      }
      digits[j * P->slots + i] = r;
    }
    digits[(P->exp - 1) * P->slots + i] = c[0];
  }
}
/* randEncodeTo tail (encoder.go:166-200) with injected samples; out: [nq][d]. */
static void rand_encode(const of_jindo* J, uint64_t* out, const uint64_t* v, int n, const int64_t* noise) {
  const of_jindo_params* P = &J->P;
  int d = P->d, sl = P->slots;
  uint64_t* digits = (uint64_t*)malloc(8 * (size_t)d);
  uint64_t* s = (uint64_t*)malloc(8 * (size_t)d);
  uint64_t* sh = (uint64_t*)malloc(8 * (size_t)d);
  base_encode(J, digits, v, n);
  for (int l = 0; l < P->nq; ++l) {
    const of_subring* S = &J->rq[l];
    uint64_t q = S->q;
    for (int i = 0; i < d; ++i) s[i] = mulmod(signed_res(noise[i], q), S->m, q); /* MForm :184 */
    for (int i = 0; i + sl < d; ++i) sh[i + sl] = s[i];                          /* :186-190 */
    for (int i = d - sl; i < d; ++i) sh[i - (d - sl)] = q - s[i];                  /* :191-195 */
    uint64_t b = P->base % q;
    for (int i = 0; i < d; ++i) { /* MulScalarThenSub :196 ; MForm(digits)+Add :198-199 */
      uint64_t x = sh[i] % q, y = mulmod(s[i], b, q);
      x = x >= y ? x - y : x + q - y;
      uint64_t dm = mulmod(digits[i] % q, S->m, q);
      x += dm;
      if (x >= q) x -= q;
      out[(size_t)l * d + i] = x;
    }
    r_ntt(S, out + (size_t)l * d); /* :200 */
  }
  free(digits);
  free(s);
  free(sh);
}
/* multi-word signed helpers for CRT rounding (rns.go:76-114) ------------------------------- */
#define W 4 /* words: Q <= 4*61 bits */
static void mw_from_u64(uint64_t* a, uint64_t v) { memset(a, 0, 8 * W); a[0] = v; }
static void mw_muladd(uint64_t* a, uint64_t m, uint64_t add) { /* a = a*m + add */
  uint64_t c = add;
  for (int i = 0; i < W; ++i) {
    u128 s = (u128)a[i] * m + c;
    a[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
}
static int mw_geq(const uint64_t* a, const uint64_t* b) { return geq(a, b, W); }
/* centred CRT + arithmetic shift + per-prime Euclidean mod; residues r[nsrc] (plain, coeff
 * domain) -> out[l] = (centre(V) >> cut) mod qo[l]. */
static void crt_round(const of_subring* src, int nsrc, const uint64_t* r, int cut, const of_subring* dst, int ndst,
                      uint64_t* out) {
  int neg = 0;
  uint64_t mag[W]; /* |value| before shift */
  {
    /* balanced fast path (rns.go:78-91); always taken for a single-prime ring */
    int64_t b0 = (int64_t)(r[0] > (src[0].q >> 1) ? r[0] - src[0].q : r[0]);
    int same = 1;
    for (int j = 1; j < nsrc; ++j) {
      int64_t bj = (int64_t)(r[j] > (src[j].q >> 1) ? r[j] - src[j].q : r[j]);
      if (bj != b0) { same = 0; break; }
    }
    if (same) {
      neg = b0 < 0;
      mw_from_u64(mag, neg ? (uint64_t)(-(b0 + 1)) + 1 : (uint64_t)b0);
      goto shifted;
    }
  }
  {
    /* Garner: V = x0 + q0*(x1 + q1*(x2 + ...)) in [0, Q)  (== sum r_j*gad_j mod Q, :93-99) */
    uint64_t x[4];
    for (int j = 0; j < nsrc; ++j) {
      uint64_t q = src[j].q, v = r[j] % q;
      for (int k = 0; k < j; ++k) { /* v = (v - x_k) * inv(q_k) mod q */
        uint64_t xk = x[k] % q;
        v = v >= xk ? v - xk : v + q - xk;
        v = mulmod(v, powmod(src[k].q % q, q - 2, q), q);
      }
      x[j] = v;
    }
    uint64_t V[W], Q[W], Qh[W];
    mw_from_u64(V, x[nsrc - 1]);
    for (int j = nsrc - 2; j >= 0; --j) mw_muladd(V, src[j].q, x[j]);
    mw_from_u64(Q, 1);
    for (int j = 0; j < nsrc; ++j) mw_muladd(Q, src[j].q, 0);
    shr_n(Qh, Q, W, 1);
    if (mw_geq(V, Qh)) { /* acc >= Q>>1 -> acc - Q (:100-102) */
      neg = 1;
      sub_n(mag, Q, V, W);
    } else {
      memcpy(mag, V, 8 * W);
    }
  }
shifted:;
  /* floor shift (big.Int.Rsh): negative -> -ceil(mag / 2^cut) */
  uint64_t sh[W];
  memcpy(sh, mag, 8 * W);
  int lost = 0;
  for (int c = cut; c > 0;) {
    int s = c > 63 ? 63 : c;
    uint64_t lowmask = (1ull << s) - 1;
    lost |= (sh[0] & lowmask) != 0;
    shr_n(sh, sh, W, s);
    c -= s;
  }
  if (neg && lost) { /* sh += 1 */
    for (int k = 0; k < W; ++k) if (++sh[k]) break;
  }
  int zero = 1;
  for (int k = 0; k < W; ++k) zero &= sh[k] == 0;
  for (int l = 0; l < ndst; ++l) { /* setBigCoeffTo: Euclidean mod (rns.go:108-114) */
    uint64_t q = dst[l].q;
    u128 rr = 0;
    for (int k = W - 1; k >= 0; --k) rr = ((rr << 64) | sh[k]) % q;
    uint64_t m = (uint64_t)rr;
    out[l] = (neg && !zero && m) ? q - m : m;
  }
}

/* IMForm -> INTT -> CRT round -> MForm -> NTT in the destination ring (prover.go:164-176). */
static void round_poly(const of_jindo* J, const of_subring* src, int nsrc, uint64_t* poly /* [nsrc][d] */, int cut,
                       const of_subring* dst, int ndst, uint64_t* out /* [ndst][d] */) {
  int d = J->P.d;
  for (int l = 0; l < nsrc; ++l) {
    uint64_t* p = poly + (size_t)l * d;
    for (int k = 0; k < d; ++k) p[k] = mulmod(p[k], src[l].minv, src[l].q);
    r_intt(&src[l], p);
  }
  uint64_t r[4], o[4];
  for (int k = 0; k < d; ++k) {
    for (int l = 0; l < nsrc; ++l) r[l] = poly[(size_t)l * d + k];
    crt_round(src, nsrc, r, cut, dst, ndst, o);
    for (int l = 0; l < ndst; ++l) out[(size_t)l * d + k] = mulmod(o[l], dst[l].m, dst[l].q);
  }
  for (int l = 0; l < ndst; ++l) r_ntt(&dst[l], out + (size_t)l * d);
}

static inline void mac_mont(uint64_t* acc, const uint64_t* a, const uint64_t* b, const of_subring* S, int d) {
  for (int k = 0; k < d; ++k) { /* MulCoeffsMontgomeryThenAdd: acc += a*b*2^-64 */
    uint64_t t = mulmod(mulmod(a[k], b[k], S->q), S->minv, S->q);
    acc[k] += t;
    if (acc[k] >= S->q) acc[k] -= S->q;
  }
}

/* The deterministic Ajtai core of Commit from the NTT-domain opening: the inner MACs, rounding
 * and InCommit of every column (prover.go:144-176), then outerCommitTo (:180-202).
 *   enc [cols+1][rows][nq][d], mlwe [cols+1][in_msis+mlwe][nq][d] -> incom, com */
int of_jindo_commit_core(const of_jindo* J, const uint64_t* ck_in, const uint64_t* ck_mlwe, const uint64_t* ck_out,
                         const uint64_t* o_enc, const uint64_t* o_mlwe, uint64_t* o_incom, uint64_t* o_com) {
  const of_jindo_params* P = &J->P;
  const int d = P->d, nq = P->nq, nqo = P->nqo, nm = P->in_msis + P->mlwe;
  const size_t polyq = (size_t)nq * d, polyo = (size_t)nqo * d;
  uint64_t* com = (uint64_t*)malloc(8 * polyq);
  for (int i = 0; i <= P->cols; ++i) {
    const uint64_t* enc = o_enc + (size_t)i * P->rows * polyq;
    const uint64_t* ml = o_mlwe + (size_t)i * nm * polyq;
    for (int j = 0; j < P->in_msis; ++j) { /* prover.go:149-176 */
      for (int l = 0; l < nq; ++l) {
        const of_subring* S = &J->rq[l];
        uint64_t* acc = com + (size_t)l * d;
        memset(acc, 0, 8 * (size_t)d);
        for (int k = 0; k < P->rows; ++k)
          mac_mont(acc, ck_in + (((size_t)j * P->rows + k) * nq + l) * d, enc + (size_t)k * polyq + (size_t)l * d, S, d);
        for (int k = 0; k < P->mlwe; ++k)
          mac_mont(acc, ck_mlwe + (((size_t)j * P->mlwe + k) * nq + l) * d, ml + (size_t)k * polyq + (size_t)l * d, S, d);
        const uint64_t* e = ml + (size_t)(P->mlwe + j) * polyq + (size_t)l * d;
        for (int k = 0; k < d; ++k) {
          acc[k] += e[k];
          if (acc[k] >= S->q) acc[k] -= S->q;
        }
      }
      round_poly(J, J->rq, nq, com, P->log_in_cut, J->ro, nqo, o_incom + (size_t)(i * P->in_msis + j) * polyo);
    }
  }
  /* outerCommitTo (prover.go:180-202) */
  memset(o_com, 0, 8 * polyq * (size_t)P->out_msis);
  uint64_t* oc = (uint64_t*)malloc(8 * polyo);
  for (int i = 0; i < P->out_msis; ++i) {
    for (int l = 0; l < nqo; ++l) {
      uint64_t* acc = oc + (size_t)l * d;
      memset(acc, 0, 8 * (size_t)d);
      for (int j = 0; j < P->dcmp; ++j)
        mac_mont(acc, ck_out + (((size_t)i * P->dcmp + j) * nqo + l) * d, o_incom + (size_t)j * polyo + (size_t)l * d,
                 &J->ro[l], d);
    }
    round_poly(J, J->ro, nqo, oc, P->log_out_cut, J->ro, nqo, o_com + (size_t)i * polyq);
  }
  free(oc);
  free(com);
  return 0;
}

/* One commit.  See include/ringo.h rg_jindo_commit for every layout. */
int of_jindo_commit(const of_jindo* J, const uint64_t* ck_in, const uint64_t* ck_mlwe, const uint64_t* ck_out,
                    const uint64_t* v, long nv, const uint64_t* last_row, const uint64_t* mask, const int64_t* enc_noise,
                    const int64_t* mlwe_noise, uint64_t* o_incom, uint64_t* o_enc, uint64_t* o_mlwe, uint64_t* o_com) {
  const of_jindo_params* P = &J->P;
  int L = J->F.L, d = P->d, nq = P->nq, cs = P->cols * P->slots, nm = P->in_msis + P->mlwe;
  if (nv > P->rank || nv < 1) return -1;
  size_t polyq = (size_t)nq * d;
  uint64_t* first = (uint64_t*)calloc((size_t)cs * L, 8);
  memcpy(first, v, 8 * L); /* genFirstLastRow (prover.go:74-83) */
  uint64_t zero[MAXL] = {0};
  for (int i = 1; i < cs; ++i)
    f_sub(&J->F, first + (size_t)i * L, i < nv ? v + (size_t)i * L : zero, last_row + (size_t)(i - 1) * L, L);
  memset(o_enc, 0, 8 * polyq * (size_t)(P->cols + 1) * P->rows);
  for (int i = 0; i <= P->cols; ++i) {
    const int64_t* en = enc_noise + (size_t)i * P->rows * d;
    uint64_t* enc = o_enc + (size_t)i * P->rows * polyq;
    int rs = i * P->slots, re = (i + 1) * P->slots;
    if (i == P->cols) { /* prover.go:93-115 */
      rand_encode(J, enc, mask, P->slots, en);
      for (int j = 1; j < P->rows - 1; ++j) {
        if ((long)j * cs > nv) break;
        rand_encode(J, enc + (size_t)j * polyq, mask + (size_t)j * P->slots * L, P->slots, en + (size_t)j * d);
      }
      rand_encode(J, enc + (size_t)(P->rows - 1) * polyq, mask + (size_t)(P->rows - 1) * P->slots * L, P->slots,
                  en + (size_t)(P->rows - 1) * d);
    } else { /* prover.go:116-128 */
      rand_encode(J, enc, first + (size_t)rs * L, P->slots, en);
      for (int j = 1; j < P->rows - 1; ++j) {
        long s0 = (long)j * cs + rs, e0 = (long)j * cs + re;
        if (s0 > nv) break;
        long e1 = e0 < nv ? e0 : nv;
        rand_encode(J, enc + (size_t)j * polyq, v + (size_t)s0 * L, (int)(e1 - s0), en + (size_t)j * d);
      }
      rand_encode(J, enc + (size_t)(P->rows - 1) * polyq, last_row + (size_t)rs * L, P->slots,
                  en + (size_t)(P->rows - 1) * d);
    }
    uint64_t* ml = o_mlwe + (size_t)i * nm * polyq; /* prover.go:130-142 */
    for (int j = 0; j < nm; ++j) {
      const int64_t* mn = mlwe_noise + ((size_t)i * nm + j) * d;
      for (int l = 0; l < nq; ++l) {
        const of_subring* S = &J->rq[l];
        uint64_t* p = ml + (size_t)j * polyq + (size_t)l * d;
        for (int k = 0; k < d; ++k) p[k] = mulmod(signed_res(mn[k], S->q), S->m, S->q);
        r_ntt(S, p);
      }
    }
  }
  free(first);
  return of_jindo_commit_core(J, ck_in, ck_mlwe, ck_out, o_enc, o_mlwe, o_incom, o_com);
}

/* ------------------------------------------------------------------------------------------ */
/* Prover.Evaluate core (jindo/prover.go:205-324) with the Fiat-Shamir challenges injected:   */
/* the transcript (SHAKE128 over Lattigo serializations), encodeChallengeTo and leftVec stay  */
/* on the host; these are the MulCoeffsMontgomeryThenAdd loops.  Layouts: include/ringo.h.   */
/* ------------------------------------------------------------------------------------------ */
/* openBatch = sum_i open[i] * batch[i] (prover.go:228-266); batch == 1: open[0] (:267-269) */
void of_jindo_eval_batch(const of_jindo* J, long batch, const uint64_t* incom, const uint64_t* enc,
                         const uint64_t* mlwe, const uint64_t* bq, const uint64_t* bo, uint64_t* ob_incom,
                         uint64_t* ob_enc, uint64_t* ob_mlwe) {
  const of_jindo_params* P = &J->P;
  const int d = P->d, nq = P->nq, nqo = P->nqo, nm = P->in_msis + P->mlwe;
  const size_t polyq = (size_t)nq * d, polyo = (size_t)nqo * d;
  const size_t n_inc = (size_t)P->dcmp, n_enc = (size_t)(P->cols + 1) * P->rows, n_ml = (size_t)(P->cols + 1) * nm;
  if (batch == 1) {
    memcpy(ob_incom, incom, 8 * n_inc * polyo);
    memcpy(ob_enc, enc, 8 * n_enc * polyq);
    memcpy(ob_mlwe, mlwe, 8 * n_ml * polyq);
    return;
  }
  memset(ob_incom, 0, 8 * n_inc * polyo);
  memset(ob_enc, 0, 8 * n_enc * polyq);
  memset(ob_mlwe, 0, 8 * n_ml * polyq);
  for (long i = 0; i < batch; ++i) {
    for (size_t j = 0; j < n_inc; ++j)
      for (int l = 0; l < nqo; ++l)
        mac_mont(ob_incom + j * polyo + (size_t)l * d, incom + ((size_t)i * n_inc + j) * polyo + (size_t)l * d,
                 bo + (size_t)i * polyo + (size_t)l * d, &J->ro[l], d);
    for (size_t j = 0; j < n_enc; ++j)
      for (int l = 0; l < nq; ++l)
        mac_mont(ob_enc + j * polyq + (size_t)l * d, enc + ((size_t)i * n_enc + j) * polyq + (size_t)l * d,
                 bq + (size_t)i * polyq + (size_t)l * d, &J->rq[l], d);
    for (size_t j = 0; j < n_ml; ++j)
      for (int l = 0; l < nq; ++l)
        mac_mont(ob_mlwe + j * polyq + (size_t)l * d, mlwe + ((size_t)i * n_ml + j) * polyq + (size_t)l * d,
                 bq + (size_t)i * polyq + (size_t)l * d, &J->rq[l], d);
  }
}

/* pf.Partial[i] = sum_j left[j] * Enc[i][j] (i < cols), PartialMask the same over column cols
   (prover.go:274-286); partial: [cols+1][nq][d], the last polynomial is PartialMask */
void of_jindo_eval_partial(const of_jindo* J, const uint64_t* ob_enc, const uint64_t* left, uint64_t* partial) {
  const of_jindo_params* P = &J->P;
  const int d = P->d, nq = P->nq;
  const size_t polyq = (size_t)nq * d;
  memset(partial, 0, 8 * (size_t)(P->cols + 1) * polyq);
  for (int i = 0; i <= P->cols; ++i)
    for (int j = 0; j < P->rows; ++j)
      for (int l = 0; l < nq; ++l)
        mac_mont(partial + (size_t)i * polyq + (size_t)l * d, left + (size_t)j * polyq + (size_t)l * d,
                 ob_enc + ((size_t)i * P->rows + j) * polyq + (size_t)l * d, &J->rq[l], d);
}

/* pf.Encode[i] = Enc[cols][i] + sum_j chals[j] * Enc[j][i]; pf.MLWE[i] likewise over the
   inMSIS + mlwe MLWE polynomials (prover.go:300-314) */
void of_jindo_eval_respond(const of_jindo* J, const uint64_t* ob_enc, const uint64_t* ob_mlwe, const uint64_t* chals,
                           uint64_t* pf_enc, uint64_t* pf_mlwe) {
  const of_jindo_params* P = &J->P;
  const int d = P->d, nq = P->nq, nm = P->in_msis + P->mlwe;
  const size_t polyq = (size_t)nq * d;
  for (int i = 0; i < P->rows; ++i) {
    memcpy(pf_enc + (size_t)i * polyq, ob_enc + ((size_t)P->cols * P->rows + i) * polyq, 8 * polyq);
    for (int j = 0; j < P->cols; ++j)
      for (int l = 0; l < nq; ++l)
        mac_mont(pf_enc + (size_t)i * polyq + (size_t)l * d, chals + (size_t)j * polyq + (size_t)l * d,
                 ob_enc + ((size_t)j * P->rows + i) * polyq + (size_t)l * d, &J->rq[l], d);
  }
  for (int i = 0; i < nm; ++i) {
    memcpy(pf_mlwe + (size_t)i * polyq, ob_mlwe + ((size_t)P->cols * nm + i) * polyq, 8 * polyq);
    for (int j = 0; j < P->cols; ++j)
      for (int l = 0; l < nq; ++l)
        mac_mont(pf_mlwe + (size_t)i * polyq + (size_t)l * d, chals + (size_t)j * polyq + (size_t)l * d,
                 ob_mlwe + ((size_t)j * nm + i) * polyq + (size_t)l * d, &J->rq[l], d);
  }
}

/* ------------------------------------------------------------------------------------------ */
/* Verifier.Verify (jindo/verifier.go:50-282) with the Fiat-Shamir challenges injected (the   */
/* transcript, encodeChallengeTo, leftVec/rightVec/encode stay with the caller, as in          */
/* Evaluate).  Layouts: include/ringo.h rg_jindo_verify_dev.                                   */
/* ------------------------------------------------------------------------------------------ */
#define NW 10 /* words of a sum of squares */
/* reconstructTo (rns.go:76-105): centred value of one coefficient -> sign + magnitude */
static void crt_centred(const of_subring* src, int nsrc, const uint64_t* r, int* neg, uint64_t* mag /* [W] */) {
  int64_t b0 = (int64_t)(r[0] > (src[0].q >> 1) ? r[0] - src[0].q : r[0]);
  int same = 1;
  for (int j = 1; j < nsrc; ++j) {
    int64_t bj = (int64_t)(r[j] > (src[j].q >> 1) ? r[j] - src[j].q : r[j]);
    if (bj != b0) { same = 0; break; }
  }
  if (same) {
    *neg = b0 < 0;
    mw_from_u64(mag, *neg ? (uint64_t)(-(b0 + 1)) + 1 : (uint64_t)b0);
    return;
  }
  uint64_t x[4];
  for (int j = 0; j < nsrc; ++j) {
    uint64_t q = src[j].q, v = r[j] % q;
    for (int k = 0; k < j; ++k) {
      uint64_t xk = x[k] % q;
      v = v >= xk ? v - xk : v + q - xk;
      v = mulmod(v, powmod(src[k].q % q, q - 2, q), q);
    }
    x[j] = v;
  }
  uint64_t V[W], Q[W], Qh[W];
  mw_from_u64(V, x[nsrc - 1]);
  for (int j = nsrc - 2; j >= 0; --j) mw_muladd(V, src[j].q, x[j]);
  mw_from_u64(Q, 1);
  for (int j = 0; j < nsrc; ++j) mw_muladd(Q, src[j].q, 0);
  shr_n(Qh, Q, W, 1);
  *neg = mw_geq(V, Qh);
  if (*neg)
    sub_n(mag, Q, V, W);
  else
    memcpy(mag, V, 8 * W);
}
/* IMForm + INTT of one [n][d] polynomial, in place (verifier.go:99-114) */
static void inv_poly(const of_jindo* J, const of_subring* R, int n, uint64_t* p) {
  int d = J->P.d;
  for (int l = 0; l < n; ++l) {
    for (int k = 0; k < d; ++k) p[(size_t)l * d + k] = mulmod(p[(size_t)l * d + k], R[l].minv, R[l].q);
    r_intt(&R[l], p + (size_t)l * d);
  }
}
/* sum of squares of the centred coefficients of npoly NTT+Montgomery polys (verifyNorm :262-276) */
static void norm_sq_add(const of_jindo* J, const of_subring* R, int n, const uint64_t* polys, long npoly,
                        size_t stride, uint64_t* acc /* [NW] */) {
  int d = J->P.d;
  uint64_t* t = (uint64_t*)malloc(8 * (size_t)n * d);
  for (long i = 0; i < npoly; ++i) {
    for (int l = 0; l < n; ++l) memcpy(t + (size_t)l * d, polys + i * stride + (size_t)l * d, 8 * (size_t)d);
    inv_poly(J, R, n, t);
    for (int k = 0; k < d; ++k) {
      uint64_t r[4], mag[W], sq[2 * W];
      int neg;
      for (int l = 0; l < n; ++l) r[l] = t[(size_t)l * d + k];
      crt_centred(R, n, r, &neg, mag);
      memset(sq, 0, sizeof(sq));
      for (int a = 0; a < W; ++a) {
        uint64_t c = 0;
        for (int b = 0; b < W; ++b) {
          u128 s2 = (u128)mag[a] * mag[b] + sq[a + b] + c;
          sq[a + b] = (uint64_t)s2;
          c = (uint64_t)(s2 >> 64);
        }
        sq[a + W] += c;
      }
      uint64_t c = 0;
      for (int w = 0; w < NW; ++w) {
        u128 s2 = (u128)acc[w] + (w < 2 * W ? sq[w] : 0) + c;
        acc[w] = (uint64_t)s2;
        c = (uint64_t)(s2 >> 64);
      }
    }
  }
  free(t);
}
/* nmTest < nm with nmTest = Float64(floor(sqrt(S))) (verifyNorm :278-281), decided exactly:
   the largest integer T with (double)T < nm is K - 1 where K = the smallest T with (double)T >= nm,
   so the test is S < K^2.  The double nm = M 2^E (M < 2^53): K = ceil(nm) when nm <= 2^53, else
   the midpoint below nm, plus one when M is odd (ties round to even). */
static int norm_below(const uint64_t* S, double nm) {
  if (!(nm > 0)) return 0;
  uint64_t K[NW] = {0}, K2[2 * NW];
  int e;
  double fr = frexp(nm, &e); /* nm = fr 2^e, fr in [0.5, 1) */
  uint64_t M = (uint64_t)ldexp(fr, 53);
  int E = e - 53;
  if (E <= 0) {
    double c = ceil(nm);
    if (c >= 18446744073709551616.0) return 1;
    K[0] = (uint64_t)c;
  } else {
    /* nm = M 2^E; the double below is nm - 2^E, or nm - 2^(E-1) when M = 2^52 */
    int sub_e = (M == (1ull << 52)) ? E - 2 : E - 1; /* half the gap below */
    /* K = M 2^E - 2^sub_e (+1 if M odd) */
    K[E / 64] = M << (E % 64);
    if (E % 64 && E / 64 + 1 < NW) K[E / 64 + 1] = M >> (64 - E % 64);
    uint64_t h[NW] = {0};
    if (sub_e >= 0) h[sub_e / 64] = 1ull << (sub_e % 64);
    sub_n(K, K, h, NW);
    if (M & 1) {
      for (int k = 0; k < NW; ++k) if (++K[k]) break;
    }
  }
  memset(K2, 0, sizeof(K2));
  for (int a = 0; a < NW; ++a) {
    uint64_t c = 0;
    for (int b = 0; b < NW; ++b) {
      u128 s2 = (u128)K[a] * K[b] + K2[a + b] + c;
      K2[a + b] = (uint64_t)s2;
      c = (uint64_t)(s2 >> 64);
    }
    K2[a + NW] += c;
  }
  for (int w = 2 * NW - 1; w >= NW; --w) if (K2[w]) return 1; /* K^2 exceeds any S */
  for (int w = NW - 1; w >= 0; --w)
    if (S[w] != K2[w]) return S[w] < K2[w];
  return 0;
}
int of_norm_below(const uint64_t* S, double nm) { return norm_below(S, nm); }
/* Decode (encoder.go:203-219) of one NTT+Montgomery ringQ polynomial: nout slots -> Montgomery */
static void decode_poly(const of_jindo* J, const uint64_t* poly, int nout, uint64_t* out) {
  const of_jindo_params* P = &J->P;
  int d = P->d, L = J->F.L, nq = P->nq;
  uint64_t* t = (uint64_t*)malloc(8 * (size_t)nq * d);
  uint64_t* ce = (uint64_t*)malloc(8 * (size_t)d * L);
  memcpy(t, poly, 8 * (size_t)nq * d);
  inv_poly(J, J->rq, nq, t);
  uint64_t two32[MAXL], two64[MAXL], bm[MAXL];
  f_from_u64(&J->F, two32, 1ull << 32);
  f_mul(&J->F, two64, two32, two32, L);
  f_from_u64(&J->F, bm, P->base);
  for (int k = 0; k < d; ++k) { /* SetBigInt of the centred value (element.go SetBigInt: mod p) */
    uint64_t r[4], mag[W], acc[MAXL] = {0}, wv[MAXL];
    int neg;
    for (int l = 0; l < nq; ++l) r[l] = t[(size_t)l * d + k];
    crt_centred(J->rq, nq, r, &neg, mag);
    for (int w = W - 1; w >= 0; --w) {
      f_mul(&J->F, acc, acc, two64, L);
      f_from_u64(&J->F, wv, mag[w]);
      f_add(&J->F, acc, acc, wv, L);
    }
    if (neg) f_neg(&J->F, acc, acc, L);
    memcpy(ce + (size_t)k * L, acc, 8 * (size_t)L);
  }
  for (int i = 0; i < nout; ++i) {
    uint64_t v[MAXL] = {0};
    for (int j = P->exp - 1; j >= 0; --j) {
      f_mul(&J->F, v, v, bm, L);
      f_add(&J->F, v, v, ce + (size_t)(j * P->slots + i) * L, L);
    }
    memcpy(out + (size_t)i * L, v, 8 * (size_t)L);
  }
  free(t);
  free(ce);
}
/* res[0..NW) outer nmSq, res[NW..2NW) inner nmSq, flags[4] = outer, inner, consistency, eval;
   evals[2][L] = (sum right*dcd, yBatch).  Returns 1 iff all four checks pass. */
int of_jindo_verify(const of_jindo* J, const uint64_t* ck_in, const uint64_t* ck_mlwe, const uint64_t* ck_out,
                    long batch, const uint64_t* com, const uint64_t* bq, const uint64_t* bo, const uint64_t* chals,
                    const uint64_t* left, const uint64_t* right, const uint64_t* y, const uint64_t* pf_incom,
                    const uint64_t* pf_partial, const uint64_t* pf_enc, const uint64_t* pf_mlwe, double in_com_dcmp_two_nm,
                    double res_two_nm, uint64_t* res, int* flags, uint64_t* evals) {
  const of_jindo_params* P = &J->P;
  const int d = P->d, nq = P->nq, nqo = P->nqo, nm = P->in_msis + P->mlwe, L = J->F.L;
  const size_t polyq = (size_t)nq * d, polyo = (size_t)nqo * d;
  memset(res, 0, 8 * 2 * NW);
  /* verifyOuterCommitment (:136-161) */
  norm_sq_add(J, J->ro, nqo, pf_incom, P->dcmp, polyo, res);
  uint64_t* c = (uint64_t*)malloc(8 * polyq);
  for (int i = 0; i < P->out_msis; ++i) {
    for (int l = 0; l < nqo; ++l) {
      const of_subring* S = &J->ro[l];
      uint64_t* a = c + (size_t)l * d;
      if (batch > 1) {
        memset(a, 0, 8 * (size_t)d);
        for (long j = 0; j < batch; ++j)
          mac_mont(a, com + ((size_t)j * P->out_msis + i) * polyq + (size_t)l * d, bo + (size_t)j * polyo + (size_t)l * d, S, d);
      } else {
        memcpy(a, com + (size_t)i * polyq + (size_t)l * d, 8 * (size_t)d);
      }
      uint64_t cut = powmod(2, (uint64_t)P->log_out_cut, S->q); /* MulRNSScalarMontgomery(MForm(2^cut)) */
      for (int k = 0; k < d; ++k) a[k] = mulmod(a[k], cut, S->q);
      uint64_t* b = (uint64_t*)calloc((size_t)d, 8);
      for (int j = 0; j < P->dcmp; ++j)
        mac_mont(b, ck_out + (((size_t)i * P->dcmp + j) * nqo + l) * d, pf_incom + (size_t)j * polyo + (size_t)l * d, S, d);
      for (int k = 0; k < d; ++k) a[k] = a[k] >= b[k] ? a[k] - b[k] : a[k] + S->q - b[k]; /* ...ThenSub */
      free(b);
    }
    norm_sq_add(J, J->ro, nqo, c, 1, polyo, res);
  }
  flags[0] = norm_below(res, in_com_dcmp_two_nm);
  /* verifyInnerCommitment (:164-200) */
  uint64_t* lift = (uint64_t*)malloc(8 * polyq * (size_t)P->dcmp);
  {
    uint64_t* t = (uint64_t*)malloc(8 * polyo);
    for (int j = 0; j < P->dcmp; ++j) { /* MForm(NTT(ModUpQtoP(pfInv.InCommit[j]))): centred lift */
      memcpy(t, pf_incom + (size_t)j * polyo, 8 * polyo);
      round_poly(J, J->ro, nqo, t, 0, J->rq, nq, lift + (size_t)j * polyq);
    }
    free(t);
  }
  norm_sq_add(J, J->rq, nq, pf_enc, P->rows, polyq, res + NW);
  norm_sq_add(J, J->rq, nq, pf_mlwe, nm, polyq, res + NW);
  for (int i = 0; i < P->in_msis; ++i) {
    for (int l = 0; l < nq; ++l) {
      const of_subring* S = &J->rq[l];
      uint64_t* a = c + (size_t)l * d;
      memset(a, 0, 8 * (size_t)d);
      for (int j = 0; j <= P->cols; ++j) {
        const uint64_t* lj = lift + (size_t)(j * P->in_msis + i) * polyq + (size_t)l * d;
        if (j == P->cols) {
          for (int k = 0; k < d; ++k) { a[k] += lj[k]; if (a[k] >= S->q) a[k] -= S->q; }
        } else {
          mac_mont(a, lj, chals + (size_t)j * polyq + (size_t)l * d, S, d);
        }
      }
      uint64_t cut = powmod(2, (uint64_t)P->log_in_cut, S->q);
      for (int k = 0; k < d; ++k) a[k] = mulmod(a[k], cut, S->q);
      uint64_t* b = (uint64_t*)calloc((size_t)d, 8);
      for (int j = 0; j < P->rows; ++j)
        mac_mont(b, ck_in + (((size_t)i * P->rows + j) * nq + l) * d, pf_enc + (size_t)j * polyq + (size_t)l * d, S, d);
      for (int j = 0; j < P->mlwe; ++j)
        mac_mont(b, ck_mlwe + (((size_t)i * P->mlwe + j) * nq + l) * d, pf_mlwe + (size_t)j * polyq + (size_t)l * d, S, d);
      const uint64_t* e = pf_mlwe + (size_t)(P->mlwe + i) * polyq + (size_t)l * d;
      for (int k = 0; k < d; ++k) {
        uint64_t bk = b[k] + e[k];
        if (bk >= S->q) bk -= S->q;
        a[k] = a[k] >= bk ? a[k] - bk : a[k] + S->q - bk;
      }
      free(b);
    }
    norm_sq_add(J, J->rq, nq, c, 1, polyq, res + NW);
  }
  free(lift);
  flags[1] = norm_below(res + NW, res_two_nm);
  /* verifyConsistency (:203-221) */
  int consistent = 1;
  for (int l = 0; l < nq; ++l) {
    const of_subring* S = &J->rq[l];
    uint64_t* a = c + (size_t)l * d;
    uint64_t* b = (uint64_t*)calloc((size_t)d, 8);
    memset(a, 0, 8 * (size_t)d);
    for (int i = 0; i < P->rows; ++i)
      mac_mont(a, left + (size_t)i * polyq + (size_t)l * d, pf_enc + (size_t)i * polyq + (size_t)l * d, S, d);
    for (int i = 0; i < P->cols; ++i)
      mac_mont(b, chals + (size_t)i * polyq + (size_t)l * d, pf_partial + (size_t)i * polyq + (size_t)l * d, S, d);
    const uint64_t* pm = pf_partial + (size_t)P->cols * polyq + (size_t)l * d;
    for (int k = 0; k < d; ++k) {
      uint64_t bk = b[k] + pm[k];
      if (bk >= S->q) bk -= S->q;
      consistent &= a[k] == bk;
    }
    free(b);
  }
  free(c);
  flags[2] = consistent;
  /* verifyEval (:224-259) */
  uint64_t* dcd = (uint64_t*)malloc(8 * (size_t)P->slots * L);
  uint64_t lhs[MAXL] = {0}, rhs[MAXL] = {0}, t[MAXL];
  for (int i = 0; i < P->cols; ++i) {
    decode_poly(J, pf_partial + (size_t)i * polyq, P->slots, dcd);
    for (int j = 0; j < P->slots; ++j) {
      f_mul(&J->F, t, right + (size_t)(i * P->slots + j) * L, dcd + (size_t)j * L, L);
      f_add(&J->F, lhs, lhs, t, L);
    }
  }
  if (batch > 1) {
    for (long i = 0; i < batch; ++i) {
      decode_poly(J, bq + (size_t)i * polyq, 1, dcd);
      f_mul(&J->F, t, dcd, y + (size_t)i * L, L);
      f_add(&J->F, rhs, rhs, t, L);
    }
  } else {
    memcpy(rhs, y, 8 * (size_t)L);
  }
  free(dcd);
  memcpy(evals, lhs, 8 * (size_t)L);
  memcpy(evals + L, rhs, 8 * (size_t)L);
  flags[3] = memcmp(lhs, rhs, 8 * (size_t)L) == 0;
  return flags[0] && flags[1] && flags[2] && flags[3];
}

/* encodeChallengeTo (utils.go:20-46) into one ring: coefficient i*slots <- signed digit i of the
   128-bit challenge in base ChallengeBound; then MForm and NTT.  ring = 0: ringQ, 1: ringQOut */
void of_jindo_encode_challenge(const of_jindo* J, int ring, const unsigned char* bytes16, uint64_t* out) {
  const of_jindo_params* P = &J->P;
  const of_subring* R = ring ? J->ro : J->rq;
  const int n = ring ? P->nqo : P->nq, d = P->d;
  uint64_t c[2] = {0, 0};
  for (int i = 0; i < 8; ++i) {
    c[0] = (c[0] << 8) | bytes16[i];
    c[1] = (c[1] << 8) | bytes16[8 + i];
  }
  uint64_t bnd = P->base < (1ull << (120 / P->exp)) ? P->base : (1ull << (120 / P->exp));
  bnd /= 2; /* ChallengeBound (params.go:357-360) */
  memset(out, 0, 8 * (size_t)n * d);
  for (int i = 0; i < P->exp; ++i) {
    uint64_t r = 0; /* divMod64 over [c0, c1] little-endian words */
    for (int k = 1; k >= 0; --k) {
      u128 num = ((u128)r << 64) | c[k];
      c[k] = (uint64_t)(num / bnd);
      r = (uint64_t)(num % bnd);
    }
    for (int l = 0; l < n; ++l) out[(size_t)l * d + (size_t)i * P->slots] = r > bnd / 2 ? R[l].q - (bnd - r) : r;
  }
  for (int l = 0; l < n; ++l) {
    uint64_t* p = out + (size_t)l * d;
    for (int k = 0; k < d; ++k) p[k] = mulmod(p[k], R[l].m, R[l].q);
    r_ntt(&R[l], p);
  }
}

/* Encoder.encode (encoder.go:105-117) of n <= slots Montgomery elements: ringQ NTT+Mont poly */
void of_jindo_encode(const of_jindo* J, const uint64_t* v, int n, uint64_t* out) {
  int64_t* zero = (int64_t*)calloc((size_t)J->P.d, 8);
  rand_encode(J, out, v, n, zero); /* no noise: MForm(digits), NTT */
  free(zero);
}

/* ------------------------------------------------------------------------------------------ */
/* Remaining bigpoly operators, literal restatements                   */
/* ------------------------------------------------------------------------------------------ */
/* CyclicEvaluator.QuoRemByVanishing (cyclic.go:18-37); N >= 0 */
void of_quorem_vanishing(const of_field* F, long rank, long N, uint64_t* quo, uint64_t* rem, const uint64_t* p) {
  const int L = F->L;
  memset(quo, 0, 8 * (size_t)rank * L);
  memcpy(rem, p, 8 * (size_t)rank * L);
  for (long i = rank - 1; i >= N; --i) {
    f_add(F, quo + (size_t)(i - N) * L, quo + (size_t)(i - N) * L, rem + (size_t)i * L, L);
    f_add(F, rem + (size_t)(i - N) * L, rem + (size_t)(i - N) * L, rem + (size_t)i * L, L);
    memset(rem + (size_t)i * L, 0, 8 * (size_t)L);
  }
}
/* CyclotomicEvaluator.AutTo (cyclotomic.go:29-86); idx odd */
void of_aut(const of_field* F, long rank, long idx, int ntt, uint64_t* out, const uint64_t* p) {
  const int L = F->L;
  const long n2 = 2 * rank;
  idx %= n2;
  if (idx < 0) idx += n2;
  uint64_t* buf = (uint64_t*)malloc(8 * (size_t)rank * L);
  if (!ntt) { /* autTo (:53-67) */
    for (long i = 0; i < rank; ++i) {
      long j = (long)(((unsigned long)i * (unsigned long)idx) % (unsigned long)n2);
      if (j < rank) memcpy(buf + (size_t)j * L, p + (size_t)i * L, 8 * (size_t)L);
      else f_neg(F, buf + (size_t)(j - rank) * L, p + (size_t)i * L, L);
    }
    memcpy(out, buf, 8 * (size_t)rank * L);
  } else { /* autNTTTo (:70-86) */
    memcpy(buf, p, 8 * (size_t)rank * L);
    bitrev_perm(buf, (int)rank, L);
    for (long i = 0; i < rank; ++i) {
      long j = (long)(((unsigned long)(2 * i + 1) * (unsigned long)idx) % (unsigned long)n2);
      j = (j - 1) >> 1;
      memcpy(out + (size_t)i * L, buf + (size_t)j * L, 8 * (size_t)L);
    }
    bitrev_perm(out, (int)rank, L);
  }
  free(buf);
}
/* Poly.Evaluate (poly.go:64-76): Horner from the top */
void of_poly_evaluate(const of_field* F, const uint64_t* p, long n, const uint64_t* x, uint64_t* out) {
  const int L = F->L;
  uint64_t z[MAXL] = {0};
  for (long i = n - 1; i >= 0; --i) {
    f_mul(F, z, z, x, L);
    f_add(F, z, z, p + (size_t)i * L, L);
  }
  memcpy(out, z, 8 * (size_t)L);
}

/* ------------------------------------------------------------------------------------------ */
/* Buckler prover device work, literal restatements                    */
/* ------------------------------------------------------------------------------------------ */
/* Encoder.EncodeTo / RandEncodeTo (buckler/encoder.go:32-54): out [emb][L] = cyclic InvNTT of
 * v [rank][L] (twinv/ninv: the CyclicTransformer's tables at `rank`), zeros above rank; with
 * rnd (the MustSetRandom draw, Montgomery) coeff[rank] = rnd and coeff[0] -= rnd. */
void of_buckler_encode(const of_field* F, const uint64_t* twinv, const uint64_t* ninv, int rank, long emb,
                       uint64_t* out, const uint64_t* v, const uint64_t* rnd) {
  const int L = F->L;
  of_ntt_inv(F, out, v, twinv, ninv, rank, 1); /* :33 InvNTTTo(pOut.Coeffs[:rank], v[:rank]) */
  memset(out + (size_t)rank * L, 0, 8 * (size_t)(emb - rank) * L); /* :34-36 SetUint64(0) */
  if (rnd) {
    memcpy(out + (size_t)rank * L, rnd, 8 * (size_t)L); /* :52 Coeffs[rank].MustSetRandom() */
    f_sub(F, out, out, out + (size_t)rank * L, L);      /* :53 Coeffs[0].Sub(Coeffs[0], Coeffs[rank]) */
  }
}
/* Prover.evalCircuit (buckler/prover.go:355-379), polynomial by polynomial as Go runs it:
 * constraint c has terms term_off[c] .. term_off[c+1]-1; term t: coeffs[t] ([L]), public
 * witness pw_idx[t] (< 0: none), witnesses wit_idx[wit_off[t] .. wit_off[t+1]-1].  w [n][rank][L]
 * and pw [n][rank][L] are the NTT-domain encodings; out [rank][L] (overwritten). */
void of_buckler_eval_circuit(const of_field* F, long rank, long nc, const long* term_off, const uint64_t* coeffs,
                             const long* pw_idx, const long* wit_off, const long* wit_idx, const uint64_t* bc,
                             const uint64_t* w, const uint64_t* pw, uint64_t* out) {
  const int L = F->L;
  const size_t n = (size_t)rank * L;
  uint64_t* eval = (uint64_t*)malloc(8 * n);
  uint64_t* term = (uint64_t*)malloc(8 * n);
  memset(out, 0, 8 * n); /* :356 pOut := NewPoly(true) */
  for (long c = 0; c < nc; ++c) {
    memset(eval, 0, 8 * n); /* :362 eval.Clear() */
    for (long t = term_off[c]; t < term_off[c + 1]; ++t) {
      for (long j = 0; j < rank; ++j) memcpy(term + (size_t)j * L, coeffs + (size_t)t * L, 8 * (size_t)L); /* :363-365 */
      if (pw_idx[t] >= 0) /* :366-368 MulTo(term, term, pwEcdNTT[..]) */
        for (long j = 0; j < rank; ++j)
          f_mul(F, term + (size_t)j * L, term + (size_t)j * L, pw + ((size_t)pw_idx[t] * rank + j) * L, L);
      for (long k = wit_off[t]; k < wit_off[t + 1]; ++k) /* :369-371 MulTo(term, term, wEcdNTT[..]) */
        for (long j = 0; j < rank; ++j)
          f_mul(F, term + (size_t)j * L, term + (size_t)j * L, w + ((size_t)wit_idx[k] * rank + j) * L, L);
      for (long j = 0; j < rank; ++j) f_add(F, eval + (size_t)j * L, eval + (size_t)j * L, term + (size_t)j * L, L); /* :372 */
    }
    for (long j = 0; j < rank; ++j) f_mul(F, eval + (size_t)j * L, eval + (size_t)j * L, bc, L); /* :374 ScalarMulTo */
    for (long j = 0; j < rank; ++j) f_add(F, out + (size_t)j * L, out + (size_t)j * L, eval + (size_t)j * L, L); /* :375 */
  }
  free(eval);
  free(term);
}

/* ------------------------------------------------------------------------------------------ */
/* Samplers (math/csprng) and the randomness Prover.Commit draws (prover.go:65-139,           */
/* encoder.go:149-183), restated from the Go source over OpenSSL's AES (loaded at run time)    */
/* with the library's instance layout (include/ringo.h rg_jindo_seeds): instance n of a domain */
/* is the UniformSampler whose IV is IV + n * 2^24.  Floats: IEEE double, no contraction       */
/* (built with -ffp-contract=off), glibc libm for exp/log/erfc.                                */
/* ------------------------------------------------------------------------------------------ */
#include <dlfcn.h>
#include <math.h>

typedef struct {
  unsigned char aes[256]; /* OpenSSL AES_KEY */
  unsigned char iv[16];
} of_dom;
static int (*p_aes_set)(const unsigned char*, int, void*);
static void (*p_aes_enc)(const unsigned char*, unsigned char*, const void*);
static unsigned char* (*p_sha384)(const unsigned char*, size_t, unsigned char*);
static int crypto_load(void) {
  if (p_aes_enc) return 0;
  void* h = dlopen("libcrypto.so.3", RTLD_NOW | RTLD_LOCAL);
  if (!h) h = dlopen("libcrypto.so", RTLD_NOW | RTLD_LOCAL);
  if (!h) return -1;
  p_aes_set = (int (*)(const unsigned char*, int, void*))dlsym(h, "AES_set_encrypt_key");
  p_sha384 = (unsigned char* (*)(const unsigned char*, size_t, unsigned char*))dlsym(h, "SHA384");
  p_aes_enc = (void (*)(const unsigned char*, unsigned char*, const void*))dlsym(h, "AES_encrypt");
  return (p_aes_set && p_sha384 && p_aes_enc) ? 0 : -1;
}
/* NewUniformSamplerWithSeed (uniform.go:38-54) */
static int dom_init(of_dom* D, const unsigned char* seed, size_t n) {
  unsigned char r[48];
  if (crypto_load()) return -1;
  p_sha384(seed, n, r);
  memcpy(D->iv, r + 32, 16);
  return p_aes_set(r, 256, D->aes) == 0 ? 0 : -1;
}
typedef struct {
  const of_dom* D;
  unsigned char ctr0[16]; /* IV + instance * 2^24 */
  uint64_t pos;
} of_uni;
static void ctr_add(unsigned char c[16], const unsigned char a[16], uint64_t hi, uint64_t lo) {
  /* c = a + (hi * 2^64 + lo) as 128-bit big-endian */
  unsigned carry = 0;
  for (int i = 15; i >= 0; --i) {
    uint64_t add = i >= 8 ? (lo >> (8 * (15 - i))) & 255 : (hi >> (8 * (7 - i))) & 255;
    unsigned s = a[i] + (unsigned)add + carry;
    c[i] = (unsigned char)s;
    carry = s >> 8;
  }
}
static void uni_init(of_uni* U, const of_dom* D, uint64_t inst) {
  U->D = D;
  ctr_add(U->ctr0, D->iv, inst >> 40, inst << 24);
  U->pos = 0;
}
static uint64_t ks_word(const of_uni* U, uint64_t w) { /* word w of the plain keystream */
  unsigned char ctr[16], out[16];
  ctr_add(ctr, U->ctr0, 0, w >> 1);
  p_aes_enc(ctr, out, U->D->aes);
  uint64_t x = 0;
  for (int i = 7; i >= 0; --i) x = (x << 8) | out[8 * (w & 1) + i];
  return x;
}
/* Sample() (uniform.go:64-82): buffer chunk c = KS_0 ^ ... ^ KS_c */
static uint64_t uni_sample(of_uni* U) {
  uint64_t p = U->pos++, c = p >> 10, o = p & 1023, x = 0;
  for (uint64_t i = 0; i <= c; ++i) x ^= ks_word(U, (i << 10) + o);
  return x;
}
static double uni_float(of_uni* U) { /* SampleFloat (uniform.go:95-100) */
  uint64_t r = uni_sample(U) % (1ull << 52);
  double rf;
  uint64_t bits = r | ((uint64_t)(1023 + 52) << 52);
  memcpy(&rf, &bits, 8);
  return (rf / (double)(1ull << 52)) - 1;
}

/* computeCDT (gaussian_twin_cdt.go:13-37); Go's amd64 float64->uint64 for x >= 2^63 */
static uint64_t go_u64(double x) {
  if (x < 9223372036854775808.0) return (uint64_t)(int64_t)x;
  double y = x - 9223372036854775808.0;
  int64_t z = y < 9223372036854775808.0 ? (int64_t)y : INT64_MIN;
  return (uint64_t)z | 0x8000000000000000ull;
}
static int cdt_table(double center, double sigma, uint64_t* t) {
  int64_t hi = (int64_t)ceil(9 * sigma), lo = -hi;
  double cdf = 0, norm = sqrt(2 * M_PI) * sigma;
  int i = 0;
  for (int64_t x = lo; x <= hi; ++x, ++i) {
    double xf = (double)x;
    double rho = exp(-(xf - center) * (xf - center) / (2 * sigma * sigma)) / norm;
    cdf += rho;
    t[i] = cdf > 1 ? UINT64_MAX : go_u64(round(cdf * 18446744073709551616.0));
  }
  return i;
}
static int64_t bsearch_go(const uint64_t* x, int n, uint64_t target, int* found) { /* slices.BinarySearch */
  int i = 0, j = n;
  while (i < j) {
    int h = (int)((unsigned)(i + j) >> 1);
    if (x[h] < target) i = h + 1; else j = h;
  }
  *found = i < n && x[i] == target;
  return i;
}
typedef struct {
  double sigma;
  int size;
  int64_t tail_lo;
  uint64_t* tables; /* [128][size] */
} of_cdt;
static void cdt_init(of_cdt* C, double sigma) {
  C->sigma = sigma;
  C->tail_lo = -(int64_t)ceil(9 * sigma);
  C->size = (int)(-2 * C->tail_lo + 1);
  C->tables = (uint64_t*)malloc(8 * (size_t)C->size * 128);
  for (int i = 0; i < 128; ++i) cdt_table((double)i / 128, sigma, C->tables + (size_t)i * C->size);
}
/* TwinCDTGaussianSampler.Sample (gaussian_twin_cdt.go:77-112) */
static int64_t cdt_sample(const of_cdt* C, of_uni* U, double center) {
  double cFloor = floor(center), cFrac = center - cFloor;
  int64_t c0 = (int64_t)floor(128 * cFrac) % 128, c1 = (int64_t)ceil(128 * cFrac) % 128;
  uint64_t u = uni_sample(U);
  int f;
  int64_t v0 = bsearch_go(C->tables + c0 * C->size, C->size, u, &f);
  if (f) v0 -= 1;
  int64_t v1 = bsearch_go(C->tables + c1 * C->size, C->size, u, &f);
  if (f) v1 -= 1;
  if (v0 == v1) return v0 + (int64_t)cFloor + C->tail_lo;
  double cdf = 0, norm = sqrt(2 * M_PI) * C->sigma;
  for (int64_t x = C->tail_lo; x <= v0; x++) {
    double xf = (double)x;
    cdf += exp(-(xf - cFrac) * (xf - cFrac) / (2 * C->sigma * C->sigma)) / norm;
  }
  double p = (double)u / 18446744073709551616.0;
  if (p < cdf) return v0 + C->tail_lo + (int64_t)cFloor;
  return v1 + C->tail_lo + (int64_t)cFloor;
}
/* ziggurat tables (gaussian_rounded.go:22-52) and normFloat (:77-116) */
static uint64_t zkn[128];
static double zwn[128], zfn[128];
static const double RN = 3.442619855899;
static double znormal(double x) { return exp(-0.5 * x * x); }
static void zig_init(void) {
  double v = RN * znormal(RN) + sqrt(M_PI / 2) * erfc(RN / sqrt(2));
  double xn[128] = {0};
  xn[127] = RN;
  for (int i = 126; i >= 1; i--) xn[i] = sqrt(-2 * log(v / xn[i + 1] + znormal(xn[i + 1])));
  const double scale = (double)(1ull << 52);
  for (int i = 1; i < 128; i++) {
    zkn[i] = go_u64((xn[i - 1] / xn[i]) * scale);
    zwn[i] = xn[i] / scale;
    zfn[i] = znormal(xn[i]);
  }
  zkn[0] = go_u64((RN * znormal(RN) / v) * scale);
  zwn[0] = (v / znormal(RN)) / scale;
  zfn[0] = 0;
}
static double norm_float(of_uni* U) {
  for (;;) {
    uint64_t r = uni_sample(U);
    uint64_t b = r >> 63, i = r % (1 << 7), j = (r >> 7) % (1ull << 52);
    double x = (double)(int64_t)((j ^ -b) + b) * zwn[i];
    if (j < zkn[i]) return x;
    if (i == 0) {
      double u, v;
      for (;;) {
        u = -log(uni_float(U)) * (1.0 / RN);
        v = -log(uni_float(U));
        if (v + v >= u * u) break;
      }
      u += RN;
      return b == 1 ? -u : u;
    }
    double f0 = zfn[i - 1], f1 = zfn[i];
    if (uni_float(U) * (f0 - f1) < exp(-0.5 * x * x) - f1) return x;
  }
}
/* COSACSampler.Sample (gaussian_cosac.go:22-57) */
static int64_t cosac_sample(of_uni* base, of_uni* rnd, double center, double stdDev) {
  double cInt = round(center), cFrac = cInt - center;
  double r = uni_float(base);
  if (r < exp(-(cFrac * cFrac) / (2 * stdDev * stdDev)) / (sqrt(2 * M_PI) * stdDev)) return (int64_t)cInt;
  for (;;) {
    double y = stdDev * norm_float(rnd);
    uint64_t b = uni_sample(base) & 1;
    double yRound;
    int cmp;
    if (b == 0) {
      yRound = round(y) - 1;
      cmp = yRound <= 0.5;
    } else {
      yRound = round(y) + 1;
      cmp = yRound >= -0.5;
    }
    if (cmp) {
      double rr = uni_float(base);
      if (rr < exp(-((yRound + cFrac) * (yRound + cFrac) - y * y) / (2 * stdDev * stdDev)))
        return (int64_t)yRound + (int64_t)cInt;
    }
  }
}
/* Uint.SetRandom (element.go:299-343) from a sampler instance's bytes */
static void set_random(const of_field* F, of_uni* U, uint64_t* z) {
  int L = F->L, bitlen = 0;
  uint64_t qm1[MAXL];
  memcpy(qm1, F->q, 8 * L);
  for (int l = 0; l < L; ++l) if (qm1[l]--) break;
  for (int l = L - 1; l >= 0; --l) if (qm1[l]) { bitlen = 64 * l + 64 - __builtin_clzll(qm1[l]); break; }
  int k = (bitlen + 7) / 8, b = bitlen % 8 ? bitlen % 8 : 8;
  unsigned char bytes[8 * MAXL];
  uint64_t word = 0;
  int left = 0;
  for (;;) {
    memset(bytes, 0, sizeof(bytes));
    for (int j = 0; j < k; ++j) {
      if (!left) { word = uni_sample(U); left = 8; }
      bytes[j] = (unsigned char)word;
      word >>= 8;
      --left;
    }
    bytes[k - 1] &= (unsigned char)((1 << b) - 1);
    for (int l = 0; l < L; ++l) {
      z[l] = 0;
      for (int i = 7; i >= 0; --i) z[l] = (z[l] << 8) | bytes[8 * l + i];
    }
    if (!geq(z, F->q, L)) return;
  }
}

/* The randomness of `batch` commits (layouts: rg_jindo_sample_dev).  sd: ecd, ecd_blind, mask,
 * mask_blind, mlwe, mask_mlwe; delta: Encoder.deltaInv[exp]; seeds: 6 x 32 bytes in
 * rg_jindo_seeds order. */
int of_jindo_sample(const of_jindo* J, const double* sd, const double* delta, const unsigned char* seeds,
                    uint64_t first, long batch, const uint64_t* v, long nv, uint64_t* o_last, uint64_t* o_mask,
                    int64_t* o_en, int64_t* o_mn) {
  const of_jindo_params* P = &J->P;
  const int L = J->F.L, d = P->d, sl = P->slots, cs = P->cols * P->slots, nm = P->in_msis + P->mlwe;
  of_dom dom[6];
  for (int i = 0; i < 6; ++i)
    if (dom_init(&dom[i], seeds + 32 * i, 32)) return -1;
  if (!zkn[1] && !zkn[2]) zig_init();
  of_cdt ce, cm;
  cdt_init(&ce, sd[0]);
  cdt_init(&cm, sd[4]);
  uint64_t* digits = (uint64_t*)malloc(8 * (size_t)d);
  double* fp = (double*)malloc(8 * (size_t)d);
  uint64_t* first_row = (uint64_t*)calloc((size_t)cs * L, 8);
  uint64_t zero[MAXL] = {0};
  const uint64_t per = (uint64_t)cs + (uint64_t)P->rows * sl;
  for (long b = 0; b < batch; ++b) {
    const uint64_t gb = first + (uint64_t)b;
    const uint64_t* vb = v + (size_t)b * nv * L;
    uint64_t* last = o_last + (size_t)b * cs * L;
    uint64_t* mask = o_mask + (size_t)b * P->rows * sl * L;
    /* MustSetRandom draws: lastRow[0 .. cs-2] (last entry 0), mask rows x slots */
    for (uint64_t i = 0; i < per; ++i) {
      uint64_t* dst = i < (uint64_t)cs ? last + i * L : mask + (i - cs) * L;
      if (i == (uint64_t)cs - 1) { memset(dst, 0, 8 * L); continue; }
      of_uni U;
      uni_init(&U, &dom[5], gb * per + i);
      set_random(&J->F, &U, dst);
    }
    memcpy(first_row, vb, 8 * L); /* genFirstLastRow (prover.go:74-83) */
    for (int i = 1; i < cs; ++i)
      f_sub(&J->F, first_row + (size_t)i * L, i < nv ? vb + (size_t)i * L : zero, last + (size_t)(i - 1) * L, L);
    for (int col = 0; col <= P->cols; ++col) {
      for (int row = 0; row < P->rows; ++row) {
        int64_t* en = o_en + (((size_t)b * (P->cols + 1) + col) * P->rows + row) * d;
        const uint64_t* src;
        int n;
        double s;
        if (col == P->cols) { /* prover.go:93-115 */
          if (row >= 1 && row < P->rows - 1 && (long)row * cs > nv) { memset(en, 0, 8 * (size_t)d); continue; }
          src = mask + (size_t)row * sl * L;
          n = sl;
          s = row == 0 ? sd[3] : sd[2];
        } else { /* prover.go:116-128 */
          long s0 = (long)row * cs + (long)col * sl, e0 = s0 + sl;
          if (row == 0) { src = first_row + (size_t)col * sl * L; n = sl; s = sd[1]; }
          else if (row == P->rows - 1) { src = last + (size_t)col * sl * L; n = sl; s = sd[0]; }
          else {
            if (s0 > nv) { memset(en, 0, 8 * (size_t)d); continue; }
            src = vb + (size_t)s0 * L;
            n = (int)((e0 < nv ? e0 : nv) - s0);
            s = sd[0];
          }
        }
        base_encode(J, digits, src, n);
        /* encoder.go:153-165, literally */
        for (int k = 0; k < d; ++k) fp[k] = 0;
        for (int i = 0; i < P->exp; i++) {
          if (delta[i] == 0) continue;
          int dd = d - (i + 1) * sl;
          for (int j = 0, jj = dd; jj < d; j++, jj++) fp[jj] += delta[i] * (double)digits[j];
          for (int j = d - dd, jj = 0; j < d; j++, jj++) fp[jj] -= delta[i] * (double)digits[j];
        }
        const uint64_t gpoly = (gb * (P->cols + 1) + (uint64_t)col) * P->rows + (uint64_t)row;
        if (s == sd[0]) { /* twinCDT: the encode's instance, one word per sample */
          of_uni U;
          uni_init(&U, &dom[0], gpoly);
          for (int k = 0; k < d; ++k) en[k] = cdt_sample(&ce, &U, -fp[k]);
        } else { /* cosac: an instance pair per group of G consecutive samples, drawn in order */
          const int G = d < 8 ? d : 8;  /* the library's partition (jindo.hip kCosGroup) */
          for (int g = 0; g < d / G; ++g) {
            of_uni B, R;
            uni_init(&B, &dom[1], gpoly * (uint64_t)(d / G) + (uint64_t)g);
            uni_init(&R, &dom[2], gpoly * (uint64_t)(d / G) + (uint64_t)g);
            for (int k = g * G; k < (g + 1) * G; ++k) en[k] = cosac_sample(&B, &R, -fp[k], s);
          }
        }
      }
      for (int j = 0; j < nm; ++j) { /* prover.go:130-139 */
        int64_t* mn = o_mn + (((size_t)b * (P->cols + 1) + col) * nm + j) * d;
        const uint64_t gpoly = (gb * (P->cols + 1) + (uint64_t)col) * nm + (uint64_t)j;
        if (col == P->cols) {
          for (int k = 0; k < d; ++k) {
            of_uni U;
            uni_init(&U, &dom[4], gpoly * d + k);
            mn[k] = (int64_t)round(0 + norm_float(&U) * sd[5]);
          }
        } else {
          of_uni U;
          uni_init(&U, &dom[3], gpoly);
          for (int k = 0; k < d; ++k) mn[k] = cdt_sample(&cm, &U, 0);
        }
      }
    }
  }
  free(ce.tables);
  free(cm.tables);
  free(digits);
  free(fp);
  free(first_row);
  return 0;
}

/* n draws of one sampler (distribution tests): kind 0 TwinCDTGaussianSampler(sigma).Sample(center),
 * 1 COSACSampler.Sample(center, sigma), 2 RoundedGaussianSampler.Sample(center, sigma).  Draw k
 * reads instance k / per_inst of seeds[0..32) (and, for COSAC's rounded sampler, of
 * seeds[32..64)), whose stream continues from draw to draw inside an instance. */
int of_sampler_draws(int kind, const unsigned char* seeds, double sigma, double center, long n, long per_inst,
                     int64_t* out) {
  of_dom d0, d1;
  if (dom_init(&d0, seeds, 32) || dom_init(&d1, seeds + 32, 32)) return -1;
  if (!zkn[1] && !zkn[2]) zig_init();
  of_cdt C;
  C.tables = NULL;
  if (kind == 0) cdt_init(&C, sigma);
  of_uni B, R;
  for (long k = 0; k < n; ++k) {
    if (k % per_inst == 0) {
      uni_init(&B, &d0, (uint64_t)(k / per_inst));
      uni_init(&R, &d1, (uint64_t)(k / per_inst));
    }
    if (kind == 0) out[k] = cdt_sample(&C, &B, center);
    else if (kind == 1) out[k] = cosac_sample(&B, &R, center, sigma);
    else out[k] = (int64_t)round(center + norm_float(&B) * sigma);
  }
  free(C.tables);
  return 0;
}

/* UniformSampler.Sample() words [first, first + n) of instance `inst` of the seed's sampler */
int of_uniform_words(const unsigned char* seed, size_t seed_len, uint64_t inst, uint64_t first, long n, uint64_t* out) {
  of_dom D;
  if (dom_init(&D, seed, seed_len)) return -1;
  of_uni U;
  uni_init(&U, &D, inst);
  U.pos = first;
  for (long i = 0; i < n; ++i) out[i] = uni_sample(&U);
  return 0;
}
