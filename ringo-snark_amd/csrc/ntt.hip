// ntt.hip -- host side of the bigpoly transformers: table construction (the reference's
// generator search and layouts, math/bigpoly/ntt.go:26-95,153-203), pass planning, and the
// C ABI (include/ringo.h).  Kernels: ntt_kernels.hpp, instantiated per limb count in
// ntt_l1.hip / ntt_l2.hip / ntt_l4.hip / ntt_lwide.hip.
#include <algorithm>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "common.hpp"
#include "field.hpp"
#include "host_field.hpp"

#include "ntt_plan.hpp"

namespace rg {
// must match ntt_kernels.hpp (RadixOf + 8, kMinTiledP)
static int pmax_of(int L) { return (L <= 2 ? 4 : 3) + 8; }
static const int kMinTiledP = 6;
static bool supported_L(int L) { return L == 1 || L == 2 || L == 4 || L == 7 || L == 14; }
}  // namespace rg

struct rg_ntt {
  rg_field f;
  int N, logN, negacyclic;
  bool shoup, tiled;
  bool halving = true;  // wide fields: rank_inv == N^-1 (finalize)
  std::vector<uint64_t> h_tw, h_twinv, h_ninv;  // Montgomery reps, [N][L]
  rg::DevBuf d_tw, d_twinv;                     // kernel format
  std::vector<rg::PassDesc> passes;             // forward order
  uint64_t nsc[16], nsc_sh, w1n[16], w1n_sh;
  std::unique_ptr<rg::Aux> aux;  // L = 4: helper stream of ntt256_run's split (ntt_l4_fast.hip)
  int device = 0;                // the tables and the helper stream live on this device
};

namespace rg {

// 2-adicity check shared by both constructors (ntt.go:27-37, 154-164)
static rg_status check_rank(const rg_field* f, int rank) {
  if (rank <= 0 || (rank & (rank - 1))) return RG_ERR_NOT_POW2;
  int logn = 0;
  while ((1 << logn) < rank) ++logn;
  uint64_t pm1[16];
  memcpy(pm1, f->q, 8 * f->L);
  pm1[0] -= 1;  // q odd
  int tz = 0;
  for (int i = 0; i < f->L; ++i) {
    if (pm1[i] == 0) {
      tz += 64;
      continue;
    }
    tz += __builtin_ctzll(pm1[i]);
    break;
  }
  if (tz < logn + 1) return RG_ERR_UNSUPPORTED;  // 2N | q-1
  return RG_OK;
}

// reference generator search: first x = 2, 3, ... with (x^((q-1)/2^lo))^(2^(lo-1)) != 1
static bool find_root(const HostField& H, int log_order, uint64_t* g) {
  const int L = H.L;
  uint64_t e[16];
  memcpy(e, H.q, 8 * L);
  e[0] -= 1;
  for (int s = log_order; s > 0;) {
    int k = s > 63 ? 63 : s;
    for (int i = 0; i < L; ++i) e[i] = (e[i] >> k) | (i + 1 < L ? e[i + 1] << (64 - k) : 0);
    s -= k;
  }
  const uint64_t half[1] = {(uint64_t)1 << (log_order - 1)};
  for (uint64_t xv = 2; xv < (1u << 24); ++xv) {
    uint64_t x[16], gp[16];
    H.from_u64(x, xv);
    H.pow(g, x, e, L);
    H.pow(gp, g, half, 1);
    if (!H.eq(gp, H.one)) return true;
  }
  return false;
}

static void bitrev_perm(std::vector<uint64_t>& v, int n, int L) {  // vec.go:123-137
  for (int i = 1, j = 0; i < n; ++i) {
    int bit = n >> 1;
    for (; j >= bit; bit >>= 1) j -= bit;
    j += bit;
    if (i < j)
      for (int l = 0; l < L; ++l) std::swap(v[(size_t)i * L + l], v[(size_t)j * L + l]);
  }
}

static rg_status build_tables(rg_ntt* t) {
  const int N = t->N, L = t->f.L;
  HostField H(&t->f);
  t->h_tw.assign((size_t)N * L, 0);
  t->h_twinv.assign((size_t)N * L, 0);
  t->h_ninv.assign(L, 0);
  uint64_t g[16], gi[16];
  if (t->negacyclic) {  // ntt.go:167-192: tw[k] = psi^brv(k)
    if (!find_root(H, t->logN + 1, g)) return RG_ERR_UNSUPPORTED;
    H.inverse(gi, g);
    memcpy(&t->h_tw[0], H.one, 8 * L);
    memcpy(&t->h_twinv[0], H.one, 8 * L);
    for (int i = 1; i < N; ++i) {
      H.mul(&t->h_tw[(size_t)i * L], &t->h_tw[(size_t)(i - 1) * L], g);
      H.mul(&t->h_twinv[(size_t)i * L], &t->h_twinv[(size_t)(i - 1) * L], gi);
    }
    bitrev_perm(t->h_tw, N, L);
    bitrev_perm(t->h_twinv, N, L);
  } else if (N >= 2) {  // ntt.go:40-84: tw[m+i] = brv_{N/2}(w^j)[i]
    if (!find_root(H, t->logN, g)) return RG_ERR_UNSUPPORTED;
    H.inverse(gi, g);
    const int h = N / 2;
    std::vector<uint64_t> ref((size_t)h * L), refi((size_t)h * L);
    memcpy(&ref[0], H.one, 8 * L);
    memcpy(&refi[0], H.one, 8 * L);
    for (int i = 1; i < h; ++i) {
      H.mul(&ref[(size_t)i * L], &ref[(size_t)(i - 1) * L], g);
      H.mul(&refi[(size_t)i * L], &refi[(size_t)(i - 1) * L], gi);
    }
    bitrev_perm(ref, h, L);
    bitrev_perm(refi, h, L);
    for (int m = 1; m <= N / 2; m <<= 1)
      for (int i = 0; i < m; ++i) {
        memcpy(&t->h_tw[(size_t)(m + i) * L], &ref[(size_t)i * L], 8 * L);
        memcpy(&t->h_twinv[(size_t)(m + i) * L], &refi[(size_t)i * L], 8 * L);
      }
  }
  uint64_t n[16];
  H.from_u64(n, (uint64_t)N);
  H.inverse(&t->h_ninv[0], n);  // rankInv (ntt.go:86-87, 194-195)
  return RG_OK;
}

static rg_status finalize(rg_ntt* t) {
  const int N = t->N, L = t->f.L;
  RG_HIP(hipGetDevice(&t->device));
  HostField H(&t->f);
  // pass plan: tiled passes of P in [kMinTiledP, pmax] for L <= 4; per-stage otherwise
  const int pm = pmax_of(L);
  t->passes.clear();
  t->tiled = (L <= 4) && t->logN >= kMinTiledP && t->logN <= 2 * pm;
  if (t->tiled) {
    if (t->logN <= pm) {
      t->passes.push_back({0, t->logN});
    } else {
      int pa = t->logN / 2;
      if (pa < kMinTiledP) pa = kMinTiledP;
      t->passes.push_back({0, pa});
      t->passes.push_back({pa, t->logN - pa});
    }
  }
  uint64_t w1n[16];
  const uint64_t* twi1 = N >= 2 ? &t->h_twinv[(size_t)1 * L] : H.one;
  H.mul(w1n, twi1, &t->h_ninv[0]);  // twInv[1] * N^-1 for the fused last inverse stage
  t->shoup = (L == 1) && (t->f.q[0] >> 63) == 0;
  if (t->shoup) {
    // tables hold the plain twiddle (Montgomery rep * R^-1) and its Shoup quotient:
    // shoup(v, w) == v * w mod q == mont(v, w*R).
    const uint64_t q = t->f.q[0];
    std::vector<uint64_t> a((size_t)2 * N), b((size_t)2 * N);
    for (int i = 0; i < N; ++i) {
      uint64_t w, wi;
      H.from_mont(&w, &t->h_tw[i]);
      H.from_mont(&wi, &t->h_twinv[i]);
      a[2 * i] = w;
      a[2 * i + 1] = h_shoup(w, q);
      b[2 * i] = wi;
      b[2 * i + 1] = h_shoup(wi, q);
    }
    if (t->logN == 16) {  // lane-ordered ROW last-round copy for ntt16_pass (ntt64.hpp)
      auto add_row_copy = [&](std::vector<uint64_t>& v) {
        const size_t base = v.size();
        v.resize(base + (size_t)2 * 256 * 192);
        for (int r = 0; r < 256; ++r)
          for (int tt = 0; tt < 32; ++tt) {
            for (int g = 0; g < 2; ++g) {
              const size_t src = (size_t)(1 << 14) + 64 * r + 2 * tt + g, dst = (size_t)r * 192 + 32 * g + tt;
              v[base + 2 * dst] = v[2 * src];
              v[base + 2 * dst + 1] = v[2 * src + 1];
            }
            for (int j = 0; j < 4; ++j) {
              const size_t src = (size_t)(1 << 15) + 128 * r + 4 * tt + j, dst = (size_t)r * 192 + 64 + 32 * j + tt;
              v[base + 2 * dst] = v[2 * src];
              v[base + 2 * dst + 1] = v[2 * src + 1];
            }
          }
      };
      add_row_copy(a);
      add_row_copy(b);
    }
    RG_TRY(t->d_tw.upload(a.data(), a.size() * 8));
    RG_TRY(t->d_twinv.upload(b.data(), b.size() * 8));
    uint64_t nv, wv;
    H.from_mont(&nv, &t->h_ninv[0]);
    H.from_mont(&wv, w1n);
    t->nsc[0] = nv;
    t->nsc_sh = h_shoup(nv, q);
    t->w1n[0] = wv;
    t->w1n_sh = h_shoup(wv, q);
  } else if (L == 7 || L == 14) {
    // wide fields: the inverse table is followed by twInv[i] / 2 (ntt_wide.hpp's inverse halves
    // every stage instead of scaling by N^-1 at the end); the per-stage kernels read the first half
    RG_TRY(t->d_tw.upload(t->h_tw.data(), t->h_tw.size() * 8));
    std::vector<uint64_t> b(2 * t->h_twinv.size());
    const size_t half = t->h_twinv.size();
    memcpy(b.data(), t->h_twinv.data(), half * 8);
    for (int i = 0; i < N; ++i) {
      const uint64_t* x = &t->h_twinv[(size_t)i * L];
      uint64_t* z = &b[half + (size_t)i * L];
      uint64_t c = 0;
      if (x[0] & 1) c = HostField::add_n(z, x, t->f.q, L);
      else memcpy(z, x, 8 * L);
      for (int l = 0; l < L; ++l) z[l] = (z[l] >> 1) | ((l + 1 < L ? z[l + 1] : c) << 63);
    }
    RG_TRY(t->d_twinv.upload(b.data(), b.size() * 8));
    memcpy(t->nsc, &t->h_ninv[0], 8 * L);
    memcpy(t->w1n, w1n, 8 * L);
    t->nsc_sh = t->w1n_sh = 0;
    // log N halvings give exactly N^-1: a table-built plan whose rank_inv is anything else keeps
    // the per-stage inverse, which multiplies by the caller's rank_inv (ntt.go:242-243)
    uint64_t n[16], ninv[16];
    H.from_u64(n, (uint64_t)N);
    H.inverse(ninv, n);
    t->halving = H.eq(ninv, &t->h_ninv[0]);
  } else {
    RG_TRY(t->d_tw.upload(t->h_tw.data(), t->h_tw.size() * 8));
    RG_TRY(t->d_twinv.upload(t->h_twinv.data(), t->h_twinv.size() * 8));
    memcpy(t->nsc, &t->h_ninv[0], 8 * L);
    memcpy(t->w1n, w1n, 8 * L);
    t->nsc_sh = t->w1n_sh = 0;
  }
  if (L == 4 && (t->logN == 15 || t->logN == 16)) {
    t->aux.reset(new Aux());
    RG_HIP(hipStreamCreateWithFlags(&t->aux->s, hipStreamNonBlocking));
    RG_HIP(hipEventCreateWithFlags(&t->aux->fork, hipEventDisableTiming));
    RG_HIP(hipEventCreateWithFlags(&t->aux->join, hipEventDisableTiming));
  }
  return RG_OK;
}

static rg_status run(const rg_ntt* t, uint64_t* out, const uint64_t* in, size_t batch, bool inv, hipStream_t st) {
  if (batch == 0) return RG_OK;
  int cur = -1;
  RG_HIP(hipGetDevice(&cur));
  if (cur != t->device) {
    set_last_error("rg_ntt plan used on device " + std::to_string(cur) + ", created on " + std::to_string(t->device));
    return RG_ERR_INVALID;
  }
  NttLaunch p;
  p.in = in;
  p.out = out;
  p.tw = inv ? t->d_twinv.as<uint64_t>() : t->d_tw.as<uint64_t>();
  p.q = t->f.q;
  p.qinv = t->f.qinv;
  p.nsc = t->nsc;
  p.nsc_sh = t->nsc_sh;
  p.w1n = t->w1n;
  p.w1n_sh = t->w1n_sh;
  p.logN = t->logN;
  p.shoup = t->shoup;
  p.inv = inv;
  p.tiled = t->tiled;
  p.halving = t->halving;
  p.passes = t->passes.data();
  p.npasses = (int)t->passes.size();
  p.batch = batch;
  p.aux = t->aux.get();
  switch (t->f.L) {
    case 1: {
      bool done = false;
      RG_TRY(ntt64_run(p, st, &done));
      return done ? RG_OK : ntt_run_L1(p, st);
    }
    case 2: return ntt_run_L2(p, st);
    case 4: {
      bool done = false;
      RG_TRY(ntt256_run(p, st, &done));
      return done ? RG_OK : ntt_run_L4(p, st);
    }
    case 7: return ntt_run_L7(p, st);
    case 14: return ntt_run_L14(p, st);
    default: return RG_ERR_UNSUPPORTED;
  }
}

static rg_ntt* new_plan(const rg_field* f, int rank, int negacyclic) {
  rg_ntt* t = new rg_ntt();
  t->f = *f;
  t->N = rank;
  t->logN = 0;
  while ((1 << t->logN) < rank) ++t->logN;
  t->negacyclic = negacyclic ? 1 : 0;
  return t;
}

const rg_field* ntt_field(const rg_ntt* t) { return &t->f; }
bool ntt_negacyclic(const rg_ntt* t) { return t->negacyclic != 0; }

}  // namespace rg

using namespace rg;

extern "C" {

rg_status rg_ntt_create(const rg_field* f, int rank, int negacyclic, rg_ntt** out) {
  if (!f || !out) return RG_ERR_INVALID;
  *out = nullptr;
  RG_TRY(check_rank(f, rank));
  if (!supported_L(f->L)) return RG_ERR_UNSUPPORTED;
  rg_ntt* t = new_plan(f, rank, negacyclic);
  rg_status s = build_tables(t);
  if (s == RG_OK) s = finalize(t);
  if (s != RG_OK) {
    delete t;
    return s;
  }
  *out = t;
  return RG_OK;
}

rg_status rg_ntt_create_from_tables(const rg_field* f, int rank, int negacyclic, const uint64_t* tw,
                                    const uint64_t* tw_inv, const uint64_t* rank_inv, rg_ntt** out) {
  if (!f || !out || !tw || !tw_inv || !rank_inv) return RG_ERR_INVALID;
  *out = nullptr;
  RG_TRY(check_rank(f, rank));
  if (!supported_L(f->L)) return RG_ERR_UNSUPPORTED;
  const int L = f->L;
  rg_ntt* t = new_plan(f, rank, negacyclic);
  t->h_tw.assign(tw, tw + (size_t)rank * L);
  t->h_twinv.assign(tw_inv, tw_inv + (size_t)rank * L);
  t->h_ninv.assign(rank_inv, rank_inv + L);
  HostField H(&t->f);
  bool ok = !HostField::geq(rank_inv, f->q, L);
  for (size_t i = 0; i < (size_t)rank && ok; ++i)
    ok = !HostField::geq(&t->h_tw[i * L], f->q, L) && !HostField::geq(&t->h_twinv[i * L], f->q, L);
  if (ok && negacyclic) ok = H.eq(&t->h_tw[0], H.one) && H.eq(&t->h_twinv[0], H.one);
  rg_status s = ok ? finalize(t) : RG_ERR_INVALID;
  if (s != RG_OK) {
    delete t;
    return s;
  }
  *out = t;
  return RG_OK;
}

void rg_ntt_destroy(rg_ntt* t) { delete t; }
int rg_ntt_rank(const rg_ntt* t) { return t ? t->N : 0; }


rg_status rg_ntt_tables(const rg_ntt* t, uint64_t* tw, uint64_t* tw_inv, uint64_t* rank_inv) {
  if (!t) return RG_ERR_INVALID;
  if (tw) memcpy(tw, t->h_tw.data(), t->h_tw.size() * 8);
  if (tw_inv) memcpy(tw_inv, t->h_twinv.data(), t->h_twinv.size() * 8);
  if (rank_inv) memcpy(rank_inv, t->h_ninv.data(), t->h_ninv.size() * 8);
  return RG_OK;
}

static rg_status dev_call(const rg_ntt* t, uint64_t* d_out, const uint64_t* d_in, size_t batch, void* stream,
                          bool inv) {
  if (!t || (batch && (!d_out || !d_in))) return RG_ERR_INVALID;
  if (batch == 0) return RG_OK;
  if (t->N == 1) {  // rank 1: identity (1^-1 = 1)
    if (d_out != d_in)
      RG_HIP(hipMemcpyAsync(d_out, d_in, batch * t->f.L * 8, hipMemcpyDeviceToDevice, as_stream(stream)));
    return RG_OK;
  }
  return run(t, d_out, d_in, batch, inv, as_stream(stream));
}

rg_status rg_ntt_fwd_dev(const rg_ntt* t, uint64_t* d_out, const uint64_t* d_in, size_t batch, void* stream) {
  return dev_call(t, d_out, d_in, batch, stream, false);
}
rg_status rg_ntt_inv_dev(const rg_ntt* t, uint64_t* d_out, const uint64_t* d_in, size_t batch, void* stream) {
  return dev_call(t, d_out, d_in, batch, stream, true);
}

static rg_status host_call(const rg_ntt* t, uint64_t* out, const uint64_t* in, size_t batch, bool inv) {
  if (!t || (batch && (!out || !in))) return RG_ERR_INVALID;
  if (batch == 0) return RG_OK;
  const size_t bytes = batch * (size_t)t->N * t->f.L * 8;
  DevBuf buf;
  RG_TRY(buf.alloc(bytes));
  RG_HIP(hipMemcpy(buf.p, in, bytes, hipMemcpyHostToDevice));
  RG_TRY(dev_call(t, buf.as<uint64_t>(), buf.as<uint64_t>(), batch, nullptr, inv));
  RG_HIP(hipMemcpy(out, buf.p, bytes, hipMemcpyDeviceToHost));
  return RG_OK;
}

rg_status rg_ntt_fwd(const rg_ntt* t, uint64_t* out, const uint64_t* in, size_t batch) {
  return host_call(t, out, in, batch, false);
}
rg_status rg_ntt_inv(const rg_ntt* t, uint64_t* out, const uint64_t* in, size_t batch) {
  return host_call(t, out, in, batch, true);
}

}  // extern "C"
