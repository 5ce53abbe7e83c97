// buckler.hip -- the Buckler prover's per-witness device work around the bigpoly evaluators
// (SURVEY.md §8f rank 4), for gfx950:
//   * Encoder.EncodeTo / RandEncodeTo (buckler/encoder.go:32-54): the cyclic InvNTT at the
//     witness rank (the library's NTT kernels) into the first `rank` coefficients of an
//     embedRank polynomial, zeros above; RandEncode then adds r (X^rank - 1) for the injected
//     MustSetRandom draw r: coeff[rank] = r, coeff[0] -= r.  A batch of witnesses runs one
//     batched InvNTT into scratch and one embedding pass (strided rows cannot be NTT outputs).
//   * Prover.evalCircuit (buckler/prover.go:355-379): pOut = sum_c batchConst * sum_t coeff_t *
//     pw_t * prod w, pointwise in the NTT domain.  The reference runs it polynomial by polynomial
//     (a term poly, an eval poly, one MulTo per factor: each factor costs a full read + write of
//     two polys).  Here it is ONE pass over the coefficients: a lane per coefficient walks the
//     circuit program (uniform across lanes: scalar loads) with term / eval / result in
//     registers, so HBM sees each referenced witness coefficient once per reference (repeats of
//     one witness in a term hit L1/L2) and the result once.  Every product is the Montgomery
//     f_mul of field.hpp; values stay canonical, so the limbs equal the reference's.
#include <cstring>
#include <vector>

#include "common.hpp"
#include "field.hpp"
#include "ntt_plan.hpp"

struct rg_circuit {
  rg_field f;
  int nc = 0;        // constraints
  long long nt = 0;  // terms
  long long max_w = -1, max_pw = -1;
  rg::DevBuf prog;   // term_off [nc+1] u32 | pw [nt] i32 | wit_off [nt+1] u32 | wit [nwit] u32 | coeffs [nt][L] u64
  size_t off_pw = 0, off_wo = 0, off_wi = 0, off_cf = 0;  // byte offsets into prog
};

namespace rg {

template <int L>
__device__ __forceinline__ void cpy(uint64_t* d, const uint64_t* s) {
#pragma unroll
  for (int l = 0; l < L; ++l) d[l] = s[l];
}

// ---- Encoder ----------------------------------------------------------------------------------
// element (b, i) of the [batch][emb][L] output: i < rank from src (the InvNTT output; src ==
// nullptr when it was written in place), zero above, then the RandEncode fix-up (encoder.go:52-53)
template <int L>
__global__ __launch_bounds__(256) void embed_kernel(FieldParams<L> F, uint64_t* out, const uint64_t* src, long long rank,
                                                    long long emb, long long batch, const uint64_t* rnd) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= batch * emb) return;
  const long long b = gid / emb, i = gid % emb;
  uint64_t* o = out + gid * L;
  if (i < rank) {
    uint64_t x[L];
    if (src) cpy<L>(x, src + (b * rank + i) * L);
    else if (i == 0 && rnd) cpy<L>(x, o);
    if (i == 0 && rnd) f_sub<L>(x, x, rnd + b * L, F);  // Coeffs[0].Sub(Coeffs[0], Coeffs[rank])
    if (src || (i == 0 && rnd)) cpy<L>(o, x);
  } else if (i == rank && rnd) {
    cpy<L>(o, rnd + b * L);  // Coeffs[rank].MustSetRandom()
  } else {
#pragma unroll
    for (int l = 0; l < L; ++l) o[l] = 0;  // Coeffs[i].SetUint64(0)
  }
}

// ---- evalCircuit ----------------------------------------------------------------------------
template <int L>
struct CircArgs {
  FieldParams<L> F;
  const uint32_t* term_off;
  const int* pw_idx;
  const uint32_t* wit_off;
  const uint32_t* wit;
  const uint64_t* coeffs;
  const uint64_t* w;
  const uint64_t* pw;
  const uint64_t* bc;
  uint64_t* out;
  long long rank;
  int nc;
};

template <int L>
__global__ __launch_bounds__(256) void circuit_kernel(CircArgs<L> a) {
  const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= a.rank) return;
  uint64_t acc[L], bc[L];
  cpy<L>(bc, a.bc);
#pragma unroll
  for (int l = 0; l < L; ++l) acc[l] = 0;  // pOut := NewPoly(true)
  uint32_t t = a.term_off[0];
  for (int c = 0; c < a.nc; ++c) {
    uint64_t ev[L];
#pragma unroll
    for (int l = 0; l < L; ++l) ev[l] = 0;  // eval.Clear()
    const uint32_t t1 = a.term_off[c + 1];
    for (; t < t1; ++t) {
      uint64_t term[L], x[L];
      cpy<L>(term, a.coeffs + (size_t)t * L);  // term.Coeffs[j].Set(c.coeffs[i])
      const int p = a.pw_idx[t];
      if (p >= 0) {  // MulTo(term, term, pwEcdNTT[...])
        cpy<L>(x, a.pw + ((size_t)p * a.rank + j) * L);
        f_mul<L>(term, term, x, a.F);
      }
      for (uint32_t k = a.wit_off[t]; k < a.wit_off[t + 1]; ++k) {  // MulTo(term, term, wEcdNTT[...])
        cpy<L>(x, a.w + ((size_t)a.wit[k] * a.rank + j) * L);
        f_mul<L>(term, term, x, a.F);
      }
      f_add<L>(ev, ev, term, a.F);  // AddTo(eval, eval, term)
    }
    f_mul<L>(ev, ev, bc, a.F);    // ScalarMulTo(eval, eval, batchConst)
    f_add<L>(acc, acc, ev, a.F);  // AddTo(pOut, pOut, eval)
  }
  cpy<L>(a.out + j * L, acc);
}

template <int L>
static FieldParams<L> params_of(const rg_field* f) {
  FieldParams<L> F;
  memcpy(F.q, f->q, 8 * L);
  F.qinv = f->qinv;
  return F;
}

static unsigned blocks_of(long long n) { return (unsigned)((n + 255) / 256); }

template <int L>
static rg_status embed_L(const rg_field* f, uint64_t* out, const uint64_t* src, long long rank, long long emb,
                         long long batch, const uint64_t* rnd, hipStream_t st) {
  hipLaunchKernelGGL(embed_kernel<L>, dim3(blocks_of(batch * emb)), dim3(256), 0, st, params_of<L>(f), out, src, rank,
                     emb, batch, rnd);
  return check_launch("buckler encode");
}

template <int L>
static rg_status circuit_L(const rg_circuit* c, long long rank, const uint64_t* bc, const uint64_t* w,
                           const uint64_t* pw, uint64_t* out, hipStream_t st) {
  CircArgs<L> a;
  a.F = params_of<L>(&c->f);
  const char* base = c->prog.as<char>();
  a.term_off = reinterpret_cast<const uint32_t*>(base);
  a.pw_idx = reinterpret_cast<const int*>(base + c->off_pw);
  a.wit_off = reinterpret_cast<const uint32_t*>(base + c->off_wo);
  a.wit = reinterpret_cast<const uint32_t*>(base + c->off_wi);
  a.coeffs = reinterpret_cast<const uint64_t*>(base + c->off_cf);
  a.w = w;
  a.pw = pw;
  a.bc = bc;
  a.out = out;
  a.rank = rank;
  a.nc = c->nc;
  hipLaunchKernelGGL(circuit_kernel<L>, dim3(blocks_of(rank)), dim3(256), 0, st, a);
  return check_launch("buckler evalCircuit");
}

#define RG_DISPATCH_L(L_, CALL)         \
  switch (L_) {                         \
    case 1: return CALL(1);             \
    case 2: return CALL(2);             \
    case 4: return CALL(4);             \
    case 7: return CALL(7);             \
    case 14: return CALL(14);           \
    default: return RG_ERR_UNSUPPORTED; \
  }

static bool lt_q(const uint64_t* x, const rg_field* f) {
  for (int i = f->L - 1; i >= 0; --i)
    if (x[i] != f->q[i]) return x[i] < f->q[i];
  return false;
}

}  // namespace rg

using namespace rg;

extern "C" {

size_t rg_buckler_encode_scratch_bytes(const rg_ntt* t, size_t batch) {
  return (t && batch > 1) ? batch * (size_t)rg_ntt_rank(t) * ntt_field(t)->L * 8 : 0;
}

rg_status rg_buckler_encode_dev(const rg_ntt* t, size_t embed_rank, uint64_t* d_out, const uint64_t* d_v,
                                size_t batch, const uint64_t* d_rand, uint64_t* d_scratch, void* stream) {
  if (!t || ntt_negacyclic(t)) return RG_ERR_INVALID;  // newEncoder: NewCyclicTransformer (encoder.go:15-20)
  const long long rank = rg_ntt_rank(t), emb = (long long)embed_rank;
  if (emb < rank + (d_rand ? 1 : 0)) return RG_ERR_INVALID;  // RandEncode writes Coeffs[rank]
  if (batch == 0) return RG_OK;
  if (!d_out || !d_v || (batch > 1 && !d_scratch)) return RG_ERR_INVALID;
  const rg_field* f = ntt_field(t);
  hipStream_t st = as_stream(stream);
  const uint64_t* src = nullptr;
  if (batch == 1) {  // InvNTTTo(pOut.Coeffs[:rank], v[:rank]) straight into the output row
    RG_TRY(rg_ntt_inv_dev(t, d_out, d_v, 1, stream));
  } else {           // a batched InvNTT into [batch][rank] scratch, then the strided embedding
    RG_TRY(rg_ntt_inv_dev(t, d_scratch, d_v, batch, stream));
    src = d_scratch;
  }
#define RG_EMB(L) embed_L<L>(f, d_out, src, rank, emb, (long long)batch, d_rand, st)
  RG_DISPATCH_L(f->L, RG_EMB)
#undef RG_EMB
}

rg_status rg_buckler_encode(const rg_ntt* t, size_t embed_rank, uint64_t* out, const uint64_t* v,
                            const uint64_t* rand) {
  if (!t || !out || !v) return RG_ERR_INVALID;
  const int L = ntt_field(t)->L;
  const size_t rank = (size_t)rg_ntt_rank(t);
  DevBuf dv, dout, dr;
  RG_TRY(dv.upload(v, rank * L * 8));
  RG_TRY(dout.alloc(embed_rank * L * 8 + 8));
  if (rand) RG_TRY(dr.upload(rand, L * 8));
  RG_TRY(rg_buckler_encode_dev(t, embed_rank, dout.as<uint64_t>(), dv.as<uint64_t>(), 1,
                               rand ? dr.as<uint64_t>() : nullptr, nullptr, nullptr));
  RG_HIP(hipMemcpy(out, dout.p, embed_rank * L * 8, hipMemcpyDeviceToHost));
  return RG_OK;
}

rg_status rg_buckler_circuit_create(const rg_field* f, size_t n_constraints, const size_t* term_off,
                                    const uint64_t* coeffs, const long long* pw_idx, const size_t* wit_off,
                                    const uint64_t* wit_idx, rg_circuit** out) {
  if (!f || !out || !term_off || n_constraints > (1u << 30)) return RG_ERR_INVALID;
  *out = nullptr;
  if (term_off[0] != 0) return RG_ERR_INVALID;
  for (size_t c = 0; c < n_constraints; ++c)
    if (term_off[c + 1] < term_off[c]) return RG_ERR_INVALID;
  const size_t nt = term_off[n_constraints];
  if (nt && (!coeffs || !pw_idx || !wit_off)) return RG_ERR_INVALID;
  if (nt >= (1u << 31)) return RG_ERR_INVALID;
  std::vector<uint32_t> to(n_constraints + 1), wo(nt + 1), wi;
  std::vector<int> pi(nt);
  auto c = new rg_circuit();
  c->f = *f;
  c->nc = (int)n_constraints;
  c->nt = (long long)nt;
  for (size_t i = 0; i <= n_constraints; ++i) to[i] = (uint32_t)term_off[i];
  if (nt && wit_off[0] != 0) {
    delete c;
    return RG_ERR_INVALID;
  }
  for (size_t t = 0; t < nt; ++t) {
    if (!lt_q(coeffs + t * f->L, f) || pw_idx[t] >= (1LL << 31) || wit_off[t + 1] < wit_off[t] ||
        wit_off[t + 1] >= (1u << 31)) {
      delete c;
      return RG_ERR_INVALID;
    }
    pi[t] = pw_idx[t] < 0 ? -1 : (int)pw_idx[t];
    if (pw_idx[t] > c->max_pw) c->max_pw = pw_idx[t];
    wo[t] = (uint32_t)wit_off[t];
    for (size_t k = wit_off[t]; k < wit_off[t + 1]; ++k) {
      if (!wit_idx || wit_idx[k] >= (1u << 31)) {
        delete c;
        return RG_ERR_INVALID;
      }
      wi.push_back((uint32_t)wit_idx[k]);
      if ((long long)wit_idx[k] > c->max_w) c->max_w = (long long)wit_idx[k];
    }
  }
  wo[nt] = nt ? (uint32_t)wit_off[nt] : 0;
  auto al = [](size_t x) { return (x + 7) & ~size_t(7); };
  c->off_pw = al(4 * to.size());
  c->off_wo = al(c->off_pw + 4 * pi.size());
  c->off_wi = al(c->off_wo + 4 * wo.size());
  c->off_cf = al(c->off_wi + 4 * wi.size());
  const size_t bytes = c->off_cf + 8 * nt * f->L + 8;
  std::vector<char> h(bytes, 0);
  memcpy(h.data(), to.data(), 4 * to.size());
  if (nt) {
    memcpy(h.data() + c->off_pw, pi.data(), 4 * pi.size());
    memcpy(h.data() + c->off_wo, wo.data(), 4 * wo.size());
    if (!wi.empty()) memcpy(h.data() + c->off_wi, wi.data(), 4 * wi.size());
    memcpy(h.data() + c->off_cf, coeffs, 8 * nt * f->L);
  }
  rg_status s = c->prog.upload(h.data(), bytes);
  if (s != RG_OK) {
    delete c;
    return s;
  }
  *out = c;
  return RG_OK;
}

void rg_buckler_circuit_destroy(rg_circuit* c) { delete c; }

rg_status rg_buckler_eval_circuit_dev(const rg_circuit* c, size_t rank, const uint64_t* d_batch_const,
                                      const uint64_t* d_w, size_t n_w, const uint64_t* d_pw, size_t n_pw,
                                      uint64_t* d_out, void* stream) {
  if (!c || !d_batch_const || (rank && !d_out)) return RG_ERR_INVALID;
  if (c->max_w >= (long long)n_w || c->max_pw >= (long long)n_pw) return RG_ERR_INVALID;  // witness index range
  if ((c->max_w >= 0 && !d_w) || (c->max_pw >= 0 && !d_pw)) return RG_ERR_INVALID;
  if (rank == 0) return RG_OK;
  hipStream_t st = as_stream(stream);
#define RG_CIRC(L) circuit_L<L>(c, (long long)rank, d_batch_const, d_w, d_pw, d_out, st)
  RG_DISPATCH_L(c->f.L, RG_CIRC)
#undef RG_CIRC
}

rg_status rg_buckler_eval_circuit(const rg_circuit* c, size_t rank, const uint64_t* batch_const, const uint64_t* w,
                                  size_t n_w, const uint64_t* pw, size_t n_pw, uint64_t* out) {
  if (!c || !batch_const || !out) return RG_ERR_INVALID;
  const size_t L = c->f.L, poly = rank * L * 8;
  DevBuf dbc, dw, dpw, dout;
  RG_TRY(dbc.upload(batch_const, L * 8));
  if (n_w) RG_TRY(dw.upload(w, n_w * poly));
  if (n_pw) RG_TRY(dpw.upload(pw, n_pw * poly));
  RG_TRY(dout.alloc(poly + 8));
  RG_TRY(rg_buckler_eval_circuit_dev(c, rank, dbc.as<uint64_t>(), n_w ? dw.as<uint64_t>() : nullptr, n_w,
                                     n_pw ? dpw.as<uint64_t>() : nullptr, n_pw, dout.as<uint64_t>(), nullptr));
  RG_HIP(hipMemcpy(out, dout.p, poly, hipMemcpyDeviceToHost));
  return RG_OK;
}

}  // extern "C"
