/* ringo.h -- C ABI of libringo, the MI355X (gfx950) implementation of ringo-snark's
 * NTT / Jindo-commit hot path.
 *
 * Every entry point is what the reference's Go side would bind through cgo (see
 * INTEGRATION.md for the binding).  The reference interface each one replaces is cited as
 * path:line into sp301415/ringo-snark.  Plain pointers and sizes only; no torch types.
 *
 * Conventions
 *  - Field elements are gnark `Uint [L]uint64` values in Montgomery form (R = 2^(64L)),
 *    little-endian limbs, fully reduced (jindo/internal/zp/element.go:37-51).  A polynomial
 *    of rank N is N consecutive elements: layout [N][L] (what a contiguous []zp.Uint holds).
 *  - Batched calls take [batch][N][L] with polys back to back.
 *  - Jindo ring polynomials use Lattigo's limb-major layout Coeffs[limb][coeff]
 *    (ring.Poly, lattigo/v6 v6.1.0).
 *  - `*_dev` entry points take DEVICE pointers and a hipStream_t (passed as void*; NULL =
 *    the null stream) and are asynchronous.  Entry points without `_dev` take HOST pointers
 *    and are synchronous (they stage through library-owned device buffers).
 *  - Outputs may alias inputs exactly (out == in); partial overlap is invalid.
 *  - Return value: RG_OK or a negative rg_status; the library never aborts.  The Go shim
 *    maps the codes to the reference's panics (messages in rg_status_string).
 *  - Handles are immutable after creation and may be shared by threads; each call is
 *    thread-safe (host staging is per call).  A Jindo handle keeps device scratch per HIP
 *    stream, so concurrent `_dev` calls on different streams never share scratch; calls on
 *    one stream are ordered by the stream.  A handle belongs to the device that was current
 *    when it was created (RG_ERR_INVALID elsewhere); one handle per GPU.
 */
#ifndef RINGO_H
#define RINGO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  RG_OK = 0,
  RG_ERR_INVALID = -1,     /* shape/argument error  -> Go panic "inconsistent input(s)" */
  RG_ERR_NOT_POW2 = -2,    /* ntt.go:27-29,154-156  "rank must be a power of two" */
  RG_ERR_UNSUPPORTED = -3, /* ntt.go:35-37,162-164  "NTT not supported" */
  RG_ERR_DEVICE = -4,      /* HIP runtime error (message via rg_last_error) */
  RG_ERR_NOMEM = -5,
  RG_ERR_RANK = -6         /* jindo/prover.go:46-49 "len(v) > params.rank" */
} rg_status;

const char* rg_status_string(int status);
/* Thread-local text of the last device error (hipGetErrorString + call site). */
const char* rg_last_error(void);
/* Library build id (kernel set + gfx target + sampler layout), for logs.  The string ends in
 * "sampler-layout N" with N = RG_SAMPLER_LAYOUT of the build: the partition of the device
 * samplers' draws into UniformSampler instances (rg_jindo_seeds).  The same seeds and
 * first_commit give the same sampled commitments only between builds of one layout.
 *   1: rounds 3-4 (COSAC instances per group of 16 coefficients)
 *   2: round 5 on (COSAC instances per group of 8 coefficients) */
#define RG_SAMPLER_LAYOUT 2
const char* rg_version(void);

/* ------------------------------------------------------------------------------------ */
/* Field (math/bignum.Uint[E], gnark-generated zp.Uint)                                   */
/* ------------------------------------------------------------------------------------ */
typedef struct rg_field rg_field;

/* Replaces the compile-time field type E.  q_le: the modulus as `limbs` little-endian
 * words (zp.q0..q{L-1}, element.go:47-50).  The library derives qInvNeg (element.go:72) and
 * R^2 (element.go:784) itself; rg_field_constants exposes them for cross-checks.
 * limbs in 1..16. */
rg_status rg_field_create(int limbs, const uint64_t* q_le, rg_field** out);
void rg_field_destroy(rg_field* f);
int rg_field_limbs(const rg_field* f);
/* qinv_neg: -q^-1 mod 2^64; r2_le, one_le: R^2 mod q and R mod q (limbs words each). */
rg_status rg_field_constants(const rg_field* f, uint64_t* qinv_neg, uint64_t* r2_le, uint64_t* one_le);

/* ------------------------------------------------------------------------------------ */
/* bigpoly transformers (math/bigpoly/ntt.go)                                             */
/* ------------------------------------------------------------------------------------ */
typedef struct rg_ntt rg_ntt;

/* Replaces NewCyclotomicTransformer (negacyclic=1, ntt.go:153-203) and
 * NewCyclicTransformer (negacyclic=0, ntt.go:26-95).  The library derives psi/omega by the
 * reference's generator search (first x = 2,3,... ; ntt.go:46-53,173-180) and builds the
 * twiddle tables itself. */
rg_status rg_ntt_create(const rg_field* f, int rank, int negacyclic, rg_ntt** out);
/* Same, but with the tables taken verbatim from the Go transformer (tw, twInv: rank
 * elements each in Montgomery form, laid out [rank][L]; rank_inv: one element), so twiddle
 * parity holds by construction.  Tables are validated (tw[0] == twInv[0] == 1). */
rg_status rg_ntt_create_from_tables(const rg_field* f, int rank, int negacyclic, const uint64_t* tw,
                                    const uint64_t* tw_inv, const uint64_t* rank_inv, rg_ntt** out);
void rg_ntt_destroy(rg_ntt* t);
int rg_ntt_rank(const rg_ntt* t); /* Rank() (ntt.go:139,469) */
/* Copy the tables out (Montgomery, [rank][L] each + one element). */
rg_status rg_ntt_tables(const rg_ntt* t, uint64_t* tw, uint64_t* tw_inv, uint64_t* rank_inv);

/* FwdNTTTo(vOut, v) (ntt.go:98-115,206-223) on `batch` polys: natural -> bit-reversed.
 * The _dev forms order all their work on `stream`; a 4-limb plan at rank 2^15 / 2^16 runs half of a
 * batch of 8+ on a helper stream of its own, forked from and joined back into `stream`. */
rg_status rg_ntt_fwd(const rg_ntt* t, uint64_t* out, const uint64_t* in, size_t batch);
rg_status rg_ntt_fwd_dev(const rg_ntt* t, uint64_t* d_out, const uint64_t* d_in, size_t batch, void* stream);
/* InvNTTTo(vOut, v) (ntt.go:118-136,226-244): bit-reversed -> natural, times rank^-1. */
rg_status rg_ntt_inv(const rg_ntt* t, uint64_t* out, const uint64_t* in, size_t batch);
rg_status rg_ntt_inv_dev(const rg_ntt* t, uint64_t* d_out, const uint64_t* d_in, size_t batch, void* stream);

/* ------------------------------------------------------------------------------------ */
/* Pointwise ops (math/bigpoly/vec.go:9-121 via baseOperator, base_op.go:49-171)         */
/* ------------------------------------------------------------------------------------ */
typedef enum {
  RG_VEC_ADD = 0,      /* out = a + b        AddTo        base_op.go:49-55   */
  RG_VEC_SUB = 1,      /* out = a - b        SubTo        base_op.go:64-70   */
  RG_VEC_NEG = 2,      /* out = -a           NegTo        base_op.go:79-85   */
  RG_VEC_MUL = 3,      /* out = a * b        MulTo        base_op.go:133-142 */
  RG_VEC_SMUL = 4,     /* out = a * c        ScalarMulTo  base_op.go:94-100 */
  RG_VEC_MUL_ADD = 5,  /* out += a * b       MulAddTo     base_op.go:144-157 */
  RG_VEC_MUL_SUB = 6,  /* out -= a * b       MulSubTo     base_op.go:159-172 */
  RG_VEC_SMUL_ADD = 7, /* out += a * c       ScalarMulAddTo base_op.go:102-112 */
  RG_VEC_SMUL_SUB = 8  /* out -= a * c       ScalarMulSubTo base_op.go:114-124 */
} rg_vec_op;

/* n elements ([n][L]).  For the SMUL* ops `b` points to ONE element (the scalar c);
 * for NEG `b` is ignored.  Domain checks (IsNTT flags) stay in the caller, as in Go. */
rg_status rg_vec(const rg_field* f, int op, uint64_t* out, const uint64_t* a, const uint64_t* b, size_t n);
rg_status rg_vec_dev(const rg_field* f, int op, uint64_t* d_out, const uint64_t* d_a, const uint64_t* d_b, size_t n,
                     void* stream);

/* ---- remaining bigpoly operators used by Buckler ------------- */
/* CyclicEvaluator.QuoRemByVanishing(p, N) (math/bigpoly/cyclic.go:18-37): quotient and
 * remainder of each of `batch` rank-coefficient polynomials by X^n_vanish - 1 (coefficient
 * domain; the IsNTT / rank panics stay with the caller).  d_rem may alias d_p, d_quo may not. */
rg_status rg_poly_quorem_vanishing_dev(const rg_field* f, size_t rank, long long n_vanish, uint64_t* d_quo,
                                       uint64_t* d_rem, const uint64_t* d_p, size_t batch, void* stream);
rg_status rg_poly_quorem_vanishing(const rg_field* f, size_t rank, long long n_vanish, uint64_t* quo, uint64_t* rem,
                                   const uint64_t* p);
/* CyclotomicEvaluator.AutTo(pOut, p, idx) (cyclotomic.go:29-86): X -> X^idx on each of `batch`
 * polynomials, coefficient domain (ntt_domain = 0, autTo) or NTT domain (autNTTTo).  idx must
 * be odd (RG_ERR_INVALID = the reference's "AutTo: idx must be odd" panic); d_out != d_p. */
rg_status rg_poly_aut_dev(const rg_field* f, size_t rank, long long idx, int ntt_domain, uint64_t* d_out,
                          const uint64_t* d_p, size_t batch, void* stream);
rg_status rg_poly_aut(const rg_field* f, size_t rank, long long idx, int ntt_domain, uint64_t* out, const uint64_t* p);
/* Poly.Evaluate(x) (poly.go:64-76): sum p_i x^i of n coefficients into ONE element d_out;
 * d_scratch holds rg_poly_evaluate_scratch_bytes(f, n) bytes. */
rg_status rg_poly_evaluate_dev(const rg_field* f, const uint64_t* d_p, size_t n, const uint64_t* d_x, uint64_t* d_out,
                               uint64_t* d_scratch, void* stream);
size_t rg_poly_evaluate_scratch_bytes(const rg_field* f, size_t n);
rg_status rg_poly_evaluate(const rg_field* f, const uint64_t* p, size_t n, const uint64_t* x, uint64_t* out);
/* CyclotomicEvaluator.ModSwitchTo(pOut, pBig, qBig) (cyclotomic.go:97-124) on n coefficients:
 * pBig[i] as w little-endian words of a two's-complement integer ([n][w], |pBig[i]| < 2^(64w-1);
 * Go's big.Int values, e.g. PolyToBigintCentered output), qBig as w words (host, 0 < qBig <
 * 2^(64w-1)); out[i] = the reference's round(pBig[i] q / qBig) mod q (remainders above
 * floor(qBig/2) round up) in Montgomery form ([n][L]).  w <= 8.  The rank check ("input size
 * not consistent") and IsNTT = false stay with the caller. */
rg_status rg_poly_modswitch_dev(const rg_field* f, size_t n, const uint64_t* d_pbig, size_t w, const uint64_t* qbig,
                                uint64_t* d_out, void* stream);
rg_status rg_poly_modswitch(const rg_field* f, size_t n, const uint64_t* pbig, size_t w, const uint64_t* qbig,
                            uint64_t* out);

/* ---- Buckler prover device work -------------------------------- */
/* Encoder.EncodeTo / RandEncodeTo (buckler/encoder.go:32-54) of `batch` witness vectors:
 * t is the encoder's CyclicTransformer at the witness rank (newEncoder, encoder.go:15-20; a
 * negacyclic plan is RG_ERR_INVALID).  d_v [batch][rank][L] -> d_out [batch][embed_rank][L]:
 * InvNTT into coefficients 0..rank-1, zeros above.  d_rand [batch][L] (NULL = EncodeTo) holds
 * RandEncodeTo's MustSetRandom draws (Montgomery, injected): coeff[rank] = r, coeff[0] -= r.
 * batch > 1 needs d_scratch of rg_buckler_encode_scratch_bytes(t, batch) bytes. */
rg_status rg_buckler_encode_dev(const rg_ntt* t, size_t embed_rank, uint64_t* d_out, const uint64_t* d_v,
                                size_t batch, const uint64_t* d_rand, uint64_t* d_scratch, void* stream);
size_t rg_buckler_encode_scratch_bytes(const rg_ntt* t, size_t batch);
rg_status rg_buckler_encode(const rg_ntt* t, size_t embed_rank, uint64_t* out, const uint64_t* v,
                            const uint64_t* rand);
/* The arithmetic constraints Prover.evalCircuit walks (buckler/constraint.go:6-12, built by
 * AddTerm / SubTerm / AddTermWithConst): constraint c owns terms term_off[c] .. term_off[c+1]-1;
 * term t = coeffs[t] ([L], Montgomery, < q) * public witness pw_idx[t] (< 0: none, the
 * hasCoeffPublicWitness flag) * witnesses wit_idx[wit_off[t] .. wit_off[t+1]-1] (witnessToID
 * numbering).  Uploaded once (Compile time); immutable. */
typedef struct rg_circuit rg_circuit;
rg_status rg_buckler_circuit_create(const rg_field* f, size_t n_constraints, const size_t* term_off,
                                    const uint64_t* coeffs, const long long* pw_idx, const size_t* wit_off,
                                    const uint64_t* wit_idx, rg_circuit** out);
void rg_buckler_circuit_destroy(rg_circuit* c);
/* Prover.evalCircuit(batchConst, constraints, wData) (buckler/prover.go:355-379): d_out [rank][L]
 * = sum_c batchConst * sum_t coeff_t * pwEcdNTT[pw_t] * prod wEcdNTT[w], NTT domain, fused in one
 * pass.  d_w [n_w][rank][L] = wEcdNTT, d_pw [n_pw][rank][L] = pwEcdNTT, d_batch_const one element;
 * a witness index >= n_w (n_pw) is RG_ERR_INVALID. */
rg_status rg_buckler_eval_circuit_dev(const rg_circuit* c, size_t rank, const uint64_t* d_batch_const,
                                      const uint64_t* d_w, size_t n_w, const uint64_t* d_pw, size_t n_pw,
                                      uint64_t* d_out, void* stream);
rg_status rg_buckler_eval_circuit(const rg_circuit* c, size_t rank, const uint64_t* batch_const, const uint64_t* w,
                                  size_t n_w, const uint64_t* pw, size_t n_pw, uint64_t* out);

/* ------------------------------------------------------------------------------------ */
/* Jindo commitment (jindo/params.go, encoder.go, rns.go, prover.go, entities.go)         */
/* ------------------------------------------------------------------------------------ */
/* Shapes exactly as jindo.Parameters holds them (params.go:64-123); taken from Go
 * (NewParameters' float search is not re-derived here). */
typedef struct {
  int rank, rows, cols, slots; /* Rank() Rows() Cols() Slots()                      */
  int exp;                     /* Exp(): digits per element (k)                      */
  int d;                       /* ring degree = max(k, 256)                          */
  int in_msis, out_msis, mlwe; /* InMSISRank() OutMSISRank() MLWERank()              */
  int dcmp;                    /* InCommitDecomposeLen()                             */
  int log_in_cut, log_out_cut; /* LogInCutOff() OutCutOff()                          */
  uint64_t base;               /* Base(): b with p = b^k + 1                          */
  int nq, nqo;                 /* limbs of RingQ() / RingQOut() (1..4, nqo <= nq)    */
  uint64_t q[4], qo[4];        /* RingQ().ModuliChain(), RingQOut().ModuliChain()   */
  int field_limbs;             /* L of E                                             */
  uint64_t field_q[16];        /* modulus of E, little-endian                        */
} rg_jindo_params;

typedef struct rg_jindo rg_jindo;

/* NewProver's deterministic part (prover.go:28-40): builds RNS NTT tables (Lattigo
 * convention: smallest primitive root >= 3) and uploads the commit key.
 * ck_in   [in_msis][rows][nq][d]   CommitKey.In   (entities.go:24-35)
 * ck_mlwe [in_msis][mlwe][nq][d]   CommitKey.MLWE (entities.go:37-48)
 * ck_out  [out_msis][dcmp][nqo][d] CommitKey.Out  (entities.go:50-61)                 */
rg_status rg_jindo_create(const rg_jindo_params* p, const uint64_t* ck_in, const uint64_t* ck_mlwe,
                          const uint64_t* ck_out, rg_jindo** out);
/* Same, with the commit key in DEVICE memory on the current device (e.g. the buffer an RCCL
 * broadcast of the key landed in): copied device-to-device on `stream`, never
 * through the host.  Returns after the copy and the key transposition have completed. */
rg_status rg_jindo_create_dev(const rg_jindo_params* p, const uint64_t* d_ck_in, const uint64_t* d_ck_mlwe,
                              const uint64_t* d_ck_out, void* stream, rg_jindo** out);
/* Same, deriving the commit key from the CRS exactly as NewCommitKey does
 * (SHA-384 -> AES-256-CTR -> SampleN, entities.go:21-73, uniform.go:38-95). */
rg_status rg_jindo_create_from_crs(const rg_jindo_params* p, const uint8_t* crs, size_t crs_len, rg_jindo** out);
void rg_jindo_destroy(rg_jindo* j);
/* Copy the commit key out (same layouts as rg_jindo_create). */
rg_status rg_jindo_commit_key(const rg_jindo* j, uint64_t* ck_in, uint64_t* ck_mlwe, uint64_t* ck_out);
/* The handle's device-resident commit key (same layouts; valid until rg_jindo_destroy), e.g. as
 * the source of a cross-GPU broadcast. */
rg_status rg_jindo_commit_key_dev(const rg_jindo* j, const uint64_t** d_ck_in, const uint64_t** d_ck_mlwe,
                                  const uint64_t** d_ck_out);

/* Prover.Commit (prover.go:45-62) with the randomness INJECTED so the result is
 * bit-exact against Go given the same draws:
 *  v          [nv][L]  the committed vector, Montgomery (1 <= nv <= rank)
 *  last_row   [cols*slots][L]  genFirstLastRow's MustSetRandom draws, last entry 0 (:68-72)
 *  mask       [rows][slots][L] the mask column's MustSetRandom draws, one row per
 *                              randEncodeTo (:95-115; rows the reference skips are ignored)
 *  enc_noise  [cols+1][rows][d] int64  the Gaussian samples c of each randEncodeTo
 *                              (encoder.go:166-183, TwinCDT or COSAC)
 *  mlwe_noise [cols+1][in_msis+mlwe][d] int64  the MLWE samples (prover.go:130-139)
 * Outputs (Lattigo limb-major residues, NTT + Montgomery domain, as Go holds them):
 *  o_incom  [dcmp][nqo][d]              Opening.InCommit
 *  o_enc    [cols+1][rows][nq][d]       Opening.Encode   (skipped rows = 0, as in Go)
 *  o_mlwe   [cols+1][in_msis+mlwe][nq][d]  Opening.MLWE
 *  o_com    [out_msis][nq][d]           Commitment.Value (rows >= nqo are 0: the reference
 *                                       allocates ringQ polys, entities.go:85-94)       */
rg_status rg_jindo_commit(const rg_jindo* j, const uint64_t* v, size_t nv, const uint64_t* last_row,
                          const uint64_t* mask, const int64_t* enc_noise, const int64_t* mlwe_noise,
                          uint64_t* o_incom, uint64_t* o_enc, uint64_t* o_mlwe, uint64_t* o_com);
/* Device-resident batch: `batch` independent commits of equal length nv; every array above
 * gains a leading [batch] dimension.  Asynchronous on `stream`. */
rg_status rg_jindo_commit_dev(const rg_jindo* j, size_t batch, const uint64_t* d_v, size_t nv,
                              const uint64_t* d_last_row, const uint64_t* d_mask, const int64_t* d_enc_noise,
                              const int64_t* d_mlwe_noise, uint64_t* d_incom, uint64_t* d_enc, uint64_t* d_mlwe,
                              uint64_t* d_com, void* stream);
/* The deterministic Ajtai core of Commit (prover.go:144-202) for a Go caller that keeps its own
 * encoder: from the NTT-domain Opening.Encode [cols+1][rows][nq][d] and Opening.MLWE
 * [cols+1][in_msis+mlwe][nq][d] (as Go holds them after commitColTo's encode and MLWE loops),
 * the inner Ajtai MACs, CRT rounding into Opening.InCommit [dcmp][nqo][d] (:144-176) and
 * outerCommitTo into Commitment.Value [out_msis][nq][d] (:180-202).  `_dev`: `batch` openings
 * back to back, asynchronous on `stream`.
 * Precondition (as in Lattigo, whose ring elements are always reduced): every word of `enc`,
 * `mlwe` and of the commit key given to rg_jindo_create* is a canonical residue (< its prime).
 * The MFMA MAC splits words into base-256 digits under that bound; a non-canonical word gives a
 * wrong commitment, not an error. */
rg_status rg_jindo_commit_core(const rg_jindo* j, const uint64_t* enc, const uint64_t* mlwe, uint64_t* o_incom,
                               uint64_t* o_com);
rg_status rg_jindo_commit_core_dev(const rg_jindo* j, size_t batch, const uint64_t* d_enc, const uint64_t* d_mlwe,
                                   uint64_t* d_incom, uint64_t* d_com, void* stream);
/* Bytes of device scratch rg_jindo_commit_dev needs for `batch` commits (allocated on first
 * use and cached inside the handle, one set per stream; exposed for capacity planning). */
size_t rg_jindo_scratch_bytes(const rg_jindo* j, size_t batch);
/* Drop the scratch cached for `stream` (and for the library-owned stream that splits a sampled
 * commit issued on it), after draining both.  Scratch sets are kept per stream for the handle's
 * lifetime otherwise; a caller that creates streams per request calls this before destroying one
 * (a destroyed stream's handle value may be reused by a new stream).  Not concurrent with calls
 * on that stream. */
rg_status rg_jindo_release_stream(rg_jindo* j, void* stream);
/* Which kernel runs the inner (prover.go:149-157) and outer (:180-191) Ajtai products of this
 * handle: RG_MAC_MFMA (mac_mfma.hip, the matrix cores; needs canonical inputs, see
 * rg_jindo_commit_core_dev) or RG_MAC_GENERIC (mac_kernel).  RG_MAC_VALU3 is never returned by this
 * build (the VALU mac3h kernel was removed in round 6; tools/experiments/jindo_knob_kernels.patch).
 * Introspection only; no reference counterpart. */
enum { RG_MAC_GENERIC = 0, RG_MAC_VALU3 = 1, RG_MAC_MFMA = 2 };
rg_status rg_jindo_mac_kinds(const rg_jindo* j, int* inner, int* outer);

/* ---- the prover's randomness on the device --------------------- */
/* The standard deviations jindo.Parameters holds (params.go:99-111): ecdStdDev,
 * ecdBlindStdDev, maskStdDev, maskBlindStdDev, mlweStdDev, maskMLWEStdDev.  Go takes them from
 * NewParameters' float search; the library builds the TwinCDT tables (gaussian_twin_cdt.go:13-70),
 * the ziggurat tables (gaussian_rounded.go:22-52) and the encoder's deltaInv (encoder.go:50-67)
 * from them.  Setup: call once per handle before the sampled entry points (not concurrently
 * with them).  All must be > 0 (RoundedGaussianSampler panics otherwise). */
typedef struct {
  double ecd, ecd_blind, mask, mask_blind, mlwe, mask_mlwe;
} rg_jindo_stddevs;
rg_status rg_jindo_set_stddevs(rg_jindo* j, const rg_jindo_stddevs* sd);
/* The encoder's deltaInv[exp] (-b^i / p as Go's big.Float computes it, zeroed below
 * 2^-50 / (b exp); encoder.go:50-67). */
rg_status rg_jindo_delta_inv(const rg_jindo* j, double* out);

/* One 32-byte seed per sampler the reference's Commit draws from (each is
 * NewUniformSamplerWithSeed(seed): key = SHA-384(seed)[:32], IV = [32:48], AES-256-CTR,
 * uniform.go:38-54): Encoder.twinCDT, Encoder.cosac and the RoundedGaussianSampler inside it,
 * Prover.mlweSampler, Prover.roundedSampler, and `uniform` in place of crypto/rand for
 * MustSetRandom (prover.go:65-139, encoder.go:149-183).  A Go caller draws them from crypto/rand.
 * On the device each sampler instance is a window of its domain's counter space (instance n =
 * the UniformSampler with IV + n 2^24, a 128-bit sum, so the 2^64 instance numbers have disjoint
 * windows): one per encode polynomial (twinCDT), per group of 8 consecutive coefficients of a
 * COSAC-encoded polynomial (COSAC and its RoundedGaussianSampler, instance poly (d/8) + group),
 * per MLWE polynomial (mlweSampler), per mask-column MLWE sample (rounded) and per field element
 * (uniform), numbered from `first_commit`, the index of
 * the batch's first commit among all commits made with these seeds (so batches and GPUs never
 * share keystream).  The sampled entry points return RG_ERR_INVALID when an instance number of
 * commits [first_commit, first_commit + batch) would pass 2^64 - 1, i.e. when
 * (first_commit + batch) * max((cols+1) rows d, (cols+1)(in_msis+mlwe) d, (cols+rows) slots) > 2^64.
 * Each instance is exactly the reference's sampler; the partition of draws among instances is
 * this library's.  Two provers (e.g. Go's SafeCopy, prover.go:327-339, which gives the copy new
 * crypto/rand samplers) either hold their own seeds or disjoint first_commit ranges. */
typedef struct {
  uint8_t enc_cdt[32], enc_cosac[32], enc_cosac_round[32], mlwe_cdt[32], mlwe_round[32], uniform[32];
} rg_jindo_seeds;
/* The randomness of `batch` commits of v (the layouts rg_jindo_commit_dev takes): lastRow (last
 * entry 0) and mask elements, the Gaussian samples of every randEncodeTo (centres from deltaInv
 * and the digits of the encoded elements) and of every MLWE polynomial.  Skipped encodes get 0. */
rg_status rg_jindo_sample_dev(const rg_jindo* j, size_t batch, const uint64_t* d_v, size_t nv,
                              const rg_jindo_seeds* seeds, unsigned long long first_commit, uint64_t* d_last_row,
                              uint64_t* d_mask, int64_t* d_enc_noise, int64_t* d_mlwe_noise, void* stream);
/* Prover.Commit end to end on the device (prover.go:45-202): rg_jindo_sample_dev, then
 * rg_jindo_commit_dev on that randomness (kept in the stream's scratch).  The batch runs as a DAG
 * over `stream` and two library-owned streams of that caller stream joined to it by events (the
 * COSAC sampler and the MLWE samplers beside TwinCDT, so each fills the others' tails); the
 * outputs are complete, as usual, when `stream` has passed the call. */
rg_status rg_jindo_commit_sampled_dev(const rg_jindo* j, size_t batch, const uint64_t* d_v, size_t nv,
                                      const rg_jindo_seeds* seeds, unsigned long long first_commit, uint64_t* d_incom,
                                      uint64_t* d_enc, uint64_t* d_mlwe, uint64_t* d_com, void* stream);
/* UniformSampler.Sample() words [first_word, first_word + n) of instance `instance` of
 * NewUniformSamplerWithSeed(seed) (instance 0 is that sampler itself; uniform.go:56-82, including
 * the XOR-accumulating 8192-byte buffer). */
rg_status rg_uniform_words_dev(const uint8_t* seed, size_t seed_len, unsigned long long instance,
                               unsigned long long first_word, size_t n, uint64_t* d_out, void* stream);

/* Prover.Evaluate (prover.go:205-324), device-resident, with the Fiat-Shamir challenges
 * INJECTED: the transcript (SHAKE128 over CommitKey/Commitment/Proof serializations),
 * encodeChallengeTo, leftVec/encode and Poly.Evaluate stay in the Go caller, which also keeps
 * the shape panics (:206-216).  Challenge polynomials are ringQ / ringQOut residues in the
 * NTT + Montgomery domain, as Go holds them; every product is MulCoeffsMontgomeryThenAdd.
 * 1. openBatch = sum_i open[i] * batch[i] (:228-266); with d_bq = d_bo = NULL (params.batch == 1,
 *    batch must be 1) openBatch = open[0] (:267-269).  A GPU holding a shard of a batch passes its
 *    openings and their challenges; the shards' openBatches sum across GPUs (RCCL all-reduce of
 *    the words, exact while n_gpus * q < 2^64) and rg_jindo_eval_reduce_dev folds them mod q.
 *      d_incom [batch][dcmp][nqo][d], d_enc [batch][cols+1][rows][nq][d],
 *      d_mlwe [batch][cols+1][in_msis+mlwe][nq][d]  the openings (rg_jindo_commit_dev layout)
 *      d_bq [batch][nq][d], d_bo [batch][nqo][d]     batch[i] in ringQ and batchOut[i] in ringQOut
 *      d_ob_*  openBatch in the single-opening layouts; openBatch.InCommit = Proof.InCommit */
rg_status rg_jindo_eval_batch_dev(const rg_jindo* j, size_t batch, const uint64_t* d_incom, const uint64_t* d_enc,
                                  const uint64_t* d_mlwe, const uint64_t* d_bq, const uint64_t* d_bo,
                                  uint64_t* d_ob_incom, uint64_t* d_ob_enc, uint64_t* d_ob_mlwe, void* stream);
/* words mod q, in place, over an openBatch (after a cross-GPU sum of partial openBatches) */
rg_status rg_jindo_eval_reduce_dev(const rg_jindo* j, uint64_t* d_ob_incom, uint64_t* d_ob_enc, uint64_t* d_ob_mlwe,
                                   void* stream);
/* 2. Proof.Partial[i] = sum_j left[j] * openBatch.Encode[i][j] (:274-278) and
 *    Proof.PartialMask over column cols (:280-282):
 *      d_left [rows][nq][d] (encode(leftVec(x)[j]))   d_partial [cols+1][nq][d], last = PartialMask */
rg_status rg_jindo_eval_partial_dev(const rg_jindo* j, const uint64_t* d_ob_enc, const uint64_t* d_left,
                                    uint64_t* d_partial, void* stream);
/* 3. Proof.Encode[i] = openBatch.Encode[cols][i] + sum_j chals[j] * openBatch.Encode[j][i] and
 *    Proof.MLWE[i] likewise (:300-314):
 *      d_chals [cols][nq][d]   d_pf_enc [rows][nq][d]   d_pf_mlwe [in_msis+mlwe][nq][d]          */
rg_status rg_jindo_eval_respond_dev(const rg_jindo* j, const uint64_t* d_ob_enc, const uint64_t* d_ob_mlwe,
                                    const uint64_t* d_chals, uint64_t* d_pf_enc, uint64_t* d_pf_mlwe, void* stream);

/* Verifier.Verify (verifier.go:50-282), device-resident, with the Fiat-Shamir challenges
 * INJECTED as in Evaluate: the caller replays the transcript (SHAKE128 over the commit key,
 * commitments, x, Proof.Partial; :56-96), encodes the challenges (encodeChallengeTo), computes
 * leftVec/encode and rightVec (utils.go:63-82) and keeps the shape panics (:51-54).
 *   d_com   [batch][out_msis][nq][d]  the commitments (rg_jindo_commit_dev layout)
 *   d_bq, d_bo [batch][nq][d], [batch][nqo][d]  batch[i] / batchOut[i]; NULL when batch == 1
 *   d_chals [cols][nq][d]   d_left [rows][nq][d] (encode(leftVec(x)[j]))
 *   d_right [cols*slots][L] rightVec(x)   d_y [batch][L]  the claimed evaluations (Montgomery)
 *   the Proof: d_pf_incom [dcmp][nqo][d], d_pf_partial [cols+1][nq][d] (Partial, then
 *   PartialMask), d_pf_enc [rows][nq][d], d_pf_mlwe [in_msis+mlwe][nq][d]  (as Evaluate wrote)
 *   in_com_dcmp_two_nm, res_two_nm: Parameters.InComDcmpTwoNm() / ResTwoNm() (params.go:432-440)
 * All four checks run (the reference stops at the first failure; `ok` is the same verdict).
 * ModUpQtoP (:173) is taken as the centred lift of the ringQOut coefficients (the reading under
 * which the reference's own TestJindo completes; Lattigo's source is absent: parity unpinned).
 * Synchronous: returns after the result is on the host. */
typedef struct {
  uint64_t outer_norm_sq[10]; /* verifyNorm's nmSq before Sqrt (:263-276), little-endian words */
  uint64_t inner_norm_sq[10];
  int outer_ok, inner_ok;     /* Float64(isqrt(nmSq)) < bound (:278-281), decided exactly  */
  int consistency_ok;         /* verifyConsistency (:203-221)                              */
  int eval_ok;                /* verifyEval (:224-259)                                     */
  uint64_t eval_lhs[16];      /* sum right * Decode(Partial) (Montgomery)                  */
  uint64_t eval_rhs[16];      /* yBatch                                                    */
  int ok;                     /* Verify's return value                                     */
} rg_jindo_verify_result;
rg_status rg_jindo_verify_dev(const rg_jindo* j, size_t batch, const uint64_t* d_com, const uint64_t* d_bq,
                              const uint64_t* d_bo, const uint64_t* d_chals, const uint64_t* d_left,
                              const uint64_t* d_right, const uint64_t* d_y, const uint64_t* d_pf_incom,
                              const uint64_t* d_pf_partial, const uint64_t* d_pf_enc, const uint64_t* d_pf_mlwe,
                              double in_com_dcmp_two_nm, double res_two_nm, rg_jindo_verify_result* res,
                              void* stream);

/* ------------------------------------------------------------------------------------ */
/* Device memory helpers (so a cgo caller needs no HIP headers)                           */
/* ------------------------------------------------------------------------------------ */
rg_status rg_malloc(void** d_ptr, size_t bytes);
rg_status rg_free(void* d_ptr);
rg_status rg_memcpy_h2d(void* d_dst, const void* src, size_t bytes, void* stream);
rg_status rg_memcpy_d2h(void* dst, const void* d_src, size_t bytes, void* stream);
rg_status rg_memcpy_d2d(void* d_dst, const void* d_src, size_t bytes, void* stream);
rg_status rg_stream_sync(void* stream);
rg_status rg_set_device(int device);
/* Measurement hook.  libringo.so refuses every probe but 0 (RG_ERR_INVALID): no production call
 * can switch a kernel.  Only the experiments build (libringo_exp.so, bench.py's compute-floor
 * legs and tools/) honours it: probe 4 makes the single-word 2^16 NTT launches (ntt16_pass), probe
 * 5 the q255 2^16 launches (ntt256_pass), skip their HBM data loads and stores, so the same
 * launches time the kernel's compute floor; their outputs are then meaningless.  0 restores the
 * production kernels.  Per calling thread. */
rg_status rg_set_probe(int probe);
/* the calling thread's current device (one rank per GPU: LOCAL_RANK -> rg_set_device) */
rg_status rg_get_device(int* device);
rg_status rg_device_count(int* n);

#ifdef __cplusplus
}
#endif
#endif /* RINGO_H */
