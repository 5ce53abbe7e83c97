// mac_mfma.hpp -- the Jindo Ajtai multiply-accumulate (prover.go:149-157 inner, :180-191 outer)
// on the gfx950 matrix cores: per (limb, coefficient) the modular GEMM
//     out[col][j] = (sum_t A[j][t] B[t][col]) 2^-64 mod q          (+ C[col][j] mod q)
// as exact integer products of base-256 digits on v_mfma_i32_16x16x64_i8 (mac_mfma.hip).
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "common.hpp"

namespace rg {

constexpr int kMfmaMaxQ = 4;

struct MfmaPrime {
  uint64_t q, rinv, rinv_sh, one_sh;  // q, 2^-64 mod q and its Shoup quotient, floor(2^64 / q)
};

struct MfmaMacArgs {
  long long per_col, ncols;  // limbs x degree (lk), columns
  int J, T1, T2, Tc;         // outputs, terms of set 1 / 2, 8-term chunks (ceil((T1 + T2) / 8))
  const uint64_t* Ak;        // key digits [per_col][Tc][64 lanes][2] (mac_mfma_key_dev)
  const uint64_t* corr;      // [per_col][16]: bxor * sum_t A[j][t] * 2^-64 mod q
  const uint64_t* B1;        // [ncols] x b1_col, [T1] x b1_term, lk innermost
  long long b1_col, b1_term;
  const uint64_t* B2;
  long long b2_col, b2_term;
  const uint64_t* C;  // nullable: added after reduction at C[col * c_col + j * c_j + lk]
  long long c_col, c_j;
  uint64_t* out;  // [ncols][J][per_col]
  int d;
  uint64_t bxor;  // the B offset, bytes 0 .. NB-2 equal to 0x80 (set by launch_mac_mfma)
  MfmaPrime P[kMfmaMaxQ];
};

// digits per residue for primes q < 2^(8 NB - 2), or 0 when the MFMA MAC does not apply
// (J > 16, 16 does not divide d, too many terms for the 32-bit diagonal sums)
int mac_mfma_nb(const uint64_t* primes, int nl, int J, int T, int d);
// key layout for `mac_mfma`: digits of A1 [J][T1][per_col] and A2 [J][T2][per_col] (nullable)
// plus the correction table; `out` is (re)allocated
rg_status mac_mfma_key_dev(const uint64_t* A1, int T1, const uint64_t* A2, int T2, int J, long long per_col, int d,
                           int NB, const MfmaPrime* P, int nl, DevBuf& out, hipStream_t st);
// the launch: a.Ak / a.corr point into the DevBuf built above (mac_mfma_key_ptrs)
void mac_mfma_key_ptrs(const DevBuf& key, long long per_col, int T, const uint64_t** Ak, const uint64_t** corr);
uint64_t mac_mfma_bxor(int NB);
rg_status launch_mac_mfma(const MfmaMacArgs& a, int NB, hipStream_t st);

}  // namespace rg
