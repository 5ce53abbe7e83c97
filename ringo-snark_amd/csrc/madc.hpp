// madc.hpp -- multiply-accumulate steps of the wide fields' 32-bit-digit product-scanning
// Montgomery products (ntt_wide.hpp, 7 and 14 limbs), as asm statements of several instructions.
//
// A column accumulator is (H:A), A a 64-bit VGPR pair and H a 32-bit VGPR: one partial product is
// `v_mad_u64_u32 A, c, x, y, A` (carry-out c, an SGPR lane mask) and `v_addc_co_u32 H, c, H, 0, c`.
// No builtin exposes the mad's carry-out, and hipcc pads one wait state (`s_nop 0`) after every
// asm statement whose outputs a following VALU touches.  A pad costs the wave ~4 issue cycles but
// no VALU cycles, so it is free where enough waves share a SIMD (the 4-limb ntt256_pass keeps its
// one-instruction statements: it is VALU-throughput-bound at 3-4 waves/SIMD, and a two-chain
// product, counted in its compiled kernel, had 23% more VALU instructions and 60% fewer pads)
// and not free at the 2-3 waves/SIMD of the 14-limb registers.  Here a statement carries 2 or 4
// partial products of a column's two independent chains.
//
// Wait states inside a statement are ours to place.  hipcc models a VALU write of an SGPR
// followed by a VALU read of it (a carry-in) as needing two wait states on gfx942 / gfx950 (it
// pads its own `v_add_co` / `v_addc_co` pairs with `s_nop 1`), so every carry read below is at
// least two instructions after the write that produced it: the four-product step writes four
// carries, then consumes them in order.  VGPR dependences (A, H) need no padding.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

namespace rg {

#if defined(__HIPCC__)

// Compile-time loops: the products are hundreds of partial products, past what the loop unroller
// fully unrolls, and a rolled loop indexes the digit arrays dynamically (s_set_gpr_idx).
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

typedef unsigned long long madc_mask;  // wave64 lane mask (SGPR pair)

// (H:A) += x y
__device__ __forceinline__ void madc1(uint64_t& A, uint32_t& H, uint32_t x, uint32_t y) {
  madc_mask c;
  asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\ts_nop 1\n\tv_addc_co_u32 %1, %2, %1, 0, %2"
      : "+v"(A), "+v"(H), "=&s"(c)
      : "v"(x), "v"(y));
}

// (H:A) += x y and (G:B) += m n
__device__ __forceinline__ void madc2(uint64_t& A, uint32_t& H, uint32_t x, uint32_t y, uint64_t& B, uint32_t& G,
                                      uint32_t m, uint32_t n) {
  madc_mask c, c2;
  asm("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %2, %5, %8, %9, %2\n\ts_nop 0\n\t"
      "v_addc_co_u32 %1, %4, %1, 0, %4\n\tv_addc_co_u32 %3, %5, %3, 0, %5"
      : "+v"(A), "+v"(H), "+v"(B), "+v"(G), "=&s"(c), "=&s"(c2)
      : "v"(x), "v"(y), "v"(m), "v"(n));
}

// (H:A) += x0 y0 + x1 y1 and (G:B) += m0 n0 + m1 n1
__device__ __forceinline__ void madc4(uint64_t& A, uint32_t& H, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1,
                                      uint64_t& B, uint32_t& G, uint32_t m0, uint32_t n0, uint32_t m1, uint32_t n1) {
  madc_mask c0, c1, c2, c3;
  asm("v_mad_u64_u32 %0, %4, %8, %9, %0\n\tv_mad_u64_u32 %2, %5, %12, %13, %2\n\t"
      "v_mad_u64_u32 %0, %6, %10, %11, %0\n\tv_mad_u64_u32 %2, %7, %14, %15, %2\n\t"
      "v_addc_co_u32 %1, %4, %1, 0, %4\n\tv_addc_co_u32 %3, %5, %3, 0, %5\n\t"
      "v_addc_co_u32 %1, %6, %1, 0, %6\n\tv_addc_co_u32 %3, %7, %3, 0, %7"
      : "+v"(A), "+v"(H), "+v"(B), "+v"(G), "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3)
      : "v"(x0), "v"(y0), "v"(x1), "v"(y1), "v"(m0), "v"(n0), "v"(m1), "v"(n1));
}

// One column of a two-chain product: (H:A) += sum_r X(r) Y(r) for r < NX and
// (G:B) += sum_r M(r) N(r) for r < NM, X/Y/M/N compile-time-indexed accessors.
template <int NX, int NM, class FX, class FY, class FM, class FN>
__device__ __forceinline__ void madc_column(uint64_t& A, uint32_t& H, uint64_t& B, uint32_t& G, FX&& X, FY&& Y,
                                            FM&& M, FN&& N) {
  constexpr int NMAX = NX > NM ? NX : NM;
  static_for<NMAX>([&](auto ic) {
    constexpr int r = decltype(ic)::value;
    if constexpr (r % 2 == 1 && r < NX && r < NM) {
      // taken by step r - 1's four-product statement
    } else if constexpr (r % 2 == 0 && r + 1 < NX && r + 1 < NM) {
      madc4(A, H, X(ic), Y(ic), X(std::integral_constant<int, r + 1>{}), Y(std::integral_constant<int, r + 1>{}), B,
            G, M(ic), N(ic), M(std::integral_constant<int, r + 1>{}), N(std::integral_constant<int, r + 1>{}));
    } else if constexpr (r < NX && r < NM) {
      madc2(A, H, X(ic), Y(ic), B, G, M(ic), N(ic));
    } else if constexpr (r < NX) {
      madc1(A, H, X(ic), Y(ic));
    } else if constexpr (r < NM) {
      madc1(B, G, M(ic), N(ic));
    }
  });
}

#endif  // __HIPCC__

}  // namespace rg
