// Read bandwidth of LDS-DMA (global_load_lds_dwordx4) streams, no compute: the Jindo MAC's opening
// pattern (8 lk = 64 B of each 4-KiB (column, term) row, 16 columns x 64 terms per step) against
// the same bytes read as contiguous 1-KiB blocks.  hipcc -O3 --offload-arch=gfx950 dma_pattern.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ void glds16(const void* g, uint32_t l) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(l) : "memory");
}

// mode 0: MAC pattern; mode 1: contiguous.  Grid: nlk (= per_col / 8) x R workgroups of 512 threads.
template <int MODE, int LKW>
__global__ __launch_bounds__(512, 1) void stream(const uint64_t* B, long long ncols, int T, long long per_col, int R, int steps_per_tile, unsigned long long* sink) {
  __shared__ uint64_t lds[4 * 4096];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const unsigned g = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  const long long nlk = per_col / LKW, nct = (ncols + 15) / 16;
  const long long lkg = g / R, rr = g % R;
  const long long lk0 = lkg * LKW;
  const long long tlo = nct * rr / R, thi = nct * (rr + 1) / R;
  const long long S = (thi - tlo) * steps_per_tile;
  const uint32_t l0 = (uint32_t)(uintptr_t)lds;
  const long long bcol = (long long)T * per_col, bterm = per_col;
  auto issue = [&](long long s) {
    if (s >= S) s = S - 1;
    const long long tile = tlo + s / steps_per_tile;
    const int c = (int)(s % steps_per_tile);
    const uint32_t sb = l0 + (uint32_t)(s & 1) * 65536u;
    for (int h = 0; h < 2; ++h)
      for (int k = 0; k < 4; ++k) {
        const int u = 8 * k + w;
        const uint64_t* src;
        if (MODE == 0) {
          // instruction q covers col group cg (cpi columns) of term tt; lanes = (lk pair, column)
          constexpr int cpi = 128 / LKW, ncg = 16 / cpi;
          const int q = h * 32 + u, cg = q % ncg, tt = q / ncg;
          int t = (64 * cpi / 16) * c + tt;
          if (t >= T) t = T - 1;
          const long long dc = tile * 16 + cg * cpi + (lane % cpi);
          src = B + dc * bcol + (long long)t * bterm + lk0 + 2 * (lane / cpi);
        } else {
          // the workgroup's share of the same bytes as contiguous 1-KiB blocks
          const long long blk = ((lkg * R + rr) * S + s) * 64 + h * 32 + u;
          src = B + (blk * 128) % (ncols * bcol - 128) + 2 * lane;
        }
        glds16(src, sb + (uint32_t)(h * 32768 + u * 1024));
      }
  };
  issue(0);
  issue(1);
  unsigned long long acc = 0;
  for (long long s = 0; s < S; ++s) {
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    acc += lds[(s & 1) * 8192 + threadIdx.x];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    issue(s + 2);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 0x123456789ull) sink[0] = acc;
}

int main() {
  const long long per_col = 512, ncols = 4608;
  const int T = 545;
  const size_t n = (size_t)ncols * T * per_col;
  uint64_t* B;
  unsigned long long* sink;
  if (hipMalloc(&B, n * 8) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess) return 1;
  (void)hipMemset(B, 1, n * 8);
  auto steps_for = [&](int lkw) { const int tps = 64 * (128 / lkw) / 16; return (T + tps - 1) / tps; };
  const double gb = (double)n * 8 / 1e9;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto bench = [&](const char* name, auto launch) {
    launch();
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    printf("%s: %.3f ms, %.2f TB/s\n", name, ms, gb / ms);
  };
  char nm[64];
  for (int R : {4, 8, 16, 32}) {
    snprintf(nm, 64, "lk8  R=%d", R);
    bench(nm, [&] { hipLaunchKernelGGL((stream<0, 8>), dim3(64 * R), dim3(512), 0, 0, B, ncols, T, per_col, R, steps_for(8), sink); });
    snprintf(nm, 64, "lk16 R=%d", R);
    bench(nm, [&] { hipLaunchKernelGGL((stream<0, 16>), dim3(32 * R), dim3(512), 0, 0, B, ncols, T, per_col, R, steps_for(16), sink); });
    snprintf(nm, 64, "lk32 R=%d", R);
    bench(nm, [&] { hipLaunchKernelGGL((stream<0, 32>), dim3(16 * R), dim3(512), 0, 0, B, ncols, T, per_col, R, steps_for(32), sink); });
  }
  bench("contiguous", [&] { hipLaunchKernelGGL((stream<1, 8>), dim3(64 * 8), dim3(512), 0, 0, B, ncols, T, per_col, 8, steps_for(8), sink); });
  return 0;
}
