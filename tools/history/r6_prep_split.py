import sys
src, dst, waves, minw = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
s = open(src).read()
def rep(old, new, cnt=1):
    global s
    assert s.count(old) == cnt, (old[:80], s.count(old)); s = s.replace(old, new)
rep('''template <int MINW, bool PAIR1, int WAVES = kPrepWaves>
__global__ __launch_bounds__(64 * WAVES, MINW) void prep256_kernel(PrepArgs a) {
  __shared__ uint64_t lds_all[WAVES][2 * 288];''', '''template <int MINW, bool PAIR1, int WAVES = kPrepWaves, bool SPLIT = false>
__global__ __launch_bounds__(64 * WAVES, MINW) void prep256_kernel(PrepArgs a) {
  // SPLIT: the wave's exchange image holds 32-bit words (2.25 KiB instead of 4.5), each exchange
  // moving the low then the high halves, so LDS allows 32 waves per CU
  __shared__ uint64_t lds_all[WAVES][SPLIT ? 288 : 2 * 288];''')
rep('''  uint64_t* lds = lds_all[wv];''', '''  uint64_t* lds = lds_all[wv];
  uint32_t* lds32 = reinterpret_cast<uint32_t*>(lds_all[wv]);''')
old = '''    prep_round<3, 5, 0, 1>(e, roots, q, q2, t);
#pragma unroll
    for (int y = 0; y < 8; ++y) lds[rH + 36 * y] = e[y];'''
new = '''    prep_round<3, 5, 0, 1>(e, roots, q, q2, t);
    if constexpr (SPLIT) {
      // xchg: write e[i] at wi(i), read back from ri(i), 32 bits at a time
      auto xchg = [&](auto wi, auto ri) {
        uint32_t h[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) lds32[wi(i)] = (uint32_t)e[i], h[i] = (uint32_t)(e[i] >> 32);
        wave_lds_fence();
        uint32_t lo[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) lo[i] = lds32[ri(i)];
        wave_lds_fence();
#pragma unroll
        for (int i = 0; i < 8; ++i) lds32[wi(i)] = h[i];
        wave_lds_fence();
#pragma unroll
        for (int i = 0; i < 8; ++i) e[i] = ((uint64_t)lds32[ri(i)] << 32) | lo[i];
        wave_lds_fence();
      };
      xchg([&](int y) { return rH + 36 * y; }, [&](int y) { return rM + 4 * y; });
      prep_round<3, 2, 1>(e, roots, q, q2, t);
      xchg([&](int y) { return rM + 4 * y + (y >> 1); }, [&](int r) { return rL9 + r; });
      prep_round<2, 0, 2>(e, roots, q, q2, t);
#pragma unroll
      for (int r = 0; r < 8; ++r) e[r] = canon_x(canon_x(canon_x(e[r], q2), 2 * q), q);  // [0, 8q) -> [0, q)
      xchg([&](int r) { return rL8 + r; }, [&](int y) { return rH + 33 * y; });
      if (active) {
        uint64_t* o = dst + (long long)limb * 256;
#pragma unroll
        for (int y = 0; y < 8; ++y) o[t + 32 * y] = e[y];
      }
      return;
    }
#pragma unroll
    for (int y = 0; y < 8; ++y) lds[rH + 36 * y] = e[y];'''
rep(old, new)
rep('''    constexpr int kBigWaves = 12;''', '''    constexpr int kBigWaves = %d;''' % waves)
rep('''      hipLaunchKernelGGL((prep256_kernel<2, true, kBigWaves>),''', '''      hipLaunchKernelGGL((prep256_kernel<%d, true, kBigWaves, true>),''' % minw)
open(dst, 'w').write(s)
