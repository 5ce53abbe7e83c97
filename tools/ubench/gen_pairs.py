"""Generate tools/ubench/pairs.hip: issue cost of single VALU ops and of op PAIRS on independent
register chains (which op classes overlap on a gfx950 SIMD)."""
OPS = {  # name: (asm with {d} = this chain's 32-bit reg, {e} = 64-bit reg, {a} = source), uses64
    "mad64": ("v_mad_u64_u32 {e}, s[40:41], {a}, {a}, {e}", True),
    "mul_lo": ("v_mul_lo_u32 {d}, {a}, {d}", False),
    "mul_hi": ("v_mul_hi_u32 {d}, {a}, {d}", False),
    "add_co": ("v_add_co_u32 {d}, s[42:43], {a}, {d}", False),
    "addc": ("v_addc_co_u32 {d}, s[44:45], {a}, {d}, s[46:47]", False),
    "cnd": ("v_cndmask_b32_e64 {d}, {a}, {d}, s[48:49]", False),
    "add3": ("v_add3_u32 {d}, {a}, {d}, {a}", False),
    "lsh64": ("v_lshl_add_u64 {e}, {e}, 1, {e}", True),
    "add": ("v_add_u32 {d}, {a}, {d}", False),
    "bfi": ("v_bfi_b32 {d}, {a}, {d}, {a}", False),
    "cmp64": ("v_cmp_gt_u64 s[50:51], {e}, {e}", True),
    "sub64": ("v_sub_co_u32 {d}, s[52:53], {a}, {d}", False),
}
CLOB = ', '.join(f'"s{i}"' for i in range(40, 54))
names = list(OPS)
pairs = [(a,) for a in names] + [(a, b) for i, a in enumerate(names) for b in names[i:]]
out = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <cstdint>', '#define ITERS 1024']
for idx, p in enumerate(pairs):
    lines = []
    ops = []
    for j, name in enumerate(p):
        asm, is64 = OPS[name]
        d = f"%{j}"
        ops.append((asm, is64, d))
    body = []
    cons = []
    for j, (asm, is64, d) in enumerate(ops):
        body.append(asm.format(d=d, e=d, a=f"%{len(ops)}"))
        cons.append(f'"+v"({"y" if is64 else "x"}{j}[i])')
    text = "\\n ".join(body)
    out.append(f'''__global__ void __launch_bounds__(256) k{idx}(uint32_t* out, uint32_t seed) {{
  uint32_t a = seed * threadIdx.x | 1; uint32_t x0[8], x1[8]; uint64_t y0[8], y1[8];
  for (int i = 0; i < 8; ++i) {{ x0[i] = a + i; x1[i] = a ^ i; y0[i] = a * 3ull + i; y1[i] = a * 5ull + i; }}
  for (int it = 0; it < ITERS; ++it) {{
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("{text}" : {", ".join(cons)} : "v"(a) : {CLOB});
  }}
  uint32_t s = 0; for (int i = 0; i < 8; ++i) s += x0[i] + x1[i] + (uint32_t)y0[i] + (uint32_t)y1[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}}''')
out.append('''template <typename F> float run(F f, uint32_t* d, int blocks) {
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  f<<<blocks, 256>>>(d, 3); (void)hipDeviceSynchronize(); (void)hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) f<<<blocks, 256>>>(d, 3 + r);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 3; double blk = (double)blocks * 256 * ITERS * 8 / 64;  // wave-iterations
  return (ms * 1e-3 * 2.4e9 * 1024) / blk; }''')
out.append('int main() { int blocks = 256 * 8 * 2; uint32_t* d; (void)hipMalloc(&d, blocks * 256 * 4);')
for idx, p in enumerate(pairs):
    out.append(f'  printf("%-16s %6.2f cyc\\n", "{"+".join(p)}", run(k{idx}, d, blocks));')
out.append('  return 0; }')
open("tools/ubench/pairs.hip", "w").write("\n".join(out) + "\n")
print(len(pairs), "kernels")
