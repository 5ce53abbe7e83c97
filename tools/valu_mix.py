"""Per-kernel VALU issue cost from the gfx950 assembly of the library build: the static mix of
each kernel's VALU instructions weighted by the measured cycles per wave64 instruction per SIMD
of its class (tools/ubench/ops2.hip, intmul.hip, ops3.hip; table below).  bench.py multiplies a
kernel's dynamic SQ_INSTS_VALU (PMC) by this mean to get its VALU issue floor, instead of one
cost for every instruction.  The static mix stands in for the dynamic one: exact for the
unrolled kernels (NTT passes, prep256, MAC), an approximation where loop bodies differ in mix.

usage: python tools/valu_mix.py out.json libringo.so file.s [file.s ...]
(the .s files: hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S, as tools/valu_mix.sh builds them)"""
import json
import re
import sys
from collections import Counter

# cycles per wave64 instruction per SIMD at 2.4 GHz, measured on MI355X
FULL, HALF = 2.4, 4.5
COST = {
    # full rate (ops2.hip): plain 32-bit add/sub/logic/moves/shifts, VOP2 cndmask on vcc
    "v_add_u32": FULL, "v_sub_u32": FULL, "v_subrev_u32": FULL, "v_and_b32": FULL, "v_or_b32": FULL,
    "v_xor_b32": FULL, "v_not_b32": FULL, "v_mov_b32": FULL, "v_lshrrev_b32": FULL, "v_ashrrev_i32": FULL,
    "v_cndmask_b32_e32": FULL, "v_readfirstlane_b32": 4.25, "v_readlane_b32": 4.25, "v_writelane_b32": 4.25,
    "v_mbcnt_lo_u32_b32": FULL, "v_mbcnt_hi_u32_b32": FULL,
    # ops3.hip (MI355X, round 3): VOP3 / 64-bit / f64 forms and lane ops
    "v_perm_b32": 4.52, "v_bitop3_b32": 3.67, "v_mov_b64_e32": 4.65, "v_lshl_add_u64": 4.80, "v_lshlrev_b64": 4.18,
    "v_add_f64": 4.58, "v_mul_f64": 4.25, "v_fma_f64": 4.65, "v_fmac_f64_e32": 4.65, "v_cvt_f32_u32_e32": 4.07,
    "v_cmp_lt_u64_e32": 4.51, "v_mul_hi_u32_u24_e32": 4.09, "v_mul_u32_u24_e32": 4.26, "v_floor_f64_e32": 4.50,
    "v_lshl_or_b32": 4.28, "v_exp_f32_e32": 8.15, "v_rcp_f64_e32": 16.41, "v_ldexp_f64": 4.20,
}
# half rate (ops2.hip / intmul.hip): multiplies, carry chains, VOP3 three-operand forms, 64-bit ops
HALF_PREFIX = ("v_mad_u64_u32", "v_mad_i64_i32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mul_hi_i32", "v_add_co_u32",
               "v_addc_co_u32", "v_sub_co_u32", "v_subb_co_u32", "v_subrev_co_u32", "v_subbrev_co_u32",
               "v_cndmask_b32_e64", "v_add3_u32", "v_bfi_b32", "v_alignbit_b32", "v_lshl_add_u64", "v_cmp_",
               "v_min_", "v_max_", "v_lshlrev_b32", "v_lshlrev_b64", "v_lshrrev_b64", "v_ashrrev_i64",
               "v_mov_b64", "v_lshl_add_u32", "v_add_lshl_u32", "v_lshl_or_b32", "v_and_or_b32", "v_or3_b32",
               "v_xad_u32", "v_med3_", "v_perm_b32", "v_bitop3_", "v_bfe_", "v_mul_u32_u24", "v_mad_u32_u24",
               "v_mul_i32_i24", "v_mad_i32_i24", "v_mul_hi_u32_u24", "v_ffb", "v_bcnt", "v_mul_lo_u16",
               "v_sub_u16", "v_lshlrev_b16", "v_lshrrev_b16", "v_add_u32_sdwa", "v_lshlrev_b32_sdwa",
               "v_or_b32_sdwa")
# f64 and conversions: half rate on MI355X (FP64 vector = half the FP32 rate); transcendental and
# f64 reciprocal / divide steps: quarter rate
QUARTER_PREFIX = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_", "v_div_", "v_frexp_",
                  "v_rcp_iflag")
F64_PREFIX = ("v_add_f64", "v_mul_f64", "v_fma_f64", "v_fmac_f64", "v_ldexp_f64", "v_floor_f64", "v_ceil_f64",
              "v_trunc_f64", "v_rndne_f64", "v_cvt_", "v_fract_f64", "v_max_f64", "v_min_f64")
F32_PREFIX = ("v_mul_f32", "v_add_f32", "v_fma_f32", "v_fmac_f32", "v_fmamk_f32", "v_trunc_f32", "v_sub_f32")


def cost(op):
    base = op.split("_e32")[0].split("_e64")[0] if op not in COST else op
    if op in COST:
        return COST[op]
    if base in COST:
        return COST[base]
    if op.startswith(QUARTER_PREFIX):
        return 2 * HALF
    if op.startswith(F64_PREFIX) or op.startswith(HALF_PREFIX):
        return HALF
    if op.startswith(F32_PREFIX):
        return FULL
    return FULL  # unlisted: the cheaper class (keeps the floor a lower bound)


def kernels(path):
    s = open(path).read()
    for m in re.finditer(r"^(_Z\S+):[ \t]*(?:;[^\n]*)?$(.*?)^\.Lfunc_end", s, re.M | re.S):
        ops = [l.split()[0] for l in m.group(2).split("\n") if l.startswith("\t") and l.strip().startswith("v_")]
        yield m.group(1), Counter(ops)


def demangle(names):
    import subprocess
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
    return r.stdout.strip().split("\n")


def main():
    import hashlib
    out, lib, files = sys.argv[1], sys.argv[2], sys.argv[3:]
    res = {"lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
           "costs": {"full": FULL, "half": HALF, "quarter": 2 * HALF},
           "note": "mean cycles per wave64 VALU instruction per SIMD of each kernel's static VALU mix", "kernels": {}}
    for f in files:
        for name, c in kernels(f):
            n = sum(c.values())
            if not n:
                continue
            cyc = sum(cost(op) * k for op, k in c.items()) / n
            res["kernels"][name] = {"valu_static": n, "mean_cycles": round(cyc, 4),
                                    "half_or_slower_frac": round(sum(k for op, k in c.items() if cost(op) > FULL) / n, 4)}
    names = list(res["kernels"])
    res["kernels"] = {d: res["kernels"][m] for m, d in zip(names, demangle(names))}  # rocprofv3's names
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(f"{len(res['kernels'])} kernels -> {out}")


if __name__ == "__main__":
    main()
