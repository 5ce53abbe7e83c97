"""bench.py -- NTT / Jindo-commit throughput of libringo on MI355X.

Contract (see task): `python bench.py --gpus N --steps K --warmup W`.  Under
torch.distributed.run (WORLD_SIZE set) each process is one rank on one GPU (RCCL); run plainly
with --gpus N > 1, bench.py starts torch.distributed.run itself as a CHILD process (before any
GPU call) and exits with its code.  Rank 0 prints ONE JSON line.

Headline (BASELINE.json configs[1]): forward + inverse negacyclic NTT, degree 2^16, the single
63-bit jindo-modulus prime p = 47104^4 + 1, batch 1024 polynomials per GPU, inputs resident in
HBM.  One step = FwdNTTTo then InvNTTTo over the whole batch (2048 transforms).  Unit: NTTs/s
(one forward or one inverse transform of one polynomial), whole job.  Scaling: weak (each rank
owns its own 1024 polys; no data-path collective).

Secondary lines in the same JSON object (also measured, not the headline value):
  * l4_ntt: the same fwd+inv step at the Jindo default 255-bit prime (configs[3]), batch 64
  * jindo_commit: device-resident Jindo commits/s at targetN 2^14 (configs[2])
  * jindo_commit_2e16 (+ jindo_evaluate_2e16): the configs[4] shape, 512 commits per GPU
    (4096 / 8); at N > 1 the commit key is derived on rank 0 and RCCL-broadcast device to device

roofline: for the NTT transform (two LDS-tiled pass kernels per transform): algorithmic bytes =
one read + one write of N*8 B per polynomial per transform; achieved = those bytes / the
transform's duration measured with HIP events on the launch stream over the timed region.
traffic / valu: per-line HBM bytes (rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE) and VALU
instruction counts (SQ_INSTS_VALU) from profiles/kernel_counters.json, which
tools/profile_bench.sh writes for the libringo.so it profiled; reported only when that file's
library hash equals the library this run loaded (else null, "stale").
cpu_baseline: the C restatement (oracle/liboracle.so, threads) timed on this host on bounded
samples of the NTT headline and of the configs[2] Jindo commit.
"""
import argparse
import hashlib
import json
import os
import re
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ringo-snark_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

P63 = 47104 ** 4 + 1
Q255 = 0x430D45996B62AFC2D65643D9E6FB65558E9630DC8C3732810000000000000001
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
SIMDS, CLOCK_HZ = 1024, 2.4e9  # 256 CUs x 4 SIMDs; sustained shader clock under this load
VALU_CYCLES = 4.5  # mean issue cost (cycles / wave64 instruction / SIMD) of the half-rate 64-bit
                   # integer ops these kernels are made of (tools/ubench)
STEPS_DONE = {}  # line -> steps executed incl. prewarm/warmup (for per-step PMC attribution)
try:  # per-kernel mean VALU issue cost of this library's static instruction mix (tools/valu_mix.py)
    VALU_MIX = json.load(open(os.path.join(ROOT, "profiles", "valu_mix.json")))
except (OSError, ValueError):
    VALU_MIX = {}


def splitmix64(seed, n):
    """SplitMix64 stream (SURVEY.md §8d synthetic inputs), vectorised in numpy."""
    with np.errstate(over="ignore"):
        idx = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform_elems(q, L, n, seed):
    """n uniform residues in [0, q) as [n][L] limbs.  The Montgomery map is a bijection on
    [0, q), so these are also uniform Montgomery representations."""
    if L == 1:
        v = splitmix64(seed, n)
        return (v % np.uint64(q)).reshape(n, 1)
    w = splitmix64(seed, n * L).reshape(n, L)
    top = (q >> (64 * (L - 1))).bit_length()
    w[:, L - 1] &= np.uint64((1 << max(top - 1, 1)) - 1)  # < 2^(bits-1) <= q: in range
    return w


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--logn", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-extra", action="store_true", help="skip the L=4 / Jindo lines")
    ap.add_argument("--extra", default="l4,wide,j14,j16",
                    help="secondary lines to run: l4, wide, j14, j16 (comma list)")
    ap.add_argument("--no-ntt", action="store_true", help="skip the headline NTT line (profiling one line)")
    ap.add_argument("--no-prewarm", action="store_true", help="no time-based prewarm (deterministic step count)")
    ap.add_argument("--plumbing", action="store_true",
                    help="CPU-only launcher/timing check: gloo ranks, a trivial host step, no GPU, no libringo")
    ap.add_argument("--j14-batch", type=int, default=256, help="commits per GPU per step, configs[2] shape")
    ap.add_argument("--j16-batch", type=int, default=512,
                    help="commits per GPU per step, configs[4] shape (4096 commits / 8 GPUs)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    return ap.parse_args()


class Events:
    """HIP-event timing of a region on one stream (the stream the kernels are launched on).
    One event pair brackets the whole timed region: an event between consecutive kernels makes
    the runtime insert a release fence that writes back the caches, which perturbs what is
    measured (tools/nttlab/pass_lab: ~15-25% slower with per-pass events)."""

    def __init__(self, torch, stream):
        self.torch, self.stream = torch, stream
        self.e0 = torch.cuda.Event(enable_timing=True)
        self.e1 = torch.cuda.Event(enable_timing=True)

    def start(self):
        self.e0.record(self.stream)

    def stop(self):
        self.e1.record(self.stream)

    def total_ms(self):
        return self.e0.elapsed_time(self.e1)


PREWARM = [True]


def prewarm(torch, fn, seconds=0.3):
    seconds = float(os.environ.get("RINGO_PREWARM_S", seconds))
    """Untimed: run the step until the GPU has held its sustained clock for a while (the first
    ~20 steps of this integer-multiply-heavy load run 10-30% slower while power management
    settles; tools/nttlab/pass_lab 'ramp').  Returns the number of steps run."""
    n = 0
    t0 = time.perf_counter()
    while PREWARM[0] and time.perf_counter() - t0 < seconds:
        fn()
        torch.cuda.synchronize()
        n += 1
    return n


def ntt_step_bench(torch, ringo, dist, q, L, batch, logn, steps, warmup, seed):
    N = 1 << logn
    dev = torch.device("cuda", torch.cuda.current_device())
    F = ringo.Field(q)
    T = ringo.CyclotomicTransformer(F, N)
    host = uniform_elems(q, L, batch * N, seed)
    x = torch.from_numpy(host.view(np.int64).reshape(-1)).to(dev)
    ref = x.clone()
    stream = torch.cuda.current_stream()

    def step():
        T.fwd_dev(x, x, batch, stream)
        T.inv_dev(x, x, batch, stream)

    nw = prewarm(torch, step)
    for _ in range(warmup):
        step()
    STEPS_DONE["ntt" if L == 1 else "l4"] = nw + warmup + steps
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ev = Events(torch, stream)
    t0 = time.perf_counter()
    ev.start()
    for _ in range(steps):
        step()
    ev.stop()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ok = bool(torch.equal(x, ref))  # fwd then inv is the identity: full-size self-check
    kern_ms = ev.total_ms()
    floor_ms = None
    if logn == 16 and L in (1, 4):
        floor_ms = compute_floor(torch, ringo, q, L, N, batch, x, stream, steps, warmup)
        ok = ok and bool(torch.equal(x, ref))
    return dict(wall_s=wall, kernel_ms=kern_ms, ok=ok, ntts=2 * batch * steps, N=N, L=L, compute_floor_ms=floor_ms)


def compute_floor(torch, ringo, q, L, N, batch, x, stream, steps, warmup):
    """The compute floor of the step's own launches: the experiments build (libringo_exp.so, a
    second copy of the library loaded beside the product) with rg_set_probe(4) (L = 1: ntt16_pass)
    or (5) (L = 4: ntt256_pass) runs the same kernels with their HBM data loads and stores removed
    (butterflies, twiddle loads and LDS exchanges kept), timed the same way.  x is not written.
    The product library refuses the probe (include/ringo.h), so this is the only way to it."""
    import ctypes
    from ringo import _lib
    try:
        E = _lib.load(_lib.EXP_LIB_PATH)
    except RuntimeError:
        return None
    probe = 4 if L == 1 else 5
    ql = (ctypes.c_uint64 * L)(*[(q >> (64 * i)) & ((1 << 64) - 1) for i in range(L)])
    f, h = ctypes.c_void_p(), ctypes.c_void_p()
    p, s = ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(stream.cuda_stream)

    def pstep():
        assert E.rg_ntt_fwd_dev(h, p, p, batch, s) == 0 and E.rg_ntt_inv_dev(h, p, p, batch, s) == 0

    try:  # every handle created inside, destroyed in the finally whichever step failed
        if E.rg_field_create(L, ql, ctypes.byref(f)) != 0 or E.rg_ntt_create(f, N, 1, ctypes.byref(h)) != 0:
            return None
        if E.rg_set_probe(probe) != 0:
            return None
        for _ in range(max(2, warmup)):
            pstep()
        torch.cuda.synchronize()
        evp = Events(torch, stream)
        evp.start()
        for _ in range(steps):
            pstep()
        evp.stop()
        torch.cuda.synchronize()
        return evp.total_ms() / steps
    finally:
        E.rg_set_probe(0)
        if h.value:
            E.rg_ntt_destroy(h)
        if f.value:
            E.rg_field_destroy(f)


def jindo_bench(torch, ringo, dist, cfg_name, batch, steps, warmup, rank, world, eval_steps=0):
    """Device-resident batched commits (rg_jindo_commit_dev) at a BASELINE Jindo config.  At
    N > 1 the commit key is derived from the CRS on rank 0 and broadcast ONCE over RCCL (xGMI),
    device to device into every rank's prover (ringo.shard.broadcast_prover)."""
    from ringo import jindo
    from ringo.shard import broadcast_prover
    P = json.load(open(os.path.join(ROOT, "tests", "golden", "jindo_params.json")))[cfg_name]
    fq = int(P["field_q_hex"], 16)
    params = jindo.Parameters.from_dict(P, fq)
    dev = torch.device("cuda", torch.cuda.current_device())
    if world > 1:
        prv = broadcast_prover(params, dist, b"Jindo!")
    else:
        prv = jindo.NewProver(params, b"Jindo!")
    L, nv = params.L, params.rank
    sh = params.shapes(batch)
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)

    def elems(shape):  # uniform limbs, top limb < 2^(bits-2) so every value is < q
        t = torch.randint(-(2 ** 63), 2 ** 63 - 1, shape, dtype=torch.int64, device=dev, generator=g)
        top = fq >> (64 * (L - 1))
        t[..., L - 1] &= (1 << max(top.bit_length() - 2, 1)) - 1
        return t

    v = elems((batch, nv, L))
    last = elems(sh["last_row"])
    last[:, -1, :] = 0
    mask = elems(sh["mask"])
    en = torch.randint(-4000, 4000, sh["enc_noise"], dtype=torch.int64, device=dev, generator=g)
    mn = torch.randint(-40, 40, sh["mlwe_noise"], dtype=torch.int64, device=dev, generator=g)
    outs = {k: torch.empty(sh[k], dtype=torch.int64, device=dev) for k in ["incom", "enc", "mlwe_out", "com"]}
    stream = torch.cuda.current_stream()

    seeds = jindo.Seeds.derive(b"bench-%d" % rank)
    first = rank * batch  # this rank's commits in the job's sequence: disjoint sampler instances

    def step_sampled():  # Prover.Commit end to end: sampling + commit (rg_jindo_commit_sampled_dev)
        prv.commit_sampled_dev(batch, v, nv, seeds, first, outs["incom"], outs["enc"], outs["mlwe_out"], outs["com"],
                               stream)

    def step_injected():  # the deterministic part on pre-drawn randomness (rg_jindo_commit_dev)
        prv.commit_dev(batch, v, nv, last, mask, en, mn, outs["incom"], outs["enc"], outs["mlwe_out"], outs["com"],
                       stream)

    def timed(step, key):
        nw = prewarm(torch, step, 0.2)
        for _ in range(warmup):
            step()
        STEPS_DONE[key] = nw + warmup + steps
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        ev = Events(torch, stream)
        t0 = time.perf_counter()
        ev.start()
        for _ in range(steps):
            step()
        ev.stop()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        return time.perf_counter() - t0, ev.total_ms()

    def selfcheck(sampled):
        """Commit c = batch - 1 of the batch just timed, re-run alone (a 1-commit call at its own
        first_commit: the small-batch dispatch, 4-wave prep256, no 12-wave workgroups) must equal
        the batch's output for it, bit for bit.  Cheap, outside the timed region."""
        c = batch - 1
        sh1 = params.shapes(1)
        o1 = {k: torch.empty(sh1[k], dtype=torch.int64, device=dev) for k in outs}
        if sampled:
            prv.commit_sampled_dev(1, v[c:], nv, seeds, first + c, o1["incom"], o1["enc"], o1["mlwe_out"], o1["com"],
                                   stream)
        else:
            prv.commit_dev(1, v[c:], nv, last[c:], mask[c:], en[c:], mn[c:], o1["incom"], o1["enc"], o1["mlwe_out"],
                           o1["com"], stream)
        torch.cuda.synchronize()
        return all(torch.equal(o1[k][0], outs[k][c]) for k in outs)

    line = "j14" if cfg_name == "t14_b1" else "j16"
    wall_i, kern_i = timed(step_injected, line + "_injected")
    ok_i = selfcheck(False)
    wall, kern = timed(step_sampled, line)
    ok_s = selfcheck(True)
    nm = params.in_msis + params.mlwe
    opening_words = (params.dcmp * params.nqo * params.d + (params.cols + 1) * params.rows * params.nq * params.d +
                     (params.cols + 1) * nm * params.nq * params.d)
    # algorithmic bytes: v read once, the Opening and Commitment written once; the injected form
    # also reads the pre-drawn lastRow, mask and int64 noise
    out_words = opening_words + params.out_msis * params.nq * params.d
    bytes_per_commit = 8 * (nv * L + out_words)
    inj_words = (nv * L + params.cols * params.slots * L + params.rows * params.slots * L +
                 (params.cols + 1) * params.rows * params.d + (params.cols + 1) * nm * params.d)
    res = dict(wall_s=wall, kernel_ms=kern, commits=batch * steps, bytes_per_commit=bytes_per_commit,
               injected_wall_s=wall_i, injected_kernel_ms=kern_i, injected_bytes_per_commit=8 * (inj_words + out_words),
               selfcheck=ok_s, selfcheck_injected=ok_i)
    if eval_steps and P["batch"] > 1:
        res["eval"] = eval_bench(torch, prv, dist, P, params, batch, outs, eval_steps, g, dev, opening_words)
    return res


def eval_bench(torch, prv, dist, P, params, batch, outs, steps, g, dev, opening_words):
    """Prover.Evaluate's device work (prover.go:228-314) over this GPU's shard of the batch
    (`batch` openings just committed): batch combination, the cross-GPU all-reduce of the partial
    openBatches (RCCL; none at N = 1) and mod-q fold, partial evaluations, responses.  The
    challenges are injected device-generated residues (the SHAKE transcript stays host-side)."""
    from ringo.shard import allreduce_open_batch
    es = prv.eval_shapes()
    q, qo = params.q, params.qo

    def res(primes, shape):
        t = torch.empty(shape, dtype=torch.int64, device=dev)
        for l, qq in enumerate(primes):
            t[..., l, :] = torch.randint(0, qq, t[..., l, :].shape, dtype=torch.int64, device=dev, generator=g)
        return t

    bq, bo = res(q, (batch, len(q), params.d)), res(qo, (batch, len(qo), params.d))
    left, chals = res(q, (params.rows, len(q), params.d)), res(q, (params.cols, len(q), params.d))
    o = {k: torch.empty(es[k], dtype=torch.int64, device=dev) for k in es}
    stream = torch.cuda.current_stream()

    def step():
        prv.eval_batch_dev(batch, outs["incom"], outs["enc"], outs["mlwe_out"], bq, bo, o["ob_incom"], o["ob_enc"],
                           o["ob_mlwe"], stream)
        allreduce_open_batch(prv, dist, o["ob_incom"], o["ob_enc"], o["ob_mlwe"], stream)
        prv.eval_partial_dev(o["ob_enc"], left, o["partial"], stream)
        prv.eval_respond_dev(o["ob_enc"], o["ob_mlwe"], chals, o["pf_enc"], o["pf_mlwe"], stream)

    step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    ms = (time.perf_counter() - t0) * 1000.0 / steps
    return dict(ms=ms, openings_per_gpu=batch, bytes_read=8 * opening_words * batch)


def lib_sha256():
    p = os.path.join(ROOT, "ringo-snark_amd", "lib", "libringo.so")
    try:
        return hashlib.sha256(open(p, "rb").read()).hexdigest()
    except OSError:
        return None


def counters():
    """profiles/kernel_counters.json (tools/profile_bench.sh -> tools/kernel_counters.py): per
    bench line, the rocprofv3 PMC totals of that line's kernels over a profiled run and the steps
    that run executed.  Used only if it was measured on THIS libringo.so."""
    try:
        C = json.load(open(os.path.join(ROOT, "profiles", "kernel_counters.json")))
    except (OSError, ValueError):
        return None, "profiles/kernel_counters.json missing"
    if C.get("lib_sha256") != lib_sha256():
        return None, "stale: profiles/kernel_counters.json was measured on another libringo.so build"
    return C, C.get("source", "")


# the kernels of one step of each line (setup kernels and the Evaluate MACs excluded)
_DET = ("digits_kernel", "prep256_kernel", "mac3_kernel<", "mac3g_kernel<", "mac3h_kernel<", "mac_mfma_kernel<",
        "round_kernel")
_SAMP = ("cdt_noise_kernel", "cdt_tail_kernel", "cosac_noise_kernel", "cdt2_noise_kernel", "cosac2_noise_kernel",
         "mlwe_noise_kernel", "uniform_elems_kernel")
# l4: the 2^16 ntt256_pass launches only (the profiled run also executes the Buckler rank-2^15 ones)
LINE_KERNELS = {"ntt": ("ntt16_pass",), "l4": ("16, 0>(rg::Ntt256Args)",), "j14": _DET + _SAMP, "j16": _DET + _SAMP}


_PROBE_KERNEL = re.compile(r"ntt16_pass<.*, [1-9][0-9]*>\(")  # PROBE != 0: rg_set_probe's measurement variants


def line_counters(C, line, units_per_step, kernel_ms_per_step):
    """traffic (HBM bytes per unit) and the VALU issue block for one line, or None.  A Jindo
    line's profiled run executes injected steps (the deterministic kernels) and sampled steps
    (samplers + the same deterministic kernels): each kernel's sums are divided by the steps it
    ran in, so the figures are per sampled step = per Prover.Commit batch."""
    if C is None or line not in C.get("lines", {}):
        return None, None
    Lc = C["lines"][line]
    se = Lc.get("steps_executed") or {line: Lc["steps"]}
    mix = VALU_MIX.get("kernels", {}) if VALU_MIX.get("lib_sha256") == C.get("lib_sha256") else {}
    fetch = write = valu = cyc = 0.0
    for n, k in Lc["kernels"].items():
        if not any(p in n for p in LINE_KERNELS[line]) or _PROBE_KERNEL.search(n):
            continue  # (the compute-floor probe's launches run in the same process: not the step)
        st = se.get(line, Lc["steps"])
        if any(p in n for p in _DET):
            st += se.get(line + "_injected", 0)
        fetch += k.get("FETCH_SIZE", 0.0) / st  # KiB per step
        write += k.get("WRITE_SIZE", 0.0) / st
        v = k.get("SQ_INSTS_VALU", 0.0) / st
        valu += v
        cyc += v * mix.get(n, {}).get("mean_cycles", VALU_CYCLES)
    traffic = (2.0 * fetch + write) * 1024.0 / units_per_step  # gfx950: FETCH_SIZE counts half
    floor_ms = cyc / (SIMDS * CLOCK_HZ) * 1e3
    vb = {"insts_per_unit": valu / units_per_step, "cycles_per_inst": cyc / valu if valu else None, "simds": SIMDS,
          "clock_ghz": CLOCK_HZ / 1e9, "issue_floor_ms_per_step": floor_ms,
          "frac": floor_ms / kernel_ms_per_step if kernel_ms_per_step else None,
          "cycle_model": ("per kernel: SQ_INSTS_VALU x the mean measured issue cost of its static VALU mix "
                          "(profiles/valu_mix.json, tools/valu_mix.py; full-rate ops 2.4, half-rate 4.5, "
                          "transcendental 9 cycles per wave64 instruction per SIMD)") if mix else
                         f"uniform {VALU_CYCLES} cycles per instruction (no valu_mix.json for this library)",
          "note": "issue floor = sum over kernels of VALU instructions x cycles / (SIMDs x clock); frac = floor / "
                  "measured time.  Static per-class costs ignore dual issue of independent full/half-rate pairs, "
                  "so this floor can sit above a kernel's true compute floor; where measured, "
                  "compute_floor_ms_per_step (the kernel with its HBM traffic removed) is the direct figure"}
    return traffic, vb


def vec_mul_bench(torch, ringo, q, L, n, steps, seed):
    """configs[3]'s pointwise product: MulTo of two NTT-domain polys (base_op.go:133-142) over n
    elements, device-resident; bytes = 2 reads + 1 write of 8L B per element."""
    from ringo.bigpoly import vec_dev
    dev = torch.device("cuda", torch.cuda.current_device())
    F = ringo.Field(q)
    a = torch.from_numpy(uniform_elems(q, L, n, seed).view(np.int64).reshape(-1)).to(dev)
    b = torch.from_numpy(uniform_elems(q, L, n, seed + 1).view(np.int64).reshape(-1)).to(dev)
    out = torch.empty_like(a)
    stream = torch.cuda.current_stream()

    def step():
        vec_dev(F, "mul", out, a, b, n, stream)

    prewarm(torch, step, 0.1)
    torch.cuda.synchronize()
    ev = Events(torch, stream)
    ev.start()
    for _ in range(steps):
        step()
    ev.stop()
    torch.cuda.synchronize()
    ms = ev.total_ms() / steps
    return dict(elems_per_s=n / (ms * 1e-3), achieved_GBs=3 * 8 * L * n / (ms * 1e-3) / 1e9, ms=ms)


def polyops_bench(torch, ringo, q, L, rank, batch, steps, seed):
    """The remaining bigpoly operators at the configs[3] shape (q255, N = 2^16), device-resident:
    AutTo in the NTT domain (cyclotomic.go:70-86) and QuoRemByVanishing by X^(N/2) - 1
    (cyclic.go:18-37) over `batch` polynomials, Poly.Evaluate (poly.go:64-76) of one.  Bytes:
    one read + one write (Aut), one read + two writes (QuoRem) of 8L B per coefficient."""
    from ringo._lib import check, lib
    dev = torch.device("cuda", torch.cuda.current_device())
    F = ringo.Field(q)
    x = torch.from_numpy(uniform_elems(q, L, batch * rank, seed).view(np.int64).reshape(-1)).to(dev)
    o1, o2 = torch.empty_like(x), torch.empty_like(x)
    xe = x[:L].clone()
    ev_out = torch.empty(L, dtype=torch.int64, device=dev)
    scratch = torch.empty(max(1, lib().rg_poly_evaluate_scratch_bytes(F.h, rank) // 8), dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream()
    sp = st.cuda_stream
    res = {}
    for name, fn, nbytes in (
            ("aut_ntt", lambda: check(lib().rg_poly_aut_dev(F.h, rank, 5, 1, o1.data_ptr(), x.data_ptr(), batch, sp)),
             2 * 8 * L * rank * batch),
            ("quorem_vanishing", lambda: check(lib().rg_poly_quorem_vanishing_dev(
                F.h, rank, rank // 2, o1.data_ptr(), o2.data_ptr(), x.data_ptr(), batch, sp)), 3 * 8 * L * rank * batch),
            ("evaluate", lambda: check(lib().rg_poly_evaluate_dev(F.h, x.data_ptr(), rank, xe.data_ptr(),
                                                                  ev_out.data_ptr(), scratch.data_ptr(), sp)),
             8 * L * rank)):
        fn()
        torch.cuda.synchronize()
        ev = Events(torch, st)
        ev.start()
        for _ in range(steps):
            fn()
        ev.stop()
        torch.cuda.synchronize()
        ms = ev.total_ms() / steps
        res[name] = {"ms": ms, "achieved_GBs": nbytes / (ms * 1e-3) / 1e9}
    res["shape"] = "N=2^16, q255 (L=4); aut/quorem over %d polys, evaluate of one" % batch
    res["buckler"] = buckler_bench(torch, ringo, F, q, L, rank, batch, steps, seed)
    return res


def buckler_bench(torch, ringo, F, q, L, emb, batch, steps, seed):
    """The Buckler prover's per-witness device work at embRank = N (q255): RandEncode of `batch`
    witnesses of rank N/2 (buckler/encoder.go:50-54: batched cyclic InvNTT + embedding; bytes =
    read rank + write embRank elements per witness) and the fused evalCircuit of one constraint
    a*b - c + pw*d over 4 witnesses + 1 public witness (prover.go:355-379; bytes = 5 polys read +
    1 written)."""
    from ringo import buckler
    dev = torch.device("cuda", torch.cuda.current_device())
    rank = emb // 2
    enc = buckler.NewEncoder(F, rank, emb)
    v = torch.from_numpy(uniform_elems(q, L, batch * rank, seed + 1).view(np.int64).reshape(-1)).to(dev)
    r = torch.from_numpy(uniform_elems(q, L, batch, seed + 2).view(np.int64).reshape(-1)).to(dev)
    out = torch.empty(batch * emb * L, dtype=torch.int64, device=dev)
    scr = torch.empty(max(1, enc.scratch_bytes(batch) // 8), dtype=torch.int64, device=dev)
    c = buckler.ArithmeticConstraint(F)
    c.AddTerm(None, 0, 1)
    c.SubTerm(None, 2)
    c.AddTerm(0, 3)
    circ = buckler.Circuit(F, [c])
    w = torch.from_numpy(uniform_elems(q, L, 4 * emb, seed + 3).view(np.int64).reshape(-1)).to(dev)
    pw = torch.from_numpy(uniform_elems(q, L, emb, seed + 4).view(np.int64).reshape(-1)).to(dev)
    bc = w[:L].clone()
    eo = torch.empty(emb * L, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream()
    res = {}
    for name, fn, nbytes in (
            ("rand_encode", lambda: enc.encode_dev(out, v, batch, d_rand=r, d_scratch=scr, stream=st),
             8 * L * (rank + emb) * batch),
            ("eval_circuit", lambda: circ.eval_dev(emb, bc, w, 4, pw, 1, eo, stream=st), 6 * 8 * L * emb)):
        fn()
        torch.cuda.synchronize()
        ev = Events(torch, st)
        ev.start()
        for _ in range(steps):
            fn()
        ev.stop()
        torch.cuda.synchronize()
        ms = ev.total_ms() / steps
        res[name] = {"ms": ms, "achieved_GBs": nbytes / (ms * 1e-3) / 1e9}
    res["shape"] = "q255 (L=4), embRank 2^16: RandEncode of %d rank-2^15 witnesses; evalCircuit a*b - c + pw*d" % batch
    return res


def cpu_baseline(q, L, logn, seconds):
    """C restatement (oracle/liboracle.so) fwd+inv on this host: bounded sample, all threads
    the OpenMP runtime gives it (OMP_NUM_THREADS)."""
    import coracle as co
    cf = co.CField(q)
    N = 1 << logn
    tw, twi, ninv = cf.tables(N)
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    chunk = max(threads, 1)
    a = uniform_elems(q, L, chunk * N, 0x52494E47).reshape(chunk, N, L)
    done = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        y = cf.ntt_fwd(a, tw)
        cf.ntt_inv(y, twi, ninv)
        done += 2 * chunk
    el = time.perf_counter() - t0
    return dict(value=done / el, unit="NTT/s", cores=threads, kind="port",
                sample=f"{done} transforms (fwd+inv pairs of {chunk} polys, N=2^{logn}, L={L}) in {el:.1f} s "
                       "by oracle/oracle.c (C restatement of ntt.go; Go toolchain absent on this host)")


def cpu_baseline_jindo(seconds):
    """The C restatement's whole Commit (oracle.c of_jindo_commit: encode, MLWE, MACs, rounding,
    outer commit; injected randomness like the GPU line) at the configs[2] shape, one commit per
    thread at a time (ctypes drops the GIL), on a bounded sample."""
    from concurrent.futures import ThreadPoolExecutor
    import coracle as co
    P = json.load(open(os.path.join(ROOT, "tests", "golden", "jindo_params.json")))["t14_b1"]
    q = int(P["field_q_hex"], 16)
    L = (q.bit_length() + 63) // 64
    cj = co.CJindo(P, q)
    rng = np.random.default_rng(5)
    nq, nqo, nm, d = len(P["q"]), len(P["qo"]), P["in_msis"] + P["mlwe"], P["d"]
    ck = (rng.integers(0, P["q"][0], size=(P["in_msis"], P["rows"], nq, d), dtype=np.uint64),
          rng.integers(0, P["q"][0], size=(P["in_msis"], P["mlwe"], nq, d), dtype=np.uint64),
          rng.integers(0, P["qo"][0], size=(P["out_msis"], P["in_com_dcmp_len"], nqo, d), dtype=np.uint64))
    v = uniform_elems(q, L, P["rank"], 3)
    last = uniform_elems(q, L, P["cols"] * P["slots"], 4)
    last[-1] = 0
    mask = uniform_elems(q, L, P["rows"] * P["slots"], 5).reshape(P["rows"], P["slots"], L)
    en = rng.integers(-4000, 4000, size=(P["cols"] + 1, P["rows"], d), dtype=np.int64)
    mn = rng.integers(-40, 40, size=(P["cols"] + 1, nm, d), dtype=np.int64)
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    t0 = time.perf_counter()

    def worker(_):
        n = 0
        while time.perf_counter() - t0 < seconds:
            cj.commit(ck[0], ck[1], ck[2], v, last, mask, en, mn)
            n += 1
        return n

    with ThreadPoolExecutor(threads) as ex:
        done = sum(ex.map(worker, range(threads)))
    el = time.perf_counter() - t0
    return dict(value=done / el, unit="commits/s", cores=threads, kind="port",
                sample=f"{done} commits (configs[2] shape, targetN 2^14, injected randomness) in {el:.1f} s by "
                       "oracle/oracle.c of_jindo_commit (C restatement of prover.go/encoder.go/rns.go)")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(args):
    """--gpus N without torch.distributed.run around us: start it as a CHILD process (one rank per
    GPU, rendezvous on 127.0.0.1) before anything touches the GPU, and exit with its code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def plumbing(args, world, rank):
    """--plumbing: the launcher, barrier and max-over-ranks timing on gloo with a trivial host step
    (no GPU, no libringo).  Proves the rank count the driver's N-GPU run will get."""
    import torch
    import torch.distributed as tdist
    if world > 1:
        tdist.init_process_group("gloo")
    x = np.arange(1 << 16, dtype=np.uint64)

    def step():
        np.bitwise_xor(x, np.uint64(rank + 1), out=x)

    for _ in range(args.warmup):
        step()
    if world > 1:
        tdist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        tdist.barrier()
    ms = (time.perf_counter() - t0) * 1e3 / max(args.steps, 1)
    ranks = [rank]
    if world > 1:
        t = torch.tensor([ms], dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        ms = float(t[0])
        got = [None] * world
        tdist.all_gather_object(got, rank)
        ranks = sorted(got)
    if rank == 0:
        print(json.dumps({"metric": "plumbing", "value": world / (ms / 1e3), "unit": "steps/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms, "ranks": ranks,
                          "plumbing": True}), flush=True)
    if world > 1:
        tdist.destroy_process_group()
    return 0


def reduce_max(torch, dist, *vals):
    if dist is None:
        return vals if len(vals) > 1 else vals[0]
    t = torch.tensor(list(vals), dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    out = tuple(float(x) for x in t)
    return out if len(out) > 1 else out[0]


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        return launch(args)
    world = int(world_env or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    if args.plumbing:
        return plumbing(args, world, rank)
    if args.no_prewarm:
        PREWARM[0] = False
    import torch

    ngpu = torch.cuda.device_count()  # counts devices without initialising the GPU on this image
    # RINGO_BENCH_REHEARSAL=1 (tests/tools only, never a measurement): every rank on cuda:0 and the
    # collectives over gloo, so the N > 1 code path (broadcast of the commit key, the Evaluate
    # all-reduce, barriers and max-over-ranks timing, the self-checks) runs on a one-GPU box
    rehearsal = os.environ.get("RINGO_BENCH_REHEARSAL") == "1" and world > 1
    if rehearsal:
        local = 0
    if world > ngpu and not rehearsal or local >= ngpu:
        print(f"bench.py: WORLD_SIZE={world} (LOCAL_RANK={local}) but {ngpu} visible GPU(s): one rank per GPU",
              file=sys.stderr)
        return 2
    dist = None
    if world > 1:
        import torch.distributed as tdist
        if rehearsal:
            tdist.init_process_group("gloo")
        else:
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dist = tdist
    import ringo
    from ringo.shard import bind_device

    bind_device(local, world)  # LOCAL_RANK -> torch and libringo's current device, checked
    C, csrc = counters()
    N = 1 << args.logn
    out = {}
    extra = set() if args.no_extra else set(x for x in args.extra.split(",") if x)
    if not args.no_ntt:
        r = ntt_step_bench(torch, ringo, dist, P63, 1, args.batch, args.logn, args.steps, args.warmup,
                           0x52494E47 + rank)
        ms_step, kern_ms = reduce_max(torch, dist, r["wall_s"] * 1000.0 / args.steps, r["kernel_ms"])
        ok = r["ok"]
        if dist is not None:
            okt = torch.tensor([0 if r["ok"] else 1], device="cuda")
            dist.all_reduce(okt)
            ok = int(okt.item()) == 0
        bytes_per_ntt = 2 * N * 8
        achieved = bytes_per_ntt * r["ntts"] / (kern_ms / 1000.0) / 1e9
        traffic, vb = line_counters(C, "ntt", 2 * args.batch, kern_ms / args.steps)
        cf = r.get("compute_floor_ms")
        if cf is not None:
            cf = reduce_max(torch, dist, cf)
            vb = dict(vb or {})
            vb.update({"compute_floor_ms_per_step": cf, "compute_frac": cf / (kern_ms / args.steps),
                       "compute_floor_note": "the same ntt16_pass launches with their HBM data loads and stores "
                                             "removed (experiments build libringo_exp.so, rg_set_probe(4): "
                                             "butterflies, twiddle loads, LDS exchanges kept), HIP-event timed on "
                                             "the launch stream; compute_frac = that time / the production step's "
                                             "kernel time"})
        out.update({
            "metric": "NTTs/sec (fwd+inv negacyclic, degree 2^16, 63-bit prime, batch 1024/GPU)",
            "value": world * 2 * args.batch / (ms_step / 1000.0),
            "unit": "NTT/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (SplitMix64 seed 0x52494E47, uniform residues mod p)",
            "config": {"workload": "configs[1]: fwd+inv negacyclic NTT, N=2^16, p=47104^4+1 (63-bit), "
                                   f"batch {args.batch} polys per GPU, HBM-resident",
                       "rank": N, "field_bits": 63, "batch_per_gpu": args.batch, "parallelism": f"replicas x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "ntt16_pass COL + ROW launches (two 8-stage passes per transform); achieved = "
                                   "algorithmic bytes (1 read + 1 write of N*8 B per transform) / HIP-event time of "
                                   "the timed region on the launch stream",
                         "bytes_per_unit": bytes_per_ntt,
                         "traffic_note": ("HBM bytes per transform, rocprofv3 PMC (2 x FETCH_SIZE + WRITE_SIZE) of "
                                          "this libringo.so: " + csrc) if traffic else csrc,
                         "valu": vb},
            "selfcheck_fwd_inv_identity": ok,
        })
    if "l4" in extra:
        st4 = max(2, args.steps // 2)
        r4 = ntt_step_bench(torch, ringo, dist, Q255, 4, 64, args.logn, st4, 1, 7 + rank)
        ms4, k4 = reduce_max(torch, dist, r4["wall_s"] * 1000.0 / st4, r4["kernel_ms"])
        vm = vec_mul_bench(torch, ringo, Q255, 4, 64 * N, 10, 11 + rank)
        tr4, vb4 = line_counters(C, "l4", 128, k4 / st4)
        cf4 = r4.get("compute_floor_ms")
        if cf4 is not None:
            cf4 = reduce_max(torch, dist, cf4)
            vb4 = dict(vb4 or {})
            vb4.update({"compute_floor_ms_per_step": cf4, "compute_frac": cf4 / (k4 / st4),
                        "compute_floor_note": "the same ntt256_pass launches without HBM data movement "
                                              "(libringo_exp.so, rg_set_probe(5)), HIP-event timed"})
        out["l4_ntt"] = {"value": world * 2 * 64 / (ms4 / 1000.0), "unit": "NTT/s",
                         "config": "configs[3]: fwd+inv negacyclic NTT, N=2^16, 255-bit Jindo prime, batch 64/GPU",
                         "kernel": "ntt256_pass (4-limb Montgomery, q = 1 mod 2^64; VALU-bound)",
                         "achieved_GBs": 2 * N * 32 * r4["ntts"] / (k4 / 1000.0) / 1e9,
                         "traffic_per_ntt": tr4, "valu": vb4,
                         "selfcheck_fwd_inv_identity": r4["ok"],
                         "pointwise_mul": {"unit": "elements/s", "value": world * vm["elems_per_s"],
                                           "achieved_GBs": vm["achieved_GBs"], "elements": 64 * N},
                         "bigpoly_ops": polyops_bench(torch, ringo, Q255, 4, N, 64, 10, 13 + rank)}
    if "wide" in extra:
        fields = json.load(open(os.path.join(ROOT, "tests", "golden", "fields.json")))
        for fname, bw in (("zp440", 32), ("zp880", 16)):
            qw = int(fields[fname]["q_hex"], 16)
            Lw = (qw.bit_length() + 63) // 64
            stw = max(2, args.steps // 4)
            rw = ntt_step_bench(torch, ringo, dist, qw, Lw, bw, args.logn, stw, 1, 17 + rank)
            msw, kw = reduce_max(torch, dist, rw["wall_s"] * 1000.0 / stw, rw["kernel_ms"])
            out["wide_ntt_" + fname] = {
                "value": world * 2 * bw / (msw / 1000.0), "unit": "NTT/s",
                "config": f"Buckler wide field {fname} ({qw.bit_length()}-bit, L={Lw}): fwd+inv negacyclic NTT, "
                          f"N=2^{args.logn}, batch {bw}/GPU (buckler_test.go:163-222 runs zp880 at LogN 15)",
                "achieved_GBs": 2 * N * 8 * Lw * rw["ntts"] / (kw / 1000.0) / 1e9,
                "ms_per_step": msw, "selfcheck_fwd_inv_identity": rw["ok"]}
    for cfg, jb, key in (("t14_b1", args.j14_batch, "j14"), ("t16_b4096", args.j16_batch, "j16")):
        if key not in extra:
            continue
        js = max(2, args.steps // 2)
        jr = jindo_bench(torch, ringo, dist, cfg, jb, js, 1, rank, world, eval_steps=js)
        jms, jk, jmi, jki, jbad = reduce_max(torch, dist, jr["wall_s"] * 1000.0 / js, jr["kernel_ms"],
                                             jr["injected_wall_s"] * 1000.0 / js, jr["injected_kernel_ms"],
                                             0.0 if jr["selfcheck"] and jr["selfcheck_injected"] else 1.0)
        trj, vbj = line_counters(C, key, jb, jk / js)
        name = "jindo_commit" if cfg == "t14_b1" else "jindo_commit_2e16"
        out[name] = {"value": world * jb / (jms / 1000.0), "unit": "commits/s",
                     "config": ("configs[2]: Jindo commit, targetN 2^14 (jindo_test params), q255" if cfg == "t14_b1"
                                else "configs[4]: Jindo commit, NewParameters(2^16, 4096), q255, "
                                     f"{jb} commits per GPU ({world * jb} in the job)"),
                     "batch_per_gpu": jb, "ms_per_batch": jms, "n_gpus": world,
                     "achieved_GBs": jr["bytes_per_commit"] * jr["commits"] / (jk / 1000.0) / 1e9,
                     "bytes_per_commit": jr["bytes_per_commit"], "traffic_per_commit": trj, "valu": vbj,
                     "selfcheck_single_commit_rerun": jbad == 0.0,
                     "selfcheck_note": "on every rank, commit batch-1 of the timed batch re-run alone (1-commit "
                                       "call at its first_commit: the small-batch kernels) equals the batch's output "
                                       "bit for bit, for both the sampled and the injected path",
                     "randomness": "sampled on the device inside the timed step (AES-256-CTR UniformSampler "
                                   "instances, TwinCDT / COSAC / rounded Gaussian, MustSetRandom): Prover.Commit end "
                                   "to end (rg_jindo_commit_sampled_dev)",
                     "injected": {"value": world * jb / (jmi / 1000.0), "unit": "commits/s", "ms_per_batch": jmi,
                                  "achieved_GBs": jr["injected_bytes_per_commit"] * jr["commits"] / (jki / 1000.0) / 1e9,
                                  "note": "the deterministic part only (rg_jindo_commit_dev) on pre-drawn randomness "
                                          "read from HBM"}}
        if "eval" in jr:
            ems = reduce_max(torch, dist, jr["eval"]["ms"])
            out["jindo_evaluate_2e16"] = {
                "value": world * jb / (ems / 1000.0), "unit": "openings/s",
                "config": "configs[4] shape: Prover.Evaluate device work over the batch (%d openings per GPU): "
                          "batch combination + RCCL all-reduce of partial openBatches + partial evaluations + "
                          "responses; challenges injected" % jb,
                "ms_per_evaluate": ems, "achieved_GBs": jr["eval"]["bytes_read"] / (ems / 1000.0) / 1e9}
    if rank == 0 and world == 1 and not args.no_cpu:
        if not args.no_ntt:
            out["cpu_baseline"] = cpu_baseline(P63, 1, args.logn, args.cpu_seconds)
        if "j14" in extra:
            out["cpu_baseline_jindo_commit"] = cpu_baseline_jindo(args.cpu_seconds)
    if rehearsal:
        out["rehearsal"] = "RINGO_BENCH_REHEARSAL: %d ranks sharing cuda:0 over gloo; not a measurement" % world
    out["steps_executed"] = dict(STEPS_DONE)
    out["libringo_sha256"] = lib_sha256()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
