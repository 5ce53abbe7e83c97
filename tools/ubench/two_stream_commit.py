"""Do two commit batches in flight (alternating two streams, separate outputs and scratch) beat
one stream?  Sampled commits at the bench shapes; prints commits/s for 1 and 2 streams."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ringo-snark_amd"))
from ringo import jindo  # noqa: E402


def run(cfg, batch, steps):
    P = json.load(open(os.path.join(ROOT, "tests", "golden", "jindo_params.json")))[cfg]
    fq = int(P["field_q_hex"], 16)
    params = jindo.Parameters.from_dict(P, fq)
    prv = jindo.NewProver(params, b"Jindo!")
    L, nv = params.L, params.rank
    sh = params.shapes(batch)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    v = torch.randint(0, 2 ** 62, (batch, nv, L), dtype=torch.int64, device="cuda", generator=g)
    v[..., L - 1] &= (1 << 40) - 1
    seeds = jindo.Seeds.derive(b"two-stream")
    outs = [{k: torch.empty(sh[k], dtype=torch.int64, device="cuda") for k in ["incom", "enc", "mlwe_out", "com"]}
            for _ in range(2)]
    sts = [torch.cuda.Stream(), torch.cuda.Stream()]
    res = {}
    for ns in (1, 2, 1, 2):
        for i in range(3):  # warm (scratch per stream)
            s = i % ns
            o = outs[s]
            prv.commit_sampled_dev(batch, v, nv, seeds, i * batch, o["incom"], o["enc"], o["mlwe_out"], o["com"], sts[s])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            s = i % ns
            o = outs[s]
            prv.commit_sampled_dev(batch, v, nv, seeds, i * batch, o["incom"], o["enc"], o["mlwe_out"], o["com"], sts[s])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res.setdefault(ns, []).append(round(steps * batch / dt))
    print(cfg, batch, "commits/s by streams:", res, flush=True)


if __name__ == "__main__":
    torch.cuda.set_device(0)
    run("t14_b1", 256, 40)
    run("t16_b4096", 512, 12)
