"""Does splitting one GPU's commit batch over S concurrent HIP streams (the library keeps scratch
per stream) beat one stream?  Times rg_jindo_commit_sampled_dev of `batch` commits at a Jindo
config as S slices of batch/S on S torch streams, S = 1, 2, 4.  usage: python tools/stream_overlap.py [cfg] [batch]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ringo-snark_amd"))
import torch  # noqa: E402

from ringo import jindo  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "t16_b4096"
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 512
P = json.load(open(os.path.join(ROOT, "tests", "golden", "jindo_params.json")))[cfg]
fq = int(P["field_q_hex"], 16)
params = jindo.Parameters.from_dict(P, fq)
prv = jindo.NewProver(params, b"Jindo!")
dev = torch.device("cuda", 0)
L, nv = params.L, params.rank
sh = params.shapes(batch)
v = torch.randint(0, 2 ** 40, (batch, nv, L), dtype=torch.int64, device=dev)
outs = {k: torch.empty(sh[k], dtype=torch.int64, device=dev) for k in ["incom", "enc", "mlwe_out", "com"]}
seeds = jindo.Seeds.derive(b"overlap")
for S in (1, 2, 4, 1):
    streams = [torch.cuda.Stream() for _ in range(S)]
    part = batch // S

    def step():
        for i, st in enumerate(streams):
            sl = slice(i * part, (i + 1) * part)
            prv.commit_sampled_dev(part, v[sl], nv, seeds, i * part, outs["incom"][sl], outs["enc"][sl],
                                   outs["mlwe_out"][sl], outs["com"][sl], st)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    n = 8
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1000 / n
    print(json.dumps({"streams": S, "ms_per_batch": ms, "commits_per_s": batch / ms * 1000}), flush=True)
