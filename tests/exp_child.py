"""Test helper run as a child process on the experiments build (libringo_exp.so): the kernel
switches (RINGO_*) are honoured only there, and one process loads one libringo, so a test that
compares kernel variants runs each variant here and reads back an .npz.  Never imported by the
product.

  python tests/exp_child.py mac <mode> <out.npz> <shape>...   Commit with RINGO_JINDO_MAC=<mode>
  python tests/exp_child.py uni <tries> <out.npz> <name> <B> <first>   sample_dev's lastRow / mask
      with RINGO_JINDO_UNI_TRIES=<tries> (uniform_whole_kernel gives up early: the fix-up path)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ringo-snark_amd"), os.path.join(ROOT, "oracle"), ROOT]
os.environ["RINGO_LIB"] = os.path.join(ROOT, "ringo-snark_amd", "lib", "libringo_exp.so")

import numpy as np  # noqa: E402


def mac(mode, out, shapes):
    import json

    from ringo import jindo
    from tests.jindo_util import make_randomness, make_v
    os.environ["RINGO_JINDO_MAC"] = mode
    P_all = json.load(open(os.path.join(ROOT, "tests", "golden", "jindo_params.json")))
    res = {}
    for sh in shapes:
        name, nv = sh.split(":")
        P = P_all[name]
        q = int(P["field_q_hex"], 16)
        params = jindo.Parameters.from_dict(P, q)
        prv = jindo.NewProver(params, b"Jindo!")
        com, op = prv.Commit(make_v(q, int(nv), seed=5), jindo.Randomness(**make_randomness(P, q, seed=9)))
        res[name + "/incom"] = op.InCommit
        res[name + "/com"] = com.Value
        res[name + "/kinds"] = np.array(prv.mac_kinds())
    np.savez(out, **res)


def uni(tries, out, name, B, first):
    import json

    import torch

    from ringo import jindo
    from tests.jindo_util import make_v
    os.environ["RINGO_JINDO_UNI_TRIES"] = tries
    P = json.load(open(os.path.join(ROOT, "tests", "golden", "jindo_params.json")))[name]
    q = int(P["field_q_hex"], 16)
    params = jindo.Parameters.from_dict(P, q)
    prv = jindo.NewProver(params, b"Jindo!")
    nv = P["rank"]
    v = np.stack([make_v(q, nv, seed=21 + b) for b in range(B)])
    sh = params.shapes(B)
    o = {k: torch.zeros(sh[k], dtype=torch.int64, device="cuda") for k in ("last_row", "mask", "enc_noise", "mlwe_noise")}
    dv = torch.from_numpy(np.ascontiguousarray(v).view(np.int64)).to("cuda")
    prv.sample_dev(B, dv, nv, jindo.Seeds.derive(b"uni-" + name.encode()), first, o["last_row"], o["mask"],
                   o["enc_noise"], o["mlwe_noise"])
    torch.cuda.synchronize()
    np.savez(out, last_row=o["last_row"].cpu().numpy(), mask=o["mask"].cpu().numpy())


if __name__ == "__main__":
    if sys.argv[1] == "mac":
        mac(sys.argv[2], sys.argv[3], sys.argv[4:])
    elif sys.argv[1] == "uni":
        uni(sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5]), int(sys.argv[6]))
    else:
        raise SystemExit("unknown mode " + sys.argv[1])
