"""Test helper run as a child process on the experiments build (libringo_exp.so): the kernel
switches (RINGO_*) are honoured only there, and one process loads one libringo, so a test that
compares kernel variants runs each variant here and reads back an .npz.  Never imported by the
product.

  python tests/exp_child.py mac <mode> <out.npz> <shape>...   Commit with RINGO_JINDO_MAC=<mode>
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


if __name__ == "__main__":
    if sys.argv[1] == "mac":
        mac(sys.argv[2], sys.argv[3], sys.argv[4:])
    else:
        raise SystemExit("unknown mode " + sys.argv[1])
