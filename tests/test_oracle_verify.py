"""CPU: the C oracle's Verifier.Verify (oracle.c of_jindo_verify, restating jindo/verifier.go:50-282)
pinned the way the reference pins it -- TestJindo's completeness (jindo_test.go:26-52): an honest
Commit + Evaluate at the jindo_test sizes (targetN 2^10, batch 1 and 8) verifies -- plus the
checks each failure mode must trip: a changed response word (inner norm / consistency), a changed
inner-commitment word (outer norm), a wrong evaluation (eval), and the norm decision against
exact integer square roots."""
import json
import math
import os

import numpy as np
import pytest

from tests.jindo_proto import honest_proof, oracle_verify, random_ck

HERE = os.path.dirname(os.path.abspath(__file__))
PARAMS = json.load(open(os.path.join(HERE, "golden", "jindo_params.json")))


# jindo_test sizes, plus the zp package's widest and narrowest fields as Jindo fields
@pytest.fixture(scope="module", params=["t10_b1", "t10_b8", "p63_t10_b2", "zp880_t10_b1"])
def proof(request):
    name = request.param
    P = PARAMS[name]
    fq = int(P["field_q_hex"], 16)
    ck = random_ck(P, 7)
    return name, P, fq, ck, honest_proof(P, fq, ck, seed=11)


def test_honest_proof_verifies(proof):
    name, P, fq, ck, pr = proof
    r = oracle_verify(P, fq, ck, pr)
    assert r["flags"] == [True, True, True, True], (name, r["flags"])
    assert r["ok"]
    # the norms are well inside the bounds (sanity of the restated parameters)
    assert math.isqrt(r["outer_sq"]) < P["in_com_dcmp_two_nm"]
    assert math.isqrt(r["inner_sq"]) < P["res_two_nm"]


@pytest.mark.parametrize("what", ["pf_enc", "pf_incom", "y", "pf_partial"])
def test_tampered_proof_rejected(proof, what):
    name, P, fq, ck, pr = proof
    bad = dict(pr)
    bad[what] = pr[what].copy()
    flat = bad[what].reshape(-1)
    i = min(3, flat.size - 1)
    flat[i] = (int(flat[i]) + 1) % (1 << 62)
    r = oracle_verify(P, fq, ck, bad)
    assert not r["ok"], (name, what)
    assert not all(r["flags"]), (name, what, r["flags"])
    # the check that must catch it, at the jindo_test sizes.  (At zp880, exp 64, ChallengeBound is
    # min(b, 2^(120/64)) / 2 = 1 (params.go:358-360), so encodeChallengeTo (utils.go:21-46) gives
    # all-zero challenges and a changed Partial word passes verifyConsistency; verifyEval rejects it.)
    if name.startswith("t10_"):
        want_fail = {"pf_enc": 1, "pf_incom": 0, "y": 3, "pf_partial": 2}[what]
        assert not r["flags"][want_fail], (name, what, r["flags"])


def test_norm_decision_is_exact():
    """norm_below(S, nm) == (Float64(isqrt(S)) < nm), Go's big.Int Sqrt + Float64 (round to nearest
    even), at and around the float boundaries, small and above 2^53, 2^64 and 2^128."""
    import coracle as co
    rng = np.random.default_rng(3)
    cases = []
    for nm in [1.0, 2.5, 1e6 + 0.5, 2.0 ** 53, 2.0 ** 53 + 2, 9.3e15, 2.0 ** 60, 1.6e17, 2.0 ** 64, 3.0e22,
               2.0 ** 100, 1.9e40, 7.49e28]:
        for nmv in (nm, np.nextafter(nm, 0), np.nextafter(nm, np.inf)):
            t = int(nmv)
            for T in {max(t + dd, 0) for dd in (-2, -1, 0, 1, 2)} | {int(float(t) * 0.9999999999999999)}:
                for s in (T * T, T * T + 1, max(T * T - 1, 0), (T + 1) ** 2 - 1):
                    cases.append((s, float(nmv)))
    for _ in range(200):
        b = int(rng.integers(1, 400))
        s = int.from_bytes(rng.bytes(64), "little") >> (512 - b)
        cases.append((s, float(math.isqrt(s)) * float(rng.uniform(0.999, 1.001))))
    for s, nm in cases:
        if s >> 640:
            continue
        assert co.norm_below(s, nm) == (float(math.isqrt(s)) < nm), (s, nm)
