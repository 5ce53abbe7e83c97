"""GPU parity of the exact commit paths bench.py times, at the bench's own batches: configs[2]
(t14_b1, 256 commits per step) and configs[4] (t16_b4096, 512 commits per GPU per step).

At 512 commits the configs[4] encode prep is 512 * 9 * 513 = 2.36 M jobs, past the 2^20 at which
prep_launch (csrc/jindo.hip) takes the 12-wave prep256_kernel<2, true, 12>; smaller batches (every
other test) take the 4-wave form.  So these tests pin the kernels the jindo_commit /
jindo_commit_2e16 lines actually run:

  * rg_jindo_commit_sampled_dev (the sampled line: the three-stream DAG of MustSetRandom, digits,
    COSAC centres, cdt2, cosac2, MLWE samplers, prep256 and the core) at the bench batch, commits
    0, B/2 and B-1 against the C oracle end to end (CJindo.sample at that commit's first_commit,
    then CJindo.commit: Encode, MLWE, InCommit and the Commitment, bit for bit);
  * every commit of that batch against the same commits run in chunks of 64 (below the 12-wave
    threshold, each chunk at its own first_commit offset);
  * rg_jindo_commit_dev (the injected line) on rg_jindo_sample_dev's draws of the whole batch: equal
    to the sampled path on every commit.

Reference: jindo/prover.go:45-202 (Commit), jindo/encoder.go:149-201 (randEncodeTo),
math/csprng (the samplers).  Oracle: oracle/oracle.c, bit-exact."""
import json
import os

import numpy as np
import pytest

import coracle as co
import pyref
from ringo import jindo
from tests.jindo_util import make_v

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
PARAMS = json.load(open(os.path.join(HERE, "golden", "jindo_params.json")))
OUT_KEYS = ("incom", "enc", "mlwe_out", "com")
RND_KEYS = ("last_row", "mask", "enc_noise", "mlwe_noise")


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to("cuda")


def _h(t):
    return t.cpu().numpy().view(np.uint64)


def _setup(name, B):
    """Prover, a device v batch whose checked commits (0, B/2, B-1) each have their own v and the
    rest share a filler, and the checked indices."""
    import torch
    P = PARAMS[name]
    q = int(P["field_q_hex"], 16)
    params = jindo.Parameters.from_dict(P, q)
    prv = jindo.NewProver(params, b"Jindo!")
    nv = P["rank"]
    checked = (0, B // 2, B - 1)
    vh = {c: make_v(q, nv, seed=900 + c) for c in checked}
    v = _t(make_v(q, nv, seed=899))[None].repeat(B, 1, 1)
    for c in checked:
        v[c] = _t(vh[c])
    torch.cuda.synchronize()
    return P, q, params, prv, nv, checked, vh, v


def _zeros(params, B, keys):
    import torch
    sh = params.shapes(B)
    return {k: torch.zeros(sh[k], dtype=torch.int64, device="cuda") for k in keys}


@pytest.mark.parametrize("name,B", [("t14_b1", 256), ("t16_b4096", 512)])
def test_commit_sampled_bench_batch_matches_oracle(name, B):
    import torch
    P, q, params, prv, nv, checked, vh, v = _setup(name, B)
    if name == "t16_b4096":  # the 12-wave encode prep's launch threshold (prep_launch)
        assert B * (P["cols"] + 1) * P["rows"] >= 1 << 20
    seeds = jindo.Seeds.derive(b"bench-batch-" + name.encode())
    first = 3 * B  # a nonzero first_commit, as rank 3 of the bench would use
    a = _zeros(params, B, OUT_KEYS)
    st = torch.cuda.Stream()  # the bench launches on a non-null stream too
    torch.cuda.synchronize()
    prv.commit_sampled_dev(B, v, nv, seeds, first, *[a[k] for k in OUT_KEYS], stream=st)
    st.synchronize()
    ck = prv.commit_key()
    cj = co.CJindo(P, q)
    sds = [P[k] for k in jindo.STDDEV_KEYS]
    dinv = pyref.delta_inv(P["base"], P["exp"])
    for c in checked:
        rnd = cj.sample(sds, dinv, seeds.raw(), first + c, vh[c][None])
        w = cj.commit(ck[0], ck[1], ck[2], vh[c], rnd["last_row"][0], rnd["mask"][0], rnd["enc_noise"][0],
                      rnd["mlwe_noise"][0])
        assert (_h(a["enc"][c]) == w["enc"]).all(), c
        assert (_h(a["mlwe_out"][c]) == w["mlwe"]).all(), c
        assert (_h(a["incom"][c]) == w["incom"]).all(), c
        assert (_h(a["com"][c]) == w["com"]).all(), c
    # every commit: the same commits in chunks of 64 (the 4-wave prep, the DAG at a small batch)
    b_ = _zeros(params, 64, OUT_KEYS)
    for lo in range(0, B, 64):
        hi = min(B, lo + 64)
        prv.commit_sampled_dev(hi - lo, v[lo:hi], nv, seeds, first + lo, *[b_[k][:hi - lo] for k in OUT_KEYS])
        torch.cuda.synchronize()
        for k in OUT_KEYS:
            assert torch.equal(a[k][lo:hi], b_[k][:hi - lo]), (lo, k)


@pytest.mark.parametrize("name,B", [("t14_b1", 256), ("t16_b4096", 512)])
def test_commit_injected_bench_batch_equals_sampled(name, B):
    """The injected line's path (rg_jindo_commit_dev: one prep launch of encode + MLWE jobs, 12-wave
    at configs[4]) on rg_jindo_sample_dev's draws == the sampled path, on all B commits."""
    import torch
    P, q, params, prv, nv, checked, vh, v = _setup(name, B)
    seeds = jindo.Seeds.derive(b"bench-inj-" + name.encode())
    first = 11
    r = _zeros(params, B, RND_KEYS)
    prv.sample_dev(B, v, nv, seeds, first, *[r[k] for k in RND_KEYS])
    a = _zeros(params, B, OUT_KEYS)
    prv.commit_dev(B, v, nv, *[r[k] for k in RND_KEYS], *[a[k] for k in OUT_KEYS])
    torch.cuda.synchronize()
    del r
    b_ = _zeros(params, B, OUT_KEYS)
    prv.commit_sampled_dev(B, v, nv, seeds, first, *[b_[k] for k in OUT_KEYS])
    torch.cuda.synchronize()
    for k in OUT_KEYS:
        assert torch.equal(a[k], b_[k]), k
