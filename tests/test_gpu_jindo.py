"""GPU parity: libringo's Jindo commit (rg_jindo_commit / rg_jindo_commit_dev) vs the C oracle
(oracle/oracle.c, itself cross-checked against the big-int restatement), bit-exact on every
output of Prover.Commit (jindo/prover.go:45-202): Opening.{InCommit, Encode, MLWE} and
Commitment.Value, plus the CRS-derived commit key (entities.go:21-73).

Shapes: tests/golden/jindo_params.json (jindo_test sizes, configs[2] 2^14, and the 3-prime
examples/mult config).  Randomness is injected (tests/jindo_util.py)."""
import json
import os

import numpy as np
import pytest

import coracle as co
import pyref
from ringo import jindo
from tests.jindo_util import make_randomness, make_v

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
PARAMS = json.load(open(os.path.join(HERE, "golden", "jindo_params.json")))


def _setup(name):
    P = PARAMS[name]
    q = int(P["field_q_hex"], 16)
    params = jindo.Parameters.from_dict(P, q)
    return P, q, params


def _oracle_commit(P, q, ck, v, rnd):
    cj = co.CJindo(P, q)
    return cj.commit(ck[0], ck[1], ck[2], v, rnd["last_row"], rnd["mask"], rnd["enc_noise"], rnd["mlwe_noise"])


@pytest.mark.parametrize("name", ["t10_b1", "t10_b8", "mult_t8193_b12"])
def test_commit_key_from_crs(name):
    P, q, params = _setup(name)
    prv = jindo.NewProver(params, b"Jindo!")
    got = prv.commit_key()
    want = pyref.commit_key(pyref.JindoParams(q, P["target_n"], P["batch"]), b"Jindo!")
    for g, w in zip(got, want):
        assert (g == np.array(w, dtype=np.uint64)).all()


def _edge_v(q, b, exp, n, seed):
    """v (Montgomery form, R = 2^(64L)) whose canonical values hit the digit split's boundaries
    (csrc/digits_dc.hpp): 0, q - 1, powers of b and of B4 = b^4 / B8 = b^8 and their neighbours,
    then seeded random values"""
    L = (q.bit_length() + 63) // 64
    R = 1 << (64 * L)
    vals = [0, 1, q - 1, q - 2]
    for k in range(exp + 1):
        vals += [b ** k - 1, b ** k, b ** k + 1, q - b ** k]
    for m in (1, 2, 3, 7):
        vals += [m * b ** 4 - 1, m * b ** 4, (q // b ** 8) * b ** 8 - m, m * b ** 8 - 1, m * b ** 8]
    rng = np.random.default_rng(seed)
    vals = [x % q for x in vals]
    vals += [int(rng.integers(0, 1 << 62)) * int(rng.integers(0, 1 << 62)) % q for _ in range(max(0, n - len(vals)))]
    vals = vals[:n]
    out = np.zeros((n, L), np.uint64)
    for i, c in enumerate(vals):
        m = c * R % q
        for j in range(L):
            out[i, j] = (m >> (64 * j)) & ((1 << 64) - 1)
    return out


@pytest.mark.parametrize("name", ["t14_b1", "mult_t8193_b12"])
def test_commit_digit_edges_match_oracle(name):
    """Encode's base-b digits of boundary values (divide-and-conquer split on the device) vs the
    oracle's repeated division, through the whole commit."""
    P, q, params = _setup(name)
    prv = jindo.NewProver(params, b"Jindo!")
    ck = prv.commit_key()
    nv = min(P["rank"], 400)
    v = _edge_v(q, P["base"], P["exp"], nv, seed=3)
    rnd = make_randomness(P, q, seed=17)
    com, op = prv.Commit(v, jindo.Randomness(**rnd))
    want = _oracle_commit(P, q, ck, v, rnd)
    assert (op.Encode == want["enc"]).all(), name
    assert (com.Value == want["com"]).all(), name


@pytest.mark.parametrize("name,nvs", [("t10_b1", [1024, 300, 33, 1]), ("t10_b8", [1024, 129]),
                                      ("mult_t8193_b12", [8193, 700]), ("t14_b1", [16384, 5000])])
def test_commit_matches_oracle(name, nvs):
    P, q, params = _setup(name)
    prv = jindo.NewProver(params, b"Jindo!")
    ck = prv.commit_key()
    for nv in nvs:
        v = make_v(q, nv, seed=nv)
        rnd = make_randomness(P, q, seed=nv + 7)
        com, op = prv.Commit(v, jindo.Randomness(**rnd))
        want = _oracle_commit(P, q, ck, v, rnd)
        assert (op.Encode == want["enc"]).all(), (name, nv, "Encode")
        assert (op.MLWE == want["mlwe"]).all(), (name, nv, "MLWE")
        assert (op.InCommit == want["incom"]).all(), (name, nv, "InCommit")
        assert (com.Value == want["com"]).all(), (name, nv, "Commitment")


def test_commit_noncanonical_v_reduces():
    """A word of v equal to q (non-canonical; Montgomery q == 0) commits as 0 does: fromMont in
    the digit encoder (encoder.go:149-158 via element.go's Slice) reduces fully, as gnark's
    fromMont does for any word below R."""
    P, q, params = _setup("t10_b1")
    prv = jindo.NewProver(params, b"Jindo!")
    L = (q.bit_length() + 63) // 64
    v = make_v(q, 300, seed=3)
    v[5] = 0
    v[17] = [(q >> (64 * j)) & ((1 << 64) - 1) for j in range(L)]
    vz = v.copy()
    vz[17] = 0
    rnd = make_randomness(P, q, seed=11)
    com, op = prv.Commit(v, jindo.Randomness(**rnd))
    comz, opz = prv.Commit(vz, jindo.Randomness(**rnd))
    assert (op.Encode == opz.Encode).all()
    assert (com.Value == comz.Value).all()


@pytest.mark.parametrize("name", ["t10_b1", "t14_b1"])
def test_commit_extreme_noise_matches_oracle(name):
    """Injected noise far outside the samplers' range (|s| up to 2^63 - 1, INT64_MIN + 1), which
    takes the encode's term-by-term reduction instead of the one-integer form."""
    P, q, params = _setup(name)
    prv = jindo.NewProver(params, b"Jindo!")
    ck = prv.commit_key()
    nv = P["rank"]
    v = make_v(q, nv, seed=3)
    rnd = make_randomness(P, q, seed=11)
    rng = np.random.default_rng(12)
    en = rnd["enc_noise"]
    ext = np.array([2**63 - 1, -(2**63 - 1), 2**62 + 12345, -(2**61), 2**45 + 1, -(2**44), 2**40, -7],
                   dtype=np.int64)
    idx = rng.integers(0, en.size, size=4000)
    en.reshape(-1)[idx] = ext[rng.integers(0, ext.size, size=idx.size)]
    mn = rnd["mlwe_noise"]
    mn.reshape(-1)[rng.integers(0, mn.size, size=500)] = ext[rng.integers(0, ext.size, size=500)]
    com, op = prv.Commit(v, jindo.Randomness(**rnd))
    want = _oracle_commit(P, q, ck, v, rnd)
    assert (op.Encode == want["enc"]).all()
    assert (op.MLWE == want["mlwe"]).all()
    assert (op.InCommit == want["incom"]).all()
    assert (com.Value == want["com"]).all()


def test_commit_golden_digests():
    """The jindo_test-size commit against the committed fixture digests."""
    import hashlib
    G = json.load(open(os.path.join(HERE, "golden", "jindo_commit_golden.json")))
    P, q, params = _setup("t10_b1")
    prv = jindo.NewProver(params, b"Jindo!")
    ck = prv.commit_key()
    assert [hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest() for x in ck] == G["ck"]
    for nv, dig in G["cases"].items():
        nv = int(nv)
        v = make_v(q, nv, seed=nv)
        rnd = make_randomness(P, q, seed=nv + 1)
        com, op = prv.Commit(v, jindo.Randomness(**rnd))
        got = {"incom": op.InCommit, "enc": op.Encode, "mlwe": op.MLWE, "com": com.Value}
        for k, d in dig.items():
            assert hashlib.sha256(np.ascontiguousarray(got[k]).tobytes()).hexdigest() == d, (nv, k)


def test_commit_dev_batch_matches_single():
    import torch
    P, q, params = _setup("t10_b1")
    prv = jindo.NewProver(params, b"Jindo!")
    ck = prv.commit_key()
    B, nv = 4, 1000
    sh = params.shapes(B)
    vs = np.stack([make_v(q, nv, seed=100 + b) for b in range(B)])
    rnd = make_randomness(P, q, seed=5, batch=B)
    dev = torch.device("cuda")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
    dv, dl, dm, de, dn = t(vs), t(rnd["last_row"]), t(rnd["mask"]), t(rnd["enc_noise"]), t(rnd["mlwe_noise"])
    outs = {k: torch.zeros(sh[k], dtype=torch.int64, device=dev) for k in ["incom", "enc", "mlwe_out", "com"]}
    prv.commit_dev(B, dv, nv, dl, dm, de, dn, outs["incom"], outs["enc"], outs["mlwe_out"], outs["com"])
    torch.cuda.synchronize()
    for b in range(B):
        want = _oracle_commit(P, q, ck, vs[b], {k: v[b] for k, v in rnd.items()})
        assert (outs["com"][b].cpu().numpy().view(np.uint64) == want["com"]).all(), b
        assert (outs["incom"][b].cpu().numpy().view(np.uint64) == want["incom"]).all(), b
        assert (outs["enc"][b].cpu().numpy().view(np.uint64) == want["enc"]).all(), b
        assert (outs["mlwe_out"][b].cpu().numpy().view(np.uint64) == want["mlwe"]).all(), b


def test_commit_dev_empty_batch_is_noop():
    """A batch of zero commits returns OK and launches nothing (the output sentinel survives)."""
    import torch
    P, q, params = _setup("t10_b1")
    prv = jindo.NewProver(params, b"Jindo!")
    s = torch.full((16,), 777, dtype=torch.int64, device="cuda")
    prv.commit_dev(0, s, 1000, s, s, s, s, s, s, s, s)
    torch.cuda.synchronize()
    assert (s.cpu() == 777).all()


def test_commit_rank_panic():
    P, q, params = _setup("t10_b1")
    prv = jindo.NewProver(params, b"Jindo!")
    v = make_v(q, P["rank"] + 1, seed=1)
    rnd = make_randomness(P, q, seed=2)
    with pytest.raises(Exception, match="len\\(v\\) > params.rank"):
        prv.Commit(v, jindo.Randomness(**rnd))


@pytest.mark.parametrize("name", ["t10_b1", "t10_b8", "t14_b1", "mult_t8193_b12"])
def test_evaluate_core_matches_oracle(name):
    """Prover.Evaluate's MulCoeffsMontgomeryThenAdd loops (prover.go:228-314) on the GPU vs the C
    oracle, bit-exact, with injected challenges; openings are the GPU's own commits."""
    import torch
    P, q, params = _setup(name)
    prv = jindo.NewProver(params, b"Jindo!")
    B = P["batch"]
    dev = torch.device("cuda")
    rng = np.random.default_rng(77)
    sh = params.shapes(B)
    nv = P["rank"]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
    vs = np.stack([make_v(q, nv, seed=200 + b) for b in range(B)])
    rnd = make_randomness(P, q, seed=9, batch=B)
    op = {k: torch.zeros(sh[k], dtype=torch.int64, device=dev) for k in ["incom", "enc", "mlwe_out", "com"]}
    prv.commit_dev(B, t(vs), nv, t(rnd["last_row"]), t(rnd["mask"]), t(rnd["enc_noise"]), t(rnd["mlwe_noise"]),
                   op["incom"], op["enc"], op["mlwe_out"], op["com"])

    def res(primes, shape):
        out = np.zeros(shape, np.uint64)
        for l, qq in enumerate(primes):
            out[..., l, :] = rng.integers(0, qq, size=out[..., l, :].shape, dtype=np.uint64)
        return out

    es = prv.eval_shapes()
    bq, bo = res(P["q"], (B, len(P["q"]), P["d"])), res(P["qo"], (B, len(P["qo"]), P["d"]))
    left = res(P["q"], (P["rows"], len(P["q"]), P["d"]))
    chals = res(P["q"], (P["cols"], len(P["q"]), P["d"]))
    out = {k: torch.zeros(es[k], dtype=torch.int64, device=dev) for k in es}
    single = B == 1  # params.batch == 1: openBatch = open[0], no challenge (prover.go:267-269)
    prv.eval_batch_dev(B, op["incom"], op["enc"], op["mlwe_out"], None if single else t(bq), None if single else t(bo),
                       out["ob_incom"], out["ob_enc"], out["ob_mlwe"])
    prv.eval_partial_dev(out["ob_enc"], t(left), out["partial"])
    prv.eval_respond_dev(out["ob_enc"], out["ob_mlwe"], t(chals), out["pf_enc"], out["pf_mlwe"])
    torch.cuda.synchronize()
    got = {k: v.cpu().numpy().view(np.uint64) for k, v in out.items()}
    cj = co.CJindo(P, q)
    host = lambda k: op[k].cpu().numpy().view(np.uint64)
    ob = cj.eval_batch(host("incom"), host("enc"), host("mlwe_out"), bq, bo)
    for k in ("ob_incom", "ob_enc", "ob_mlwe"):
        assert (got[k] == ob[k]).all(), k
    assert (got["partial"] == cj.eval_partial(ob["ob_enc"], left)).all()
    pe, pm = cj.eval_respond(ob["ob_enc"], ob["ob_mlwe"], chals)
    assert (got["pf_enc"] == pe).all()
    assert (got["pf_mlwe"] == pm).all()


def test_evaluate_batch_shards_sum_to_whole():
    """A batch split across "ranks" (here: two shards on one GPU): each shard's partial openBatch,
    summed word-wise (what the RCCL all-reduce does) and folded mod q by rg_jindo_eval_reduce_dev,
    equals the single-GPU openBatch bit for bit."""
    import torch
    P, q, params = _setup("t10_b8")
    prv = jindo.NewProver(params, b"Jindo!")
    B = P["batch"]
    dev = torch.device("cuda")
    rng = np.random.default_rng(3)
    es = prv.eval_shapes()

    def res(primes, shape):
        out = np.zeros(shape, np.uint64)
        for l, qq in enumerate(primes):
            out[..., l, :] = rng.integers(0, qq, size=out[..., l, :].shape, dtype=np.uint64)
        return out

    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)
    incom = t(res(P["qo"], (B,) + es["ob_incom"]))
    enc = t(res(P["q"], (B,) + es["ob_enc"]))
    mlwe = t(res(P["q"], (B,) + es["ob_mlwe"]))
    bq, bo = t(res(P["q"], (B, len(P["q"]), P["d"]))), t(res(P["qo"], (B, len(P["qo"]), P["d"])))
    zeros = lambda: {k: torch.zeros(es[k], dtype=torch.int64, device=dev) for k in ("ob_incom", "ob_enc", "ob_mlwe")}
    whole = zeros()
    prv.eval_batch_dev(B, incom, enc, mlwe, bq, bo, whole["ob_incom"], whole["ob_enc"], whole["ob_mlwe"])
    parts = []
    for lo, hi in ((0, 3), (3, B)):
        o = zeros()
        prv.eval_batch_dev(hi - lo, incom[lo:hi], enc[lo:hi], mlwe[lo:hi], bq[lo:hi], bo[lo:hi], o["ob_incom"],
                           o["ob_enc"], o["ob_mlwe"])
        parts.append(o)
    summed = {k: parts[0][k] + parts[1][k] for k in parts[0]}
    prv.eval_reduce_dev(summed["ob_incom"], summed["ob_enc"], summed["ob_mlwe"])
    torch.cuda.synchronize()
    for k in summed:
        assert torch.equal(summed[k], whole[k]), k



MAC_SHAPES = [("t14_b1", 16384), ("mult_t8193_b12", 8193), ("t10_b8", 1024)]


def test_mac_paths_agree(tmp_path):
    """The two inner/outer MAC kernels (the MFMA digit MAC and mac_kernel) produce the same
    Opening.InCommit and Commitment.Value bit for bit.  The product library (this process) must
    run the MFMA MAC on both products of every shape; mac_kernel runs in a child process on the
    experiments build with RINGO_JINDO_MAC=l (tests/exp_child.py), checked to have taken it.  MSIS
    ranks J > 16 (examples/mult's 21) take mac_kernel in both: there this compares the product's
    fallback with itself, and test_commit_matches_oracle pins it."""
    import subprocess
    import sys

    def expect(J, mode):
        return "generic" if J > 16 or mode == "l" else "mfma"

    want = {}
    for name, nv in MAC_SHAPES:
        P, q, params = _setup(name)
        prv = jindo.NewProver(params, b"Jindo!")
        assert prv.mac_kinds() == (expect(P["in_msis"], ""), expect(P["out_msis"], "")), name
        com, op = prv.Commit(make_v(q, nv, seed=5), jindo.Randomness(**make_randomness(P, q, seed=9)))
        want[name] = (op.InCommit.copy(), com.Value.copy())
    for mode in ("l",):
        out = tmp_path / f"mac_{mode}.npz"
        r = subprocess.run([sys.executable, os.path.join(HERE, "exp_child.py"), "mac", mode, str(out)] +
                           [f"{n}:{nv}" for n, nv in MAC_SHAPES], capture_output=True, text=True, timeout=110)
        assert r.returncode == 0, r.stderr[-2000:]
        got = np.load(out)
        for name, _ in MAC_SHAPES:
            P = PARAMS[name]
            assert tuple(got[name + "/kinds"]) == (expect(P["in_msis"], mode), expect(P["out_msis"], mode)), (name, mode)
            assert (got[name + "/incom"] == want[name][0]).all(), (name, mode, "InCommit")
            assert (got[name + "/com"] == want[name][1]).all(), (name, mode, "Commitment")
