"""CPU, world_size 2 (gloo): the multi-GPU host logic -- contiguous sharding of commits /
polynomials and the one-time commit-key broadcast -- exercised with real processes.  The
per-rank compute is the C oracle here (no GPU); on the box the same code drives libringo."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from ringo.shard import shard_range


def test_shard_range_partitions():
    for n in [0, 1, 7, 512, 4096, 4097]:
        for w in [1, 2, 3, 8]:
            parts = [shard_range(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "ringo-snark_amd"))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import coracle as co
    from ringo.shard import broadcast_commit_key, shard_range
    shapes = [(3, 5, 2, 8), (3, 2, 2, 8), (2, 6, 1, 8)]
    if rank == 0:
        rng = np.random.default_rng(42)
        ck = tuple(rng.integers(0, 2 ** 62, size=s, dtype=np.int64).astype(np.uint64) for s in shapes)
    else:
        ck = tuple(np.zeros(s, np.uint64) for s in shapes)
    ck = broadcast_commit_key(ck, dist)
    digest = np.array([int(a.sum() % (1 << 61)) for a in ck], dtype=np.int64)
    # sharded independent work: each rank transforms its slice of 10 polys
    q = 47104 ** 4 + 1
    cf = co.CField(q)
    tw, twi, ninv = cf.tables(64)
    rng = np.random.default_rng(7)
    allp = (rng.integers(0, 2 ** 62, size=(10, 64, 1), dtype=np.int64).astype(np.uint64)) % np.uint64(q)
    lo, hi = shard_range(10, rank, world)
    mine = cf.ntt_fwd(allp[lo:hi], tw)
    out[rank] = (digest.tolist(), lo, hi, mine.tolist())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_broadcast_and_shard():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    d0, d1 = out[0][0], out[1][0]
    assert d0 == d1  # every rank holds rank 0's key
    import coracle as co
    q = 47104 ** 4 + 1
    cf = co.CField(q)
    tw, _, _ = cf.tables(64)
    rng = np.random.default_rng(7)
    allp = (rng.integers(0, 2 ** 62, size=(10, 64, 1), dtype=np.int64).astype(np.uint64)) % np.uint64(q)
    want = cf.ntt_fwd(allp, tw)
    got = np.concatenate([np.array(out[r][3], dtype=np.uint64) for r in range(world)])
    assert (got == want).all()


def _eval_worker(rank, world, port, out):
    """Sharded Evaluate batch combination: each rank combines its slice of the openings with the
    C oracle (standing in for rg_jindo_eval_batch_dev), then ringo.shard.allreduce_open_batch
    sums the partial openBatches over gloo; the mod-q fold (rg_jindo_eval_reduce_dev on the box)
    is done on the CPU here."""
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "ringo-snark_amd"))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import coracle as co
    from ringo.shard import allreduce_open_batch, shard_range
    P = json.load(open(os.path.join(root, "tests", "golden", "jindo_params.json")))["t10_b8"]
    cj = co.CJindo(P, int(P["field_q_hex"], 16))
    es = cj.eval_shapes()
    B = P["batch"]
    rng = np.random.default_rng(21)

    def res(primes, shape):
        o = np.zeros(shape, np.uint64)
        for l, qq in enumerate(primes):
            o[..., l, :] = rng.integers(0, qq, size=o[..., l, :].shape, dtype=np.uint64)
        return o

    incom, enc = res(P["qo"], (B,) + es["ob_incom"]), res(P["q"], (B,) + es["ob_enc"])
    mlwe = res(P["q"], (B,) + es["ob_mlwe"])
    bq, bo = res(P["q"], (B, len(P["q"]), P["d"])), res(P["qo"], (B, len(P["qo"]), P["d"]))
    lo, hi = shard_range(B, rank, world)
    part = cj.eval_batch(incom[lo:hi], enc[lo:hi], mlwe[lo:hi], bq[lo:hi], bo[lo:hi])

    class FakeProver:  # the parameters allreduce_open_batch reads, and a CPU mod-q fold
        class params:
            q, qo = P["q"], P["qo"]

        @staticmethod
        def eval_reduce_dev(a, b, c, stream=None):
            for x, primes in ((a, P["qo"]), (b, P["q"]), (c, P["q"])):
                v = x.numpy().view(np.uint64)
                for l, qq in enumerate(primes):
                    v[..., l, :] %= np.uint64(qq)

    ts = [torch.from_numpy(part[k].view(np.int64).copy()) for k in ("ob_incom", "ob_enc", "ob_mlwe")]
    allreduce_open_batch(FakeProver, dist, *ts)
    whole = cj.eval_batch(incom, enc, mlwe, bq, bo)
    out[rank] = all(bool((t.numpy().view(np.uint64) == whole[k]).all())
                    for t, k in zip(ts, ("ob_incom", "ob_enc", "ob_mlwe")))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_evaluate_batch_allreduce():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_eval_worker, args=(world, port, out), nprocs=world, join=True)
    assert out[0] and out[1]
