"""GPU, world_size 2 on one card: the multi-GPU host path driving libringo with real ranks.
Both processes use cuda:0 (the pool's boxes have one GPU) and talk over gloo (CUDA tensors are
staged through the host by gloo; on an 8-GPU node bench.py uses RCCL, with the same code):
  * broadcast_prover: rank 0 derives the commit key from the CRS, copies it device to device
    into a flat buffer, broadcasts it; rank 1 builds its prover from the received DEVICE buffer;
  * each rank commits its contiguous shard of the params.batch commits (rg_jindo_commit_dev);
  * the sharded Evaluate batch combination sums the ranks' partial openBatches
    (allreduce_open_batch) and folds them mod q on the device.
Checked against one process doing the whole batch, bit for bit."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(P, q):
    from tests.jindo_util import make_randomness, make_v
    B, nv = P["batch"], 900
    vs = np.stack([make_v(q, nv, seed=80 + b) for b in range(B)])
    rnd = make_randomness(P, q, seed=81, batch=B)
    rng = np.random.default_rng(82)
    bq = np.stack([np.stack([rng.integers(0, x, size=P["d"], dtype=np.uint64) for x in P["q"]]) for _ in range(B)])
    bo = np.stack([np.stack([rng.integers(0, x, size=P["d"], dtype=np.uint64) for x in P["qo"]]) for _ in range(B)])
    return nv, vs, rnd, bq, bo


def _run(prv, params, lo, hi, nv, vs, rnd, bq, bo):
    import torch
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to("cuda")
    B = hi - lo
    sh = params.shapes(B)
    o = {k: torch.zeros(sh[k], dtype=torch.int64, device="cuda") for k in ["incom", "enc", "mlwe_out", "com"]}
    prv.commit_dev(B, t(vs[lo:hi]), nv, t(rnd["last_row"][lo:hi]), t(rnd["mask"][lo:hi]),
                   t(rnd["enc_noise"][lo:hi]), t(rnd["mlwe_noise"][lo:hi]), o["incom"], o["enc"], o["mlwe_out"],
                   o["com"])
    es = prv.eval_shapes()
    ob = {k: torch.zeros(es[k], dtype=torch.int64, device="cuda") for k in ("ob_incom", "ob_enc", "ob_mlwe")}
    prv.eval_batch_dev(B, o["incom"], o["enc"], o["mlwe_out"], t(bq[lo:hi]), t(bo[lo:hi]), ob["ob_incom"],
                       ob["ob_enc"], ob["ob_mlwe"])
    torch.cuda.synchronize()
    return o, ob


def _worker(rank, world, port, out):
    import sys
    root = os.path.dirname(HERE)
    for p in (os.path.join(root, "ringo-snark_amd"), os.path.join(root, "oracle"), root):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from ringo.shard import bind_device
    assert bind_device(0, world) == 0  # one card: every rank's LOCAL_RANK -> device 0
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ringo import jindo
    from ringo.shard import allreduce_open_batch, broadcast_prover, shard_range
    P = json.load(open(os.path.join(HERE, "golden", "jindo_params.json")))["t10_b8"]
    q = int(P["field_q_hex"], 16)
    params = jindo.Parameters.from_dict(P, q)
    prv = broadcast_prover(params, dist, b"Jindo!")
    nv, vs, rnd, bq, bo = _inputs(P, q)
    lo, hi = shard_range(P["batch"], rank, world)
    o, ob = _run(prv, params, lo, hi, nv, vs, rnd, bq, bo)
    allreduce_open_batch(prv, dist, ob["ob_incom"], ob["ob_enc"], ob["ob_mlwe"])
    torch.cuda.synchronize()
    out[rank] = {"lo": lo, "hi": hi, "com": o["com"].cpu().numpy().tobytes(),
                 "ob": b"".join(ob[k].cpu().numpy().tobytes() for k in ("ob_incom", "ob_enc", "ob_mlwe")),
                 "ck": b"".join(np.ascontiguousarray(x).tobytes() for x in prv.commit_key())}
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_two_ranks_broadcast_commit_evaluate():
    import torch
    from ringo import jindo
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    P = json.load(open(os.path.join(HERE, "golden", "jindo_params.json")))["t10_b8"]
    q = int(P["field_q_hex"], 16)
    params = jindo.Parameters.from_dict(P, q)
    prv = jindo.NewProver(params, b"Jindo!")
    nv, vs, rnd, bq, bo = _inputs(P, q)
    o, ob = _run(prv, params, 0, P["batch"], nv, vs, rnd, bq, bo)
    ck = b"".join(np.ascontiguousarray(x).tobytes() for x in prv.commit_key())
    com = o["com"].cpu().numpy()
    whole = b"".join(ob[k].cpu().numpy().tobytes() for k in ("ob_incom", "ob_enc", "ob_mlwe"))
    for r in range(world):
        d = out[r]
        assert d["ck"] == ck, r  # the broadcast key
        assert d["com"] == com[d["lo"]:d["hi"]].tobytes(), r  # the shard's commitments
        assert d["ob"] == whole, r  # the all-reduced openBatch
    assert out[0]["hi"] == out[1]["lo"]


def _rccl_worker(rank, world, port, out):
    """world 1 on the `nccl` backend (RCCL): the exact calls bench.py makes on an N-GPU node
    (init_process_group("nccl", device_id=...), bind_device, broadcast_prover's device-buffer
    broadcast, allreduce_open_batch's all-reduce of device words + the mod-q fold), on real RCCL
    collectives over device pointers.  One card cannot host two RCCL ranks (RCCL refuses a
    duplicate GPU), so the multi-rank data movement is the gloo test above."""
    import sys
    root = os.path.dirname(HERE)
    for p in (os.path.join(root, "ringo-snark_amd"), os.path.join(root, "oracle"), root):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from ringo.shard import bind_device
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    bind_device(0, world)
    from ringo import jindo
    from ringo.shard import allreduce_open_batch, broadcast_prover
    P = json.load(open(os.path.join(HERE, "golden", "jindo_params.json")))["t10_b8"]
    q = int(P["field_q_hex"], 16)
    params = jindo.Parameters.from_dict(P, q)
    prv = broadcast_prover(params, dist, b"Jindo!")
    nv, vs, rnd, bq, bo = _inputs(P, q)
    o, ob = _run(prv, params, 0, P["batch"], nv, vs, rnd, bq, bo)
    before = b"".join(ob[k].cpu().numpy().tobytes() for k in ("ob_incom", "ob_enc", "ob_mlwe"))
    allreduce_open_batch(prv, dist, ob["ob_incom"], ob["ob_enc"], ob["ob_mlwe"])
    torch.cuda.synchronize()
    out[rank] = {"com": o["com"].cpu().numpy().tobytes(), "before": before,
                 "ob": b"".join(ob[k].cpu().numpy().tobytes() for k in ("ob_incom", "ob_enc", "ob_mlwe")),
                 "ck": b"".join(np.ascontiguousarray(x).tobytes() for x in prv.commit_key())}
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_rccl_single_rank_bench_path():
    from ringo import jindo
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_rccl_worker, args=(1, _free_port(), out), nprocs=1, join=True)
    P = json.load(open(os.path.join(HERE, "golden", "jindo_params.json")))["t10_b8"]
    q = int(P["field_q_hex"], 16)
    params = jindo.Parameters.from_dict(P, q)
    prv = jindo.NewProver(params, b"Jindo!")
    nv, vs, rnd, bq, bo = _inputs(P, q)
    o, ob = _run(prv, params, 0, P["batch"], nv, vs, rnd, bq, bo)
    d = out[0]
    assert d["ck"] == b"".join(np.ascontiguousarray(x).tobytes() for x in prv.commit_key())
    assert d["com"] == o["com"].cpu().numpy().tobytes()
    whole = b"".join(ob[k].cpu().numpy().tobytes() for k in ("ob_incom", "ob_enc", "ob_mlwe"))
    assert d["before"] == whole and d["ob"] == whole  # all-reduce over one rank + fold: identity
