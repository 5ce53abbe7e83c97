"""Multi-GPU layout for the hot path: one process per GPU (torch.distributed; backend "nccl"
is RCCL on ROCm), independent polynomials / commitments sharded in contiguous ranges with no
data-path collective, and ONE collective at setup: the commit key is broadcast
from rank 0 over xGMI (or regenerated from the CRS per rank, which needs no collective)."""
import ctypes

import numpy as np


def shard_range(n_units, rank, world):
    """Contiguous [lo, hi) slice of n_units owned by `rank` (sizes differ by at most one)."""
    base, extra = divmod(n_units, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def bind_device(local_rank, world_size=1):
    """One rank per GPU: LOCAL_RANK -> torch's current device and libringo's (rg_set_device), then
    check both agree.  Fails (ValueError) when the node has fewer visible GPUs than ranks need."""
    import torch
    from ._lib import check, lib
    n = torch.cuda.device_count()
    if n < 1 or local_rank >= n:
        raise ValueError(f"LOCAL_RANK {local_rank} (world {world_size}) but {n} visible GPU(s)")
    torch.cuda.set_device(local_rank)
    check(lib().rg_set_device(local_rank))
    got = ctypes.c_int(-1)
    check(lib().rg_get_device(ctypes.byref(got)))
    if got.value != local_rank or torch.cuda.current_device() != local_rank:
        raise RuntimeError(f"rank bound to device {got.value} / torch {torch.cuda.current_device()}, "
                           f"want {local_rank}")
    return local_rank


def broadcast_commit_key(ck, dist, device=None, src=0):
    """Host-array variant: broadcast the three commit-key arrays (uint64, any shape) from `src`
    (zero arrays of the right shape elsewhere) through one flat buffer; returns host arrays.
    For the throughput path use `broadcast_prover`, which never leaves the GPU."""
    import torch
    sizes = [a.size for a in ck]
    flat = np.concatenate([np.ascontiguousarray(a, np.uint64).reshape(-1) for a in ck])
    t = torch.from_numpy(flat.view(np.int64).copy())
    if device is not None:
        t = t.to(device)
    dist.broadcast(t, src=src)
    out = t.cpu().numpy().view(np.uint64)
    res, off = [], 0
    for a, n in zip(ck, sizes):
        res.append(out[off:off + n].reshape(a.shape))
        off += n
    return tuple(res)


def broadcast_prover(params, dist, crs, src=0, stream=None):
    """One jindo.Prover per GPU with ONE collective: rank `src` derives the
    commit key from the CRS (NewCommitKey, entities.go:21-73), copies it device-to-device into a
    flat buffer, RCCL broadcasts that buffer over xGMI (one large message: the links are
    point-to-point), and every other rank builds its prover straight from the received device
    buffer (rg_jindo_create_dev).  The key never passes through host memory after `src` made it."""
    import torch
    from ._lib import check, lib
    from .jindo import Prover, _words
    dev = torch.device("cuda", torch.cuda.current_device())
    sh = params.ck_shapes()
    n = [_words(sh[k]) for k in ("ck_in", "ck_mlwe", "ck_out")]
    flat = torch.empty(sum(n), dtype=torch.int64, device=dev)
    st = None if stream is None else getattr(stream, "cuda_stream", stream)
    prv = None
    if dist.get_rank() == src:
        prv = Prover(params, crs=crs)
        off = 0
        for p_src, w in zip(prv.commit_key_dev(), n):
            if w:
                check(lib().rg_memcpy_d2d(flat.data_ptr() + 8 * off, p_src, 8 * w, st))
            off += w
        check(lib().rg_stream_sync(st))
    dist.broadcast(flat, src=src)
    if prv is None:
        torch.cuda.synchronize()
        parts = torch.split(flat, n)
        prv = Prover(params, ck_dev=parts, stream=stream)
    return prv


def allreduce_open_batch(prv, dist, ob_incom, ob_enc, ob_mlwe, stream=None):
    """Sharded Prover.Evaluate batch combination (jindo/prover.go:254-266): every rank has run
    rg_jindo_eval_batch_dev over its own commits (its slice of the batch challenges); the
    partial openBatches (residues < q) are summed across ranks with ONE all-reduce over a flat
    buffer (exact: world * q < 2^64 for the <= 60-bit ring primes) and folded mod q on device.
    The tensors are int64 views of the uint64 words; they hold the full openBatch afterwards."""
    import torch
    if dist is None:
        return
    P = prv.params
    assert dist.get_world_size() * max(max(P.q), max(P.qo)) < 2 ** 64
    flat = torch.cat([ob_incom.reshape(-1), ob_enc.reshape(-1), ob_mlwe.reshape(-1)])
    dist.all_reduce(flat)  # int64 wrap-around addition == uint64 addition
    n1, n2 = ob_incom.numel(), ob_enc.numel()
    ob_incom.view(-1).copy_(flat[:n1])
    ob_enc.view(-1).copy_(flat[n1:n1 + n2])
    ob_mlwe.view(-1).copy_(flat[n1 + n2:])
    prv.eval_reduce_dev(ob_incom, ob_enc, ob_mlwe, stream)
