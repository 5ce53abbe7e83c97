"""CPU: bench.py's multi-GPU launcher.  `python bench.py --gpus N` (no torch.distributed.run
around it) must start N ranks itself, keep the barrier + max-over-ranks timing, and have rank 0
print ONE JSON line with n_gpus == N.  --plumbing swaps the GPU step for a trivial host step on
gloo, so this runs without a GPU; the rank/launch logic is the same code the driver's N-GPU run
takes."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=e, timeout=240)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [1, 2, 3])
def test_launcher_runs_n_ranks(n):
    p = _run(["--gpus", str(n), "--plumbing", "--steps", "3", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["ranks"] == list(range(n)) and d["steps"] == 3


@pytest.mark.timeout(120)
def test_world_size_mismatch_fails():
    p = _run(["--gpus", "2", "--plumbing"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2 and "WORLD_SIZE=1" in p.stderr


@pytest.mark.timeout(240)
def test_more_ranks_than_gpus_fails():
    """A real (non-plumbing) run whose WORLD_SIZE exceeds the visible GPUs stops before any
    collective, with a message naming both (here: 0 GPUs in this container; on a GPU box the same
    check refuses N > device_count)."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("needs a host with fewer than 2 visible GPUs")
    p = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-extra", "--no-cpu"])
    assert p.returncode != 0
    assert "visible GPU(s)" in p.stderr, p.stderr[-2000:]
