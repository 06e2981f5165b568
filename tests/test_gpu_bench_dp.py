"""bench.py's own N>1 code path (VERDICT r03 'do this' 2c): two ranks launched exactly as the driver launches
the scaling bench (python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 bench.py --gpus 2),
with UNET_DIST_BACKEND=gloo so that both ranks can share this box's one GPU (the driver's N>1 runs use RCCL, one
rank per GPU).  Exercises set_device before init_process_group, DDP over the per-module autograd nodes, the
barrier + max-over-ranks timing and rank 0's JSON line."""

import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_gloo():
    env = dict(os.environ, UNET_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "1", "--size", "128"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]      # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2", line
    assert line["config"]["global_batch"] == 2
    assert line["value"] > 0 and line["value"] == line["value"], line
    assert "gloo" in line["config"]["grad_sync"]
    assert "cpu_baseline" not in line            # rank 0 at N=1 only
