"""world_size-2 gloo tests of the data-parallel path, CPU only.

The HIP path shards by batch: each rank runs the whole network on its own micro-batch (BN uses
per-rank batch statistics, as the reference's per-micro-batch BN) and the only exchange is the
gradient all-reduce (average).  These tests pin the two facts the multi-GPU bench relies on:

* DDP's averaged gradients over 2 ranks x 1 micro-batch equal the reference semantics of
  gradient accumulation over the same 2 micro-batches (scripts/train.py:133-143: loss / accum,
  backward per micro-step), computed here with the oracle (test infrastructure);
* bench.py's job time is the max over ranks, identical on every rank.
"""

from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _setup(rank: int, world: int, port: int):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _micro_batch(i: int):
    g = torch.Generator().manual_seed(100 + i)
    x = torch.rand(2, 1, 32, 32, generator=g) * 2 - 1
    t = torch.zeros(2, 32, 32, dtype=torch.int64)
    t[0, 4:12, 5:14] = 1
    t[1, 20:27, 9:30] = 1
    return x, t


def _grads(i: int):
    from oracle import unet_oracle as O
    from unet.models import AttentionUNet
    torch.manual_seed(0)
    m = AttentionUNet(1, 2, base_features=4)
    p = O.params_from_module(m)
    x, t = _micro_batch(i)
    loss = O.dice_bce_loss(O.attention_unet_forward(p, x, training=True), t)
    loss.backward()
    return {k: v.grad.clone() for k, v in p.items() if v.grad is not None}


def _ddp_worker(rank: int, world: int, port: int, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root / "unet-segment-pytorch_amd"), str(root)]
    _setup(rank, world, port)
    g = _grads(rank)
    for k in sorted(g):
        dist.all_reduce(g[k])
        g[k] /= world
    if rank == 0:
        q.put({k: v.numpy() for k, v in g.items()})
    dist.barrier()
    dist.destroy_process_group()


def _max_worker(rank: int, world: int, port: int, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root)]
    _setup(rank, world, port)
    import bench
    q.put((rank, bench.max_over_ranks(1.0 + rank, torch.device("cpu"))))
    dist.barrier()
    dist.destroy_process_group()


def _run(fn, world: int):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(len(procs) if fn is _max_worker else 1)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_ddp_average_equals_grad_accumulation():
    (ddp,) = _run(_ddp_worker, 2)
    g0, g1 = _grads(0), _grads(1)
    assert set(ddp) == set(g0)
    worst = 0.0
    for k in g0:
        acc = (g0[k] + g1[k]) / 2   # accum 2: loss/2 per micro-step, summed
        d = (torch.from_numpy(ddp[k]) - acc).abs().max().item()
        worst = max(worst, d / (acc.abs().max().item() + 1e-12))
    assert worst < 1e-4, worst  # fp32 reduction-order noise (workers run single-threaded)


def test_bench_time_is_max_over_ranks():
    out = _run(_max_worker, 2)
    assert sorted(v for _, v in out) == [2.0, 2.0]


def test_single_process_time_passthrough():
    import bench
    assert bench.max_over_ranks(3.5, torch.device("cpu")) == 3.5


def test_graphed_train_step_refuses_ddp():
    """GraphedTrainStep takes its gradients on leaf aliases of the parameters, so a DDP-wrapped
    model's reducer hooks would never fire; it must refuse DDP up front (before touching any device)."""
    from unet.utils.graphed import GraphedTrainStep
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        ddp = torch.nn.parallel.DistributedDataParallel(torch.nn.Linear(4, 2))
        opt = torch.optim.AdamW(ddp.parameters(), lr=1e-3, capturable=True)
        with pytest.raises(RuntimeError, match="DDP"):
            GraphedTrainStep(ddp, torch.nn.functional.mse_loss, opt, (2, 4), (2, 2))
    finally:
        dist.destroy_process_group()
