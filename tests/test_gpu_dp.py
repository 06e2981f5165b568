"""GPU: the overlapped gradient averaging (unet.utils.distributed.OverlappedGradSync) through the real
HIP backward, 2 ranks on one GPU over gloo (the driver's N>1 bench runs the same hooks over RCCL).

Each rank runs AttentionUNet on its own micro-batch.  The per-stage buckets launched from
NetworkPlan.backward must give every rank the average of the per-rank gradients that an unsynchronised
copy of the model computes (DDP semantics), including no_sync gradient accumulation
(scripts/train.py:133-143).
"""

import copy
import os
import socket
import sys
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch(i, dev):
    g = torch.Generator().manual_seed(500 + i)
    x = (torch.rand(2, 1, 64, 64, generator=g) * 2 - 1).to(dev)
    t = torch.zeros(2, 64, 64, dtype=torch.int64)
    t[0, 8 + i:30, 10:40 - i] = 1
    t[1, 33:50, 5 + 2 * i:60] = 1
    return x, t.to(dev)


def _worker(rank, world, port, q):
    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root / "unet-segment-pytorch_amd"), str(root)]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from unet.models import AttentionUNet
    from unet.utils.distributed import OverlappedGradSync
    from unet.utils.loss import DiceBCELoss
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.manual_seed(0)
        m = AttentionUNet(1, 2, base_features=8).to(dev).train()
        m.hip_precision = "fp32"
        ref = copy.deepcopy(m)                       # unsynchronised copy: local gradients only
        sync = OverlappedGradSync(m, bucket_cap_mb=0.05)
        crit = DiceBCELoss()

        def averaged_ref(micro):
            ref.zero_grad(set_to_none=True)
            for i in micro:
                x, t = _batch(i, dev)
                (crit(ref(x), t) / len(micro)).backward()
            out = {}
            for k, p in ref.named_parameters():
                g = p.grad.clone()
                dist.all_reduce(g)
                out[k] = g / world
            return out

        def worst(expect):
            w = 0.0
            for k, p in m.named_parameters():
                d = (p.grad - expect[k]).abs().max().item()
                w = max(w, d / (expect[k].abs().max().item() + 1e-12))
            return w

        # one synchronised micro-batch
        x, t = _batch(rank, dev)
        crit(sync(x), t).backward()
        w1 = worst(averaged_ref([rank]))
        # accumulation over two micro-batches, the first under no_sync
        m.zero_grad(set_to_none=True)
        with sync.no_sync():
            x, t = _batch(rank, dev)
            (crit(sync(x), t) / 2).backward()
        x, t = _batch(rank + 2, dev)
        (crit(sync(x), t) / 2).backward()
        torch.cuda.synchronize()
        w2 = worst(averaged_ref([rank, rank + 2]))
        q.put((rank, w1, w2, None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, None, None, repr(e)))


def test_overlapped_grad_sync_hip_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    for rank, w1, w2, err in res:
        assert err is None, f"rank {rank}: {err}"
        # fp32 operand mode: same kernels on both sides, differences are the bucket average's rounding
        assert w1 < 1e-5 and w2 < 1e-5, (rank, w1, w2)
    assert all(p.exitcode == 0 for p in procs)
