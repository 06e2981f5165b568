"""GPU: data-parallel training through stock torch DistributedDataParallel on the HIP backward
(reference caller scripts/train.py:132-143).

* The network's backward is one autograd node per reference module (unet._hip.functions), so parameter
  gradients become ready stage by stage — outc, up4 .. up1, down4 .. down1, inc — which is what lets
  DDP's reducer all-reduce full buckets while later stages still compute.
* 2 ranks on one GPU over gloo (the driver's N>1 bench runs the same reducer over RCCL): DDP's averaged
  gradients equal the average of the per-rank gradients of an unsynchronised copy, including no_sync
  gradient accumulation (loss / accum per micro-batch).
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


@pytest.mark.parametrize("ds", [False, True])
def test_stage_nodes_release_grads_in_stage_order(ds):
    """Parameter gradients are accumulated stage by stage in reverse data-flow order (one autograd node
    per module), not all at once at the end of the backward."""
    from unet.models import AttentionUNet
    from unet.utils.loss import DeepSupervisionLoss, DiceBCELoss
    torch.manual_seed(0)
    m = AttentionUNet(1, 2, base_features=8, deep_supervision=ds).cuda().train()
    m.hip_precision = "fp32"
    order = []
    for name, p in m.named_parameters():
        p.register_post_accumulate_grad_hook(lambda p, name=name: order.append(name.split(".")[0]))
    x, t = _batch(0, "cuda")
    out = m(x)
    crit = DeepSupervisionLoss(DiceBCELoss()) if ds else DiceBCELoss()
    loss = crit(out, t)
    nodes, seen, stack = 0, set(), [loss.grad_fn]
    while stack:
        f = stack.pop()
        if f is None or f in seen:
            continue
        seen.add(f)
        nodes += type(f).__name__ == "_StageFnBackward"
        stack.extend(nf for nf, _ in f.next_functions)
    assert nodes == 10 + (3 if ds else 0), nodes
    loss.backward()
    stages = []
    for s in order:
        if not stages or stages[-1] != s:
            stages.append(s)
    main = [s for s in stages if not s.startswith("ds_out")]
    assert main == ["outc", "up4", "up3", "up2", "up1", "down4", "down3", "down2", "down1", "inc"], stages
    assert len(order) == len(list(m.parameters()))


def _worker(rank, world, port, q):
    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root / "unet-segment-pytorch_amd"), str(root)]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from unet.models import AttentionUNet
    from unet.utils.distributed import wrap_ddp
    from unet.utils.loss import DiceBCELoss
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.manual_seed(rank)                      # different init per rank: DDP broadcasts rank 0's
        m = AttentionUNet(1, 2, base_features=8).to(dev).train()
        m.hip_precision = "fp32"
        ddp = wrap_ddp(m, None, bucket_cap_mb=0.05)  # small buckets: several all-reduces during the backward
        ref = copy.deepcopy(m)                       # unsynchronised copy of the broadcast weights
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

        x, t = _batch(rank, dev)
        crit(ddp(x), t).backward()
        w1 = worst(averaged_ref([rank]))
        m.zero_grad(set_to_none=True)
        with ddp.no_sync():
            x, t = _batch(rank, dev)
            (crit(ddp(x), t) / 2).backward()
        x, t = _batch(rank + 2, dev)
        (crit(ddp(x), t) / 2).backward()
        torch.cuda.synchronize()
        w2 = worst(averaged_ref([rank, rank + 2]))
        w0 = float(sum(p.detach().double().sum() for p in m.parameters()))
        q.put((rank, w1, w2, w0, None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, None, None, None, traceback.format_exc()))


def test_torch_ddp_hip_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    for rank, w1, w2, w0, err in res:
        assert err is None, f"rank {rank}: {err}"
        # fp32 operand mode: same kernels on both sides, differences are the bucket average's rounding
        assert w1 < 1e-5 and w2 < 1e-5, (rank, w1, w2)
    assert res[0][3] == res[1][3]                   # identical (broadcast) weights on both ranks
    assert all(p.exitcode == 0 for p in procs)
