"""RCCL on the GPU box ("RCCL has never executed in any form"): one rank, backend "nccl" (= RCCL on
ROCm), device 0.  The N>1 scaling runs are the driver's (8-GPU node); what one GPU can show is that the path the
ranks take there initialises an RCCL communicator and runs its collectives: raw all_reduce / all_gather /
reduce_scatter / broadcast on device tensors, then stock DDP (unet.utils.distributed.wrap_ddp, 1 MB buckets) over
the HIP AttentionUNet, whose gradients must equal the unwrapped model's bit for bit (one rank: the bucket
all-reduce sums one contribution and divides by 1).  Prints one JSON line.  Launched by tests/test_gpu_rccl.py as
its own process (MASTER_ADDR / MASTER_PORT from the test), with NCCL_DEBUG=VERSION so the log names the library."""

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "unet-segment-pytorch_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
    out = {"backend": dist.get_backend(), "nccl_version": list(torch.cuda.nccl.version())}

    x = torch.arange(1 << 20, device=dev, dtype=torch.float32)
    y = x.clone()
    dist.all_reduce(y)
    g = [torch.empty_like(x)]
    dist.all_gather(g, x)
    r = torch.empty_like(x)
    dist.reduce_scatter(r, [x.clone()])
    b = x.clone()
    dist.broadcast(b, 0)
    torch.cuda.synchronize()
    out["collectives_exact"] = bool(torch.equal(y, x) and torch.equal(g[0], x) and torch.equal(r, x)
                                    and torch.equal(b, x))

    from unet.models import AttentionUNet
    from unet.utils.distributed import wrap_ddp
    from unet.utils.loss import DiceBCELoss
    torch.manual_seed(0)
    m = AttentionUNet(1, 2, base_features=16).to(dev).train()
    ref = AttentionUNet(1, 2, base_features=16).to(dev).train()
    ref.load_state_dict(m.state_dict())
    m.hip_precision = ref.hip_precision = "bf16"
    net = wrap_ddp(m, 0, bucket_cap_mb=1, broadcast_buffers=False)
    gen = torch.Generator().manual_seed(1)
    xin = (torch.rand(2, 1, 96, 128, generator=gen) * 2 - 1).to(dev)
    tgt = (torch.rand(2, 96, 128, generator=gen) < 0.2).long().to(dev)
    crit = DiceBCELoss()
    for _ in range(2):                      # two steps: the second reuses DDP's rebuilt buckets
        net.zero_grad(set_to_none=False)
        ref.zero_grad(set_to_none=False)
        crit(net(xin), tgt).backward()
        crit(ref(xin), tgt).backward()
    torch.cuda.synchronize()
    diff = [n for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters())
            if not torch.equal(p.grad, q.grad)]
    out["ddp_params"] = sum(1 for _ in m.parameters())
    out["ddp_grads_differing"] = diff
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
