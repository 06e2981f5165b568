"""Host-side cost of one bench step: CPU time to enqueue it (GPU idle at the start) vs its GPU time."""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "unet-segment-pytorch_amd"))
sys.path.insert(0, str(ROOT))
import torch
from bench import disc_targets
from unet.models import AttentionUNet
from unet.utils.loss import DiceBCELoss

torch.manual_seed(0)
dev = torch.device("cuda", 0)
m = AttentionUNet(1, 2).to(dev).train()
m.hip_precision = "bf16"
opt = torch.optim.AdamW(m.parameters(), lr=5e-5, weight_decay=1e-4, fused=True)
crit = DiceBCELoss()
g = torch.Generator().manual_seed(1)
x = (torch.rand(4, 1, 512, 512, generator=g) * 2 - 1).to(dev)
t = disc_targets(4, 512, 512, g).to(dev)
params = list(m.parameters())


def fwd():
    return crit(m(x), t)


def fwd_bwd():
    crit(m(x), t).backward()


def step():
    crit(m(x), t).backward()
    torch.nn.utils.clip_grad_norm_(params, 1.0)
    opt.step()
    opt.zero_grad(set_to_none=True)


for name, fn in (("forward", fwd), ("fwd+bwd", fwd_bwd), ("step", step)):
    for _ in range(3):
        fn()
    cpu, tot = [], []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        cpu.append(t1 - t0)
        tot.append(t2 - t0)
    opt.zero_grad(set_to_none=True)
    print(f"{name:8s}: host enqueue {min(cpu) * 1e3:7.3f} ms, enqueue+drain {min(tot) * 1e3:7.3f} ms", flush=True)

# the same step captured once and replayed (unet.utils.graphed.GraphedTrainStep; capturable fused AdamW)
from unet.utils.graphed import GraphedTrainStep
torch.manual_seed(0)
m2 = AttentionUNet(1, 2).to(dev).train()
m2.hip_precision = "bf16"
opt2 = torch.optim.AdamW(m2.parameters(), lr=5e-5, weight_decay=1e-4, fused=True, capturable=True)
gs = GraphedTrainStep(m2, crit, opt2, x.shape, t.shape)
for _ in range(3):
    gs(x, t)
cpu, tot = [], []
for _ in range(10):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gs(x, t)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    cpu.append(t1 - t0)
    tot.append(t2 - t0)
print(f"{'graphed':8s}: host enqueue {min(cpu) * 1e3:7.3f} ms, enqueue+drain {min(tot) * 1e3:7.3f} ms", flush=True)
for name, fn in (("eager step", step), ("graphed step", lambda: gs(x, t))):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(30):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 30
    print(f"{name:12s}: {dt * 1e3:7.3f} ms/step back to back = {4 / dt:7.1f} img/s", flush=True)
