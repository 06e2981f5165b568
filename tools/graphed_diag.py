"""Diagnostic (GPU): per-step losses of the eager step, the eager step run through functional_call on leaf
aliases (no graph, parameters swapped around forward and backward), and GraphedTrainStep, from the same weights; prints the first differing step and any
parameter whose alias gradient is None."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "unet-segment-pytorch_amd"))
import torch  # noqa: E402

from unet.models import AttentionUNet  # noqa: E402
from unet.utils.graphed import GraphedTrainStep, _swapped_parameters  # noqa: E402
from unet.utils.loss import DiceBCELoss  # noqa: E402


def make():
    torch.manual_seed(0)
    m = AttentionUNet(1, 2, base_features=16).cuda().train()
    m.hip_precision = "bf16"
    return m


def main():
    ms = [make() for _ in range(3)]
    for m in ms[1:]:
        m.load_state_dict(ms[0].state_dict())
    opts = [torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=1e-4, fused=True, capturable=True) for m in ms]
    crit = DiceBCELoss()
    g = torch.Generator().manual_seed(3)
    batches = [((torch.rand(2, 1, 128, 128, generator=g) * 2 - 1).cuda(),
                (torch.rand(2, 128, 128, generator=g) < 0.1).long().cuda()) for _ in range(3)]
    gs = GraphedTrainStep(ms[2], crit, opts[2], (2, 1, 128, 128), (2, 128, 128))
    named = [(n, p) for n, p in ms[1].named_parameters()]
    leaves = {n: p.detach().requires_grad_(True) for n, p in named}
    for i, (x, t) in enumerate(batches):
        # eager
        opts[0].zero_grad(set_to_none=True)
        l0 = crit(ms[0](x), t)
        l0.backward()
        torch.nn.utils.clip_grad_norm_(list(ms[0].parameters()), 1.0)
        # functional_call on aliases
        opts[1].zero_grad(set_to_none=True)
        with _swapped_parameters(ms[1], leaves):
            l1 = crit(ms[1](x), t)
            grads = torch.autograd.grad(l1, list(leaves.values()), allow_unused=True)
        none = [n for (n, _), gr in zip(named, grads) if gr is None]
        for (_, p), gr in zip(named, grads):
            p.grad = gr
        torch.nn.utils.clip_grad_norm_(list(ms[1].parameters()), 1.0)
        gdiff = [n for (n, p0), (_, p1) in zip(ms[0].named_parameters(), named)
                 if p1.grad is None or not torch.equal(p0.grad, p1.grad)]
        opts[0].step()
        opts[1].step()
        l2 = gs(x, t).clone()
        torch.cuda.synchronize()
        print(f"step {i}: eager {float(l0):.9f} alias {float(l1):.9f} graph {float(l2):.9f}; alias grads None: "
              f"{none[:5]}; alias grads differing from eager: {len(gdiff)} {gdiff[:5]}", flush=True)
        gd = [n for (n, p0), (_, p2) in zip(ms[0].named_parameters(), ms[2].named_parameters())
              if p2.grad is None or not torch.equal(p0.grad, p2.grad)]
        print(f"   graph grads differing from eager: {len(gd)} {gd[:6]}", flush=True)
        wd = [n for (n, p0), (_, p2) in zip(ms[0].named_parameters(), ms[2].named_parameters()) if not torch.equal(p0, p2)]
        print(f"   weights differing eager vs graph after step: {len(wd)} {wd[:6]}", flush=True)


if __name__ == "__main__":
    main()
