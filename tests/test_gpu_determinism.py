"""Run-to-run determinism of the whole training step (SURVEY §5 determinism row; round-2 verdict: "no
double-run determinism test of the training step").

The same seeded model trained twice on the same batches (scripts/train.py:127-143: forward, DiceBCE,
backward, clip_grad_norm_(1.0), AdamW) must give bit-identical losses, parameter gradients and weights:
every reduction in the path is fixed-order (split-K weight-gradient slabs summed by one launch in slab
order, BN / loss / gate partial sums per block then finalised in block order) and no float atomics are
used.  At the bench size the conv5 / wgrad5 / smallcin MFMA kernels and the LDS-DMA pipelines all run,
so a race in one of them (an LDS slot consumed before its DMA landed, a missing barrier) shows up here as
a flipped bit between the two runs."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(model_kind, prec, shape, base, steps, seed=0):
    from unet.models import AttentionUNet, UNet
    from unet.utils.loss import DiceBCELoss
    torch.manual_seed(seed)
    cls = AttentionUNet if model_kind == "attention" else UNet
    m = cls(shape[1], 2, base_features=base).cuda().train()
    m.hip_precision = prec
    opt = torch.optim.AdamW(m.parameters(), lr=5e-5, weight_decay=1e-4, fused=True)
    crit = DiceBCELoss()
    g = torch.Generator().manual_seed(seed + 1)
    losses, grads = [], None
    for _ in range(steps):
        x = (torch.rand(*shape, generator=g) * 2 - 1).cuda()
        t = (torch.rand(shape[0], shape[2], shape[3], generator=g) < 0.1).long().cuda()
        opt.zero_grad(set_to_none=True)
        loss = crit(m(x), t)
        loss.backward()
        grads = [p.grad.clone() for p in m.parameters()]
        torch.nn.utils.clip_grad_norm_(list(m.parameters()), 1.0)
        opt.step()
        losses.append(loss.detach().clone())
    torch.cuda.synchronize()
    return losses, grads, {k: v.clone() for k, v in m.state_dict().items()}


@pytest.mark.parametrize("model_kind,prec,shape,base", [
    ("attention", "bf16", (4, 1, 512, 512), 64),      # C3, the bench configuration
    ("unet", "bf16", (4, 1, 512, 512), 64),           # C2
    ("attention", "fp16", (1, 3, 1024, 1024), 64),    # C5's image size and input channels
    ("attention", "fp32", (2, 1, 256, 256), 32),
], ids=["c3-bf16", "c2-bf16", "c5-fp16", "fp32"])
def test_train_step_bit_identical_across_runs(model_kind, prec, shape, base):
    la, ga, sa = _train(model_kind, prec, shape, base, steps=2)
    lb, gb, sb = _train(model_kind, prec, shape, base, steps=2)
    for i, (a, b) in enumerate(zip(la, lb)):
        assert torch.isfinite(a) and torch.equal(a, b), (i, float(a), float(b))
    for i, (a, b) in enumerate(zip(ga, gb)):
        assert torch.equal(a, b), (i, float((a - b).abs().max()))
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
