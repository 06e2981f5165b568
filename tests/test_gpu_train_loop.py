"""The reference's training caller (row a14): `train_one_epoch` of scripts/train.py:103-161 — forward,
loss / accumulation_steps, backward, every `accumulation_steps` micro-batches clip_grad_norm_(1.0) +
AdamW.step + zero_grad, `total_loss += loss.item() * accumulation_steps`, and the leftover step when the
number of batches is not a multiple of accumulation_steps — run through the HIP path (fp32 operand mode)
and through the CPU oracle from the same seeded weights and batches (configs/lung_tumor.yaml: AdamW
lr 5e-5, weight decay 1e-4, grad clip 1.0).

Bounds: the per-micro-batch losses and the epoch average agree to fp32 noise; after the optimizer steps
every parameter agrees within 2 * lr * steps + 1e-6 (AdamW moves a parameter by at most ~lr per step,
whatever its gradient, so a parameter whose gradient is rounding noise may step in either direction in
two correct implementations) and 99 % of them within 1e-6."""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def train_one_epoch(forward, params, batches, criterion, optimizer, grad_clip, accumulation_steps):
    """scripts/train.py:103-161 (the tqdm bar and the EMA hook aside)."""
    total_loss = 0.0
    losses = []
    optimizer.zero_grad()
    for i, (images, masks) in enumerate(batches):
        outputs = forward(images)
        loss = criterion(outputs, masks) / accumulation_steps
        loss.backward()
        if (i + 1) % accumulation_steps == 0:
            if grad_clip > 0:
                torch.nn.utils.clip_grad_norm_(params, grad_clip)
            optimizer.step()
            optimizer.zero_grad()
        total_loss += loss.item() * accumulation_steps
        losses.append(loss.item() * accumulation_steps)
    if len(batches) % accumulation_steps != 0:
        if grad_clip > 0:
            torch.nn.utils.clip_grad_norm_(params, grad_clip)
        optimizer.step()
        optimizer.zero_grad()
    return total_loss / len(batches), losses


def _batches(n, dev):
    out = []
    for i in range(n):
        g = torch.Generator().manual_seed(900 + i)
        x = torch.rand(2, 1, 64, 64, generator=g) * 2 - 1
        t = torch.zeros(2, 64, 64, dtype=torch.int64)
        t[0, 10 + i:30, 12:40] = 1
        t[1, 30:52, 8 + 3 * i:30 + 3 * i] = 1
        out.append((x.to(dev), t.to(dev)))
    return out


@pytest.mark.parametrize("accum,n", [(2, 5), (3, 6)])
def test_train_one_epoch_matches_oracle(accum, n):
    from oracle import unet_oracle as O
    from unet.models import AttentionUNet
    from unet.utils.loss import DiceBCELoss
    lr, wd, clip = 5e-5, 1e-4, 1.0
    torch.manual_seed(0)
    m = AttentionUNet(1, 2, base_features=8)
    p = O.params_from_module(m)
    names = [k for k, _ in m.named_parameters()]
    m = m.cuda().train()
    m.hip_precision = "fp32"
    opt_h = torch.optim.AdamW(m.parameters(), lr=lr, weight_decay=wd)
    avg_h, l_h = train_one_epoch(m, list(m.parameters()), _batches(n, "cuda"), DiceBCELoss(), opt_h, clip, accum)
    ref_params = [p[k] for k in names]
    opt_o = torch.optim.AdamW(ref_params, lr=lr, weight_decay=wd)
    avg_o, l_o = train_one_epoch(lambda x: O.attention_unet_forward(p, x, training=True), ref_params,
                                 _batches(n, "cpu"), O.dice_bce_loss, opt_o, clip, accum)
    steps = math.ceil(n / accum)
    print(f"\navg loss HIP {avg_h:.7f} oracle {avg_o:.7f}; per batch {l_h} / {l_o}")
    for a, b in zip(l_h, l_o):
        assert abs(a - b) <= 2e-5 * abs(b) + 1e-6, (l_h, l_o)
    assert abs(avg_h - avg_o) <= 2e-5 * abs(avg_o)
    named = dict(m.named_parameters())
    diffs = torch.cat([(named[k].detach().cpu() - p[k].detach()).abs().reshape(-1) for k in names])
    frac_tight = float((diffs <= 1e-6).float().mean())
    print(f"params after {steps} steps: max |d| {float(diffs.max()):.2e}, within 1e-6: {frac_tight:.4f}")
    assert float(diffs.max()) <= 2 * lr * steps + 1e-6
    assert frac_tight >= 0.99
    bufs = dict(m.named_buffers())
    for k, v in p.items():
        if "running" in k:
            assert (bufs[k].cpu() - v).abs().max() <= 1e-4 * (1 + v.abs().max()), k
