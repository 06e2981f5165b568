"""Full-size numerics diagnostic (not a test): AttentionUNet(1, 2) base 64, 4x1x512^2, train-mode
fwd + DiceBCE + bwd.  Every implementation is compared against the oracle run in fp64 on the GPU:
  oracle fp32 on the CPU (oneDNN), oracle fp32 on the GPU (MIOpen), oracle under torch.autocast(bf16)
  on the GPU, and the HIP path in fp32 and bf16 operand modes.
Prints logits max|d| / rel-L2, argmax agreement, loss rel, worst max-normalised parameter-gradient error
and the all-parameter gradient rel-L2.  Usage: python tools/fullsize_diag.py [batch]"""

import os
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "unet-segment-pytorch_amd"))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT))

from oracle import unet_oracle as O  # noqa: E402
from test_gpu_fullsize import _discs  # noqa: E402


def oracle(init, x, t, dev, dtype, autocast=False):
    p = {}
    for k, v in init.items():
        v = v.detach().clone().to(dev)
        if v.is_floating_point():
            v = v.to(dtype)
            if "running" not in k:
                v.requires_grad_(True)
        p[k] = v
    xx = x.to(dev, dtype)
    if autocast:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = O.attention_unet_forward(p, xx, training=True)
        out = out.float()
    else:
        out = O.attention_unet_forward(p, xx, training=True)
    loss = O.dice_bce_loss(out, t.to(dev))
    loss.backward()
    grads = {k: p[k].grad.detach().double().cpu() for k in init if k in p and p[k].grad is not None}
    return out.detach().double().cpu(), float(loss), grads


def hip(init, x, t, prec):
    from unet.models import AttentionUNet
    from unet.utils.loss import DiceBCELoss
    m = AttentionUNet(1, 2)
    m.load_state_dict(init)
    m = m.cuda().train()
    m.hip_precision = prec
    out = m(x.cuda())
    loss = DiceBCELoss()(out, t.cuda())
    loss.backward()
    grads = {k: p.grad.detach().double().cpu() for k, p in m.named_parameters()}
    return out.detach().double().cpu(), float(loss), grads


def report(name, res, ref):
    out, loss, grads = res
    ro, rl, rg = ref
    d = out - ro
    agree = float((out.argmax(1) == ro.argmax(1)).double().mean())
    worst = max((float((grads[k] - g).abs().max()) / (float(g.abs().max()) + 1e-30), k) for k, g in rg.items())
    num = sum(float((grads[k] - g).pow(2).sum()) for k, g in rg.items())
    den = sum(float(g.pow(2).sum()) for g in rg.values())
    rels = sorted(((float((grads[k] - g).norm() / (g.norm() + 1e-30)), k) for k, g in rg.items()), reverse=True)
    print(f"[{name:>14}] logits max|d| {float(d.abs().max()):.2e} rel-L2 {float(d.norm() / ro.norm()):.2e} "
          f"argmax-agree {agree:.6f} loss-rel {abs(loss - rl) / abs(rl):.1e} | grads: worst max-norm "
          f"{worst[0]:.2e} ({worst[1]}) all rel-L2 {(num / den) ** 0.5:.2e}; worst rel-L2 "
          f"{rels[0][0]:.2e} ({rels[0][1]}), {rels[1][0]:.2e} ({rels[1][1]})", flush=True)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    from unet.models import AttentionUNet
    torch.manual_seed(0)
    init = {k: v.clone() for k, v in AttentionUNet(1, 2).state_dict().items()}
    g = torch.Generator().manual_seed(2024)
    x = torch.rand(n, 1, 512, 512, generator=g) * 2 - 1
    t = _discs(n, 512, 512, g)
    t0 = time.time()
    ref = oracle(init, x, t, "cuda", torch.float64)
    print(f"fp64 oracle on the GPU: {time.time() - t0:.1f} s, loss {ref[1]:.8f}", flush=True)
    report("oracle gpu f32", oracle(init, x, t, "cuda", torch.float32), ref)
    report("oracle ac-bf16", oracle(init, x, t, "cuda", torch.float32, autocast=True), ref)
    report("hip fp32", hip(init, x, t, "fp32"), ref)
    report("hip bf16", hip(init, x, t, "bf16"), ref)
    t0 = time.time()
    report("oracle cpu f32", oracle(init, x, t, "cpu", torch.float32), ref)
    print(f"cpu oracle: {time.time() - t0:.1f} s", flush=True)


if __name__ == "__main__":
    main()
