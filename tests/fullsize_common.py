"""Shared pieces of the full-size (BASELINE-config) GPU tests: seeded batches, the oracle runs the HIP
path is measured against, gradient error summaries and the HIP run itself.

The oracle (oracle/unet_oracle.py) is the checker only: the CPU fp32 run is the reference's own
execution; the GPU fp64 run is the exact-arithmetic yardstick; the GPU autocast runs are PyTorch's own
16-bit execution of the reference network on the same weights and batch."""

from __future__ import annotations

import os

import torch


def discs(n, h, w, gen):
    """1-3 random discs of radius 6-20 px per image (SURVEY §8(d) synthetic targets)."""
    t = torch.zeros(n, h, w, dtype=torch.int64)
    yy, xx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    for i in range(n):
        for _ in range(int(torch.randint(1, 4, (1,), generator=gen))):
            cy, cx = int(torch.randint(0, h, (1,), generator=gen)), int(torch.randint(0, w, (1,), generator=gen))
            r = int(torch.randint(6, 21, (1,), generator=gen))
            t[i][(yy - cy) ** 2 + (xx - cx) ** 2 <= r * r] = 1
    return t


def forward_fn(kind: str):
    from oracle import unet_oracle as O
    return O.attention_unet_forward if kind == "attention" else O.unet_forward


def make_model(kind: str, in_ch: int):
    from unet.models import AttentionUNet, UNet
    return AttentionUNet(in_ch, 2) if kind == "attention" else UNet(in_ch, 2)


def seeded_init(kind: str, in_ch: int):
    torch.manual_seed(0)
    return {k: v.clone() for k, v in make_model(kind, in_ch).state_dict().items()}


def linear_probe(shape, seed=77):
    """fixed N(0,1) weights R for the linear loss L = mean(logits * R): dL/dlogits = R / numel exactly, so a
    gradient comparison through the network is not dominated by the conditioning of the loss"""
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g)


def _loss(out, t, loss):
    from oracle import unet_oracle as O
    if isinstance(loss, str):
        return O.dice_bce_loss(out, t)
    r = loss.to(out.device, out.dtype)
    return (out * r).sum() / out.numel()


def oracle_run(init, x, t, dev, dtype, kind="attention", training=True, autocast=None, want_eval=True,
               loss="dice_bce"):
    """The oracle's fwd + loss + bwd with the parameters/buffers of `init` on `dev` in `dtype`.
    autocast: None, or the 16-bit dtype of a torch.autocast region around the forward.  loss: "dice_bce"
    (the reference's DiceBCELoss) or a tensor R (the linear loss mean(logits * R))."""
    from oracle import unet_oracle as O
    fwd = forward_fn(kind)
    p = {}
    for k, v in init.items():
        v = v.detach().clone().to(dev)
        if v.is_floating_point():
            v = v.to(dtype)
            if "running" not in k:
                v.requires_grad_(True)
        p[k] = v
    xx = x.to(dev, dtype)
    if autocast is not None:
        with torch.autocast("cuda", dtype=autocast):
            out = fwd(p, xx, training=training)
        out = out.float()
    else:
        out = fwd(p, xx, training=training)
    loss = _loss(out, t.to(dev), loss)
    loss.backward()
    grads = {k: p[k].grad.detach().double().cpu() for k in init if p[k].requires_grad}
    bufs = {k: v.detach().cpu() for k, v in p.items() if "running" in k or "num_batches" in k}
    res = {"out": out.detach().double().cpu(), "loss": float(loss.detach()), "grads": grads, "bufs": bufs}
    if want_eval:
        with torch.no_grad():
            res["eval"] = fwd(p, xx, training=False).double().cpu()
    return res


def batch_running_stats(init, x, kind="attention"):
    """`init` with every BatchNorm's running statistics set to the batch statistics of `x` (one fp64
    train-mode pass with momentum 1, on the GPU): an eval-mode network that normalises like the train-mode
    one, so the eval-mode gradient checks see realistic activations instead of an un-normalised stack."""
    from oracle import unet_oracle as O
    p = {k: v.detach().clone().cuda().double() if v.is_floating_point() else v.detach().clone().cuda()
         for k, v in init.items()}
    old = O.BN_MOMENTUM
    O.BN_MOMENTUM = 1.0
    try:
        with torch.no_grad():
            forward_fn(kind)(p, x.cuda().double(), training=True)
    finally:
        O.BN_MOMENTUM = old
    out = {}
    for k, v in init.items():
        out[k] = p[k].to(v.dtype).cpu() if "running" in k else v.clone()
    return out


def grad_errs(grads, ref):
    """(worst max-normalised error, its name, all-parameter rel-L2) of `grads` against `ref`."""
    worst = max((float((grads[k] - g).abs().max()) / (float(g.abs().max()) + 1e-30), k) for k, g in ref.items())
    num = sum(float((grads[k] - g).pow(2).sum()) for k, g in ref.items())
    den = sum(float(g.pow(2).sum()) for g in ref.values())
    return worst[0], worst[1], (num / den) ** 0.5


def hip_model(init, prec, kind="attention", in_ch=1, training=True):
    m = make_model(kind, in_ch)
    m.load_state_dict(init)
    m = m.cuda().train(training)
    m.hip_precision = prec
    return m


def hip_run(init, x, t, prec, kind="attention", in_ch=1, training=True, log=None, env=None, loss="dice_bce"):
    """HIP fwd + loss (DiceBCE, or the linear loss of a tensor R) + bwd; `log` collects the (conv
    instantiation, output mode) pairs launched; `env` temporarily sets environment switches."""
    from unet._hip.runtime import probe
    from unet.utils.loss import DiceBCELoss
    m = hip_model(init, prec, kind, in_ch, training)
    old = {k: os.environ.get(k) for k in (env or {})}
    probe.log = log
    try:
        os.environ.update(env or {})
        out = m(x.cuda())
        if isinstance(loss, str):
            lv = DiceBCELoss()(out, t.cuda())
        else:
            lv = (out * loss.cuda()).sum() / out.numel()
        lv.backward()
        torch.cuda.synchronize()
    finally:
        probe.log = None
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    grads = {k: p.grad.detach().double().cpu() for k, p in m.named_parameters()}
    return m, out.detach(), float(lv.detach()), grads


def rel_l2(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def report16(name, out, loss, grads, f64):
    e = rel_l2(out, f64["out"])
    agree = float((out.double().cpu().argmax(1) == f64["out"].argmax(1)).double().mean())
    lrel = abs(loss - f64["loss"]) / abs(f64["loss"])
    w, k, r = grad_errs(grads, f64["grads"])
    print(f"{name}: logits rel-L2 {e:.3e} argmax agreement {agree:.6f} loss rel {lrel:.1e} | grads all rel-L2 "
          f"{r:.3e} worst max-norm {w:.2e} ({k})")
    return e, agree, lrel, r
