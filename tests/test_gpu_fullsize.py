"""Full-size parity at the benchmark's configuration (BASELINE C3): AttentionUNet(1, 2), base 64,
batch 4 x 1 x 512 x 512, train-mode forward + DiceBCE + backward (reference unet.py:175-211,
loss.py:153-191), HIP path vs the CPU oracle on the same seeded weights and inputs.

At this size the dispatcher picks the same kernel instantiations as `bench.py` (conv5 on the large maps, the
conv3 tiles on the 32^2 / 64^2 ones, the persistent multi-tile loops, wgrad2 with >32 split-K slabs, the
pointwise gate kernels); the 16-bit tests assert that no fallback kernel ran and that conv5 did.

Gates:
  fp32 operand mode, against the CPU fp32 oracle (the reference's own execution) — logits within 1e-4
  abs; argmax identical except pixels whose oracle margin |z1 - z0| < 1e-4 (count reported); confusion
  matrix (device kernel on our logits) equal to the oracle's up to those pixels; loss within 1e-5 rel;
  BN running buffers within 1e-4; eval-mode logits within 1e-4 (1 + max).  Parameter gradients against
  the fp64 oracle: no worse than 1.5x the CPU fp32 oracle's own error.
  bf16 / fp16 operand modes — see test_fullsize_16bit_vs_oracle: no worse than PyTorch's own 16-bit execution.
"""

import os

import pytest
import torch

from hip_helpers import max_abs, rel_err

pytestmark = pytest.mark.gpu

N, S = 4, 512


def _discs(n, h, w, gen):
    t = torch.zeros(n, h, w, dtype=torch.int64)
    yy, xx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    for i in range(n):
        for _ in range(int(torch.randint(1, 4, (1,), generator=gen))):
            cy, cx = int(torch.randint(0, h, (1,), generator=gen)), int(torch.randint(0, w, (1,), generator=gen))
            r = int(torch.randint(6, 21, (1,), generator=gen))
            t[i][(yy - cy) ** 2 + (xx - cx) ** 2 <= r * r] = 1
    return t


def _oracle(init, x, t, dev, dtype, autocast=False):
    """The oracle's fwd + DiceBCE + bwd with the parameters/buffers of `init` on `dev` in `dtype`
    (autocast=True / a 16-bit dtype: the reference's network under torch.autocast(bf16 / that dtype),
    i.e. PyTorch's own 16-bit run)."""
    from oracle import unet_oracle as O
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
        with torch.autocast("cuda", dtype=torch.bfloat16 if autocast is True else autocast):
            out = O.attention_unet_forward(p, xx, training=True)
        out = out.float()
    else:
        out = O.attention_unet_forward(p, xx, training=True)
    loss = O.dice_bce_loss(out, t.to(dev))
    loss.backward()
    grads = {k: p[k].grad.detach().double().cpu() for k in init if p[k].requires_grad}
    bufs = {k: v.detach().cpu() for k, v in p.items() if "running" in k or "num_batches" in k}
    with torch.no_grad():
        ev = O.attention_unet_forward(p, xx, training=False).double().cpu()
    return {"out": out.detach().double().cpu(), "loss": float(loss.detach()), "grads": grads, "bufs": bufs,
            "eval": ev}


def _grad_errs(grads, ref):
    """(worst max-normalised error, its name, all-parameter rel-L2) of `grads` against `ref`."""
    worst = max((float((grads[k] - g).abs().max()) / (float(g.abs().max()) + 1e-30), k) for k, g in ref.items())
    num = sum(float((grads[k] - g).pow(2).sum()) for k, g in ref.items())
    den = sum(float(g.pow(2).sum()) for g in ref.values())
    return worst[0], worst[1], (num / den) ** 0.5


@pytest.fixture(scope="module")
def full_ref():
    """Seeded weights / batch; the oracle in fp32 on the CPU (the reference's own execution), in fp64
    (ATen on the GPU: the exact-arithmetic yardstick) and under torch.autocast(bf16) on the GPU."""
    from unet.models import AttentionUNet
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    torch.manual_seed(0)
    init = {k: v.clone() for k, v in AttentionUNet(1, 2).state_dict().items()}
    g = torch.Generator().manual_seed(2024)
    x = torch.rand(N, 1, S, S, generator=g) * 2 - 1
    t = _discs(N, S, S, g)
    return {"init": init, "x": x, "t": t,
            "cpu32": _oracle(init, x, t, "cpu", torch.float32),
            "f64": _oracle(init, x, t, "cuda", torch.float64),
            "ac16": _oracle(init, x, t, "cuda", torch.float32, autocast=True)}


def _model(ref, prec):
    from unet.models import AttentionUNet
    m = AttentionUNet(1, 2)
    m.load_state_dict(ref["init"])
    m = m.cuda().train()
    m.hip_precision = prec
    return m


def _run(ref, prec, log=None):
    from unet._hip.runtime import probe
    from unet.utils.loss import DiceBCELoss
    m = _model(ref, prec)
    probe.log = log
    try:
        out = m(ref["x"].cuda())
        loss = DiceBCELoss()(out, ref["t"].cuda())
        loss.backward()
        torch.cuda.synchronize()
    finally:
        probe.log = None
    return m, out.detach(), float(loss.detach())


def test_fullsize_fp32_vs_oracle(full_ref):
    from unet.utils.metrics import SegmentationMetrics
    from oracle import unet_oracle as O
    ref, c32, f64 = full_ref, full_ref["cpu32"], full_ref["f64"]
    m, out, loss = _run(ref, "fp32")
    z, zr = out.double().cpu(), c32["out"]
    e = float((z - zr).abs().max())
    margin = (zr[:, 1] - zr[:, 0]).abs()
    flips = z.argmax(1) != zr.argmax(1)
    near = int((flips & (margin < 1e-4)).sum())
    hard = int((flips & (margin >= 1e-4)).sum())
    sm = SegmentationMetrics(2)
    sm.update(out, ref["t"].cuda())
    cm_ref = O.confusion_matrix(zr.argmax(1), ref["t"]).numpy()
    cm_diff = int(abs(sm.get_confusion_matrix() - cm_ref).sum())
    print(f"\nfp32 full-size: logits max|d| {e:.2e} (absmax {float(zr.abs().max()):.2f}); argmax flips "
          f"{near} near-tie / {hard} other of {zr[:, 0].numel()}; confusion |d| {cm_diff}; loss {loss:.7f} vs "
          f"{c32['loss']:.7f}")
    assert e <= 1e-4, e                                   # logits within 1e-4 (north_star)
    assert hard == 0, hard
    assert cm_diff <= 2 * near, (cm_diff, near)
    assert abs(loss - c32["loss"]) <= 1e-5 * abs(c32["loss"])
    # parameter gradients: at this size the reference's own fp32 execution is not exact (BN over a 4x32x32
    # batch, long reductions): measured against the fp64 oracle, the CPU fp32 oracle's worst max-normalised
    # gradient error is ~4e-2 (down4.0 weight).  Gate: ours no worse than 1.5x the reference's own fp32 error.
    named = dict(m.named_parameters())
    mine = {k: p.grad.detach().double().cpu() for k, p in named.items()}
    w_h, k_h, r_h = _grad_errs(mine, f64["grads"])
    w_c, k_c, r_c = _grad_errs(c32["grads"], f64["grads"])
    print(f"fp32 full-size grads vs fp64 oracle: ours worst {w_h:.2e} ({k_h}) all rel-L2 {r_h:.2e}; "
          f"CPU fp32 oracle worst {w_c:.2e} ({k_c}) all rel-L2 {r_c:.2e}")
    assert w_h <= 1.5 * w_c + 1e-4, (w_h, k_h, w_c)
    assert r_h <= 1.5 * r_c + 1e-4, (r_h, r_c)
    bufs = dict(m.named_buffers())
    for k, b in c32["bufs"].items():
        assert max_abs(bufs[k].float(), b.float()) <= 1e-4 * (1 + float(b.float().abs().max())), k
    m.eval()
    with torch.no_grad():
        ev = m(ref["x"].cuda())
    ee = max_abs(ev, c32["eval"])
    print(f"fp32 full-size: eval logits max|d| {ee:.2e} (absmax {float(c32['eval'].abs().max()):.2f})")
    assert ee <= 1e-4 * (1 + float(c32["eval"].abs().max())), ee


def _bf16_report(name, out, loss, grads, f64):
    e = rel_err(out, f64["out"])
    agree = float((out.double().cpu().argmax(1) == f64["out"].argmax(1)).double().mean())
    lrel = abs(loss - f64["loss"]) / abs(f64["loss"])
    w, k, r = _grad_errs(grads, f64["grads"])
    print(f"{name}: logits rel-L2 {e:.3e} argmax agreement {agree:.6f} loss rel {lrel:.1e} | grads all rel-L2 "
          f"{r:.3e} worst max-norm {w:.2e} ({k})")
    return e, agree, lrel, r


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_fullsize_16bit_vs_oracle(full_ref, prec):
    """bf16 operand mode at the bench configuration, against the fp64 oracle, beside PyTorch's own bf16
    execution of the reference network (torch.autocast on the GPU) on the same weights and batch.
    SURVEY §8(d) proposed rel-L2 <= 1e-2 on the logits; measured here, autocast-bf16 itself is at ~0.14
    (argmax agreement ~0.960): the random-init network with train-mode BN over 4 images amplifies bf16
    rounding (it is not a kernel error: the fp32 mode of the same kernels is at 2e-5).  The gate is
    therefore: no worse than PyTorch's bf16 (logits rel-L2 and gradient rel-L2 within 1.1x + small,
    argmax agreement within 0.5 %), loss within 1e-2 rel (measured ~1e-3), plus absolute ceilings."""
    ref, f64 = full_ref, full_ref["f64"]
    ac = full_ref["ac16"] if prec == "bf16" else _oracle(ref["init"], ref["x"], ref["t"], "cuda", torch.float32,
                                                         autocast=torch.float16)
    log = []
    m, out, loss = _run(ref, prec, log)
    from test_gpu_configs import _assert_16bit_paths
    _assert_16bit_paths(log, prec)
    grads = {k: p.grad.detach().double().cpu() for k, p in m.named_parameters()}
    print()
    e, agree, lrel, r = _bf16_report(f"{prec} HIP      ", out, loss, grads, f64)
    e_a, agree_a, lrel_a, r_a = _bf16_report(f"{prec} autocast ", ac["out"], ac["loss"], ac["grads"], f64)
    assert e <= 1.1 * e_a + 5e-3 and e <= 0.2, (e, e_a)
    assert agree >= agree_a - 5e-3 and agree >= 0.95, (agree, agree_a)
    assert lrel <= 1e-2, lrel
    assert r <= 1.1 * r_a + 2e-2 and r <= 0.7, (r, r_a)
    # eval mode (running statistics, no batch-statistics amplification)
    m.eval()
    with torch.no_grad():
        ev = m(ref["x"].cuda())
    ee = rel_err(ev, f64["eval"])
    print(f"{prec} HIP eval-mode logits rel-L2 {ee:.3e}; autocast eval {rel_err(ac['eval'], f64['eval']):.3e}")
    assert ee <= 1e-2, ee        # SURVEY §8(d)'s bf16 logits gate holds once BN uses running statistics
