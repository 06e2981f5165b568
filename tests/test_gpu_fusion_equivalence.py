"""The backward fusions of round 2 change where an addition happens, not what is added: with the
MaxPool2d gradient folded into the BatchNorm backward (unet_bn_bwd_*_pool) and the attention gate's x*s
term added by the W_x dgrad (UNET_OUT_F32_GATED), every parameter gradient must be bit-identical to the
unfused path (the pool-routing dgrad epilogue's read-modify-write; gate pass 1 writing dx).  The switches
UNET_NO_POOL_FOLD / UNET_NO_GATE_FUSE select the unfused path at run time."""

import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _grads(model, x, t, env, seen=None):
    from unet._hip import lib as L
    from unet.utils.loss import DiceBCELoss
    old = {k: os.environ.get(k) for k in ("UNET_NO_POOL_FOLD", "UNET_NO_GATE_FUSE")}
    orig = L.call

    def rec(name, *args):
        if seen is not None:
            seen.add(name if name != "unet_conv" else f"unet_conv:{args[0].out_mode}")
        return orig(name, *args)

    L.call = rec
    try:
        for k in old:
            os.environ.pop(k, None)
        os.environ.update(env)
        model.zero_grad(set_to_none=True)
        out = model(x)
        DiceBCELoss()(out, t).backward()
        torch.cuda.synchronize()
        return out.detach().clone(), {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    finally:
        L.call = orig
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("prec", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("size", [128, 98])
def test_fused_backward_bit_identical(prec, size):
    """base 64 at 2 x 128^2: the top gate's W_x dgrad (32 -> 64 channels, 32768 pixels) runs on the 1x1
    kernel that serves the gated epilogue; 98^2 has odd pooled maps below 49^2 (last row / column without
    a window)."""
    from unet.models import AttentionUNet
    torch.manual_seed(3)
    m = AttentionUNet(1, 2, base_features=64).cuda().train()
    m.hip_precision = prec
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(2, 1, size, size, generator=g) * 2 - 1).cuda()
    t = (torch.rand(2, size, size, generator=g) < 0.1).long().cuda()
    state = {k: v.clone() for k, v in m.state_dict().items()}
    seen0, seen1 = set(), set()
    out0, g0 = _grads(m, x, t, {}, seen0)
    m.load_state_dict(state)   # the same BN running statistics going in
    out1, g1 = _grads(m, x, t, {"UNET_NO_POOL_FOLD": "1", "UNET_NO_GATE_FUSE": "1"}, seen1)
    assert "unet_bn_bwd_reduce_pool" in seen0 and "unet_bn_bwd_reduce_pool" not in seen1
    assert ("unet_conv:4" in seen0) == (prec != "fp32" and size == 128), sorted(seen0)
    assert "unet_conv:4" not in seen1 and "unet_conv:2" in seen1
    assert torch.equal(out0, out1)
    diff = [n for n in g0 if not torch.equal(g0[n], g1[n])]
    assert not diff, diff
