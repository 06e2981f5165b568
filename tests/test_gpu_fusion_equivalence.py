"""The backward fusions of round 2 change where an addition happens, not what is added: with the
MaxPool2d gradient folded into the BatchNorm backward (unet_bn_bwd_*_pool) and the attention gate's x*s
term added by the W_x dgrad (UNET_OUT_F32_GATED), every parameter gradient must be bit-identical to the
unfused path (the pool-routing dgrad epilogue's read-modify-write; gate pass 1 writing dx).  The switches
UNET_NO_POOL_FOLD / UNET_NO_GATE_FUSE select the unfused path at run time."""

import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _grads(model, x, t, env, seen=None, split=False):
    from unet._hip import lib as L
    from unet.utils.loss import DiceBCELoss
    old = {k: os.environ.get(k) for k in ("UNET_NO_POOL_FOLD", "UNET_NO_GATE_FUSE", "UNET_NO_ACT_OUT", "UNET_NO_OC_FUSE",
                                         "UNET_NO_GATE_VEC", "UNET_CONV5_SPLIT")}
    orig = L.call

    def rec(name, *args):
        if seen is not None:
            seen.add(name if name != "unet_conv" else f"unet_conv:{args[0].out_mode}")
            if name == "unet_conv" and args[0].workspace:
                seen.add("splitk")
            if name == "unet_conv_wgrad" and args[0].ksize == 3:
                seen.add(f"wgrad3:src0kind={args[0].src[0].kind}")
        return orig(name, *args)

    L.call = rec
    try:
        for k in old:
            os.environ.pop(k, None)
        # split-K (round 5) sums a small-map conv's reduction in a different order; the pooled dgrad of the fused
        # path is one of them and the pool-routing epilogue of the unfused path is not, so both runs here keep the
        # unsplit form: what these tests compare is where the fusions add, not the conv's summation order
        if not split:
            os.environ["UNET_CONV5_SPLIT"] = "0"
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
    kernel that serves the gated epilogue (at 98^2 too since round 6: 19208 pixels); 98^2 has odd pooled maps
    below 49^2 (last row / column without a window)."""
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
    # the gated W_x dgrad runs on the 1x1 kernel from 16384 pixels (csrc/pw.hip pw_conv_ok; 32768 before round 6)
    assert ("unet_conv:4" in seen0) == (prec != "fp32" and 2 * size * size >= 16384), sorted(seen0)
    assert "unet_conv:4" not in seen1 and "unet_conv:2" in seen1
    assert torch.equal(out0, out1)
    diff = [n for n in g0 if not torch.equal(g0[n], g1[n])]
    assert not diff, diff


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_fusions_with_splitk_on(prec):
    """The production configuration: split-K on for the small maps in both runs.  The gate
    fusion (the x*s term added by the W_x dgrad) does not touch a split conv, so its gradients stay bit-identical
    with split-K on; the pool fold does — the fused path's pooled dgrad is a split-K conv, the unfused path's
    pool-routing epilogue is not split — so there the same sums in another order, equal up to the 16-bit
    roundings such a reorder flips downstream (gated as test_outconv_bn_backward_fused's 16-bit case)."""
    from unet.models import AttentionUNet
    torch.manual_seed(3)
    m = AttentionUNet(1, 2, base_features=64).cuda().train()
    m.hip_precision = prec
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(2, 1, 128, 128, generator=g) * 2 - 1).cuda()
    t = (torch.rand(2, 128, 128, generator=g) < 0.1).long().cuda()
    state = {k: v.clone() for k, v in m.state_dict().items()}
    seen0, seen1, seen2 = set(), set(), set()
    out0, g0 = _grads(m, x, t, {}, seen0, split=True)
    m.load_state_dict(state)
    out1, g1 = _grads(m, x, t, {"UNET_NO_GATE_FUSE": "1"}, seen1, split=True)
    m.load_state_dict(state)
    out2, g2 = _grads(m, x, t, {"UNET_NO_POOL_FOLD": "1"}, seen2, split=True)
    assert "splitk" in seen0 and "splitk" in seen1 and "splitk" in seen2, sorted(seen0)
    assert "unet_conv:4" in seen0 and "unet_conv:4" not in seen1
    assert "unet_bn_bwd_reduce_pool" in seen0 and "unet_bn_bwd_reduce_pool" not in seen2
    assert torch.equal(out0, out1) and torch.equal(out0, out2)
    diff = [n for n in g0 if not torch.equal(g0[n], g1[n])]
    assert not diff, diff
    a = torch.cat([g0[n].double().flatten() for n in g0])
    b = torch.cat([g2[n].double().flatten() for n in g0])
    assert float((a - b).norm() / b.norm()) <= 1e-2
    for n in g0:
        if g0[n].numel() < 16:
            continue    # a 1-channel BN's gamma / beta gradient (see test_outconv_bn_backward_fused)
        d = float((g0[n].double() - g2[n].double()).abs().max() / (g2[n].double().abs().max() + 1e-30))
        assert d <= 0.1, (n, d)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_act_out_wgrad_equivalent(prec):
    """The forward conv writes its transformed BN-activation input once (unet_conv act_out, conv5) and the
    3x3 weight gradients read that stored map instead of re-applying BN + ReLU (+ the attention gate): the
    same 16-bit values, so the logits and every gradient that is not a 3x3 conv weight are bit-identical to
    the re-transforming path (UNET_NO_ACT_OUT); the 3x3 weight gradients agree to fp32 summation order (a
    stored-source wgrad may walk taller pixel stages).  2 x 256^2, base 64: the 256^2 convs run on conv5."""
    from unet.models import AttentionUNet
    torch.manual_seed(4)
    m = AttentionUNet(1, 2, base_features=64).cuda().train()
    m.hip_precision = prec
    g = torch.Generator().manual_seed(6)
    x = (torch.rand(2, 1, 256, 256, generator=g) * 2 - 1).cuda()
    t = (torch.rand(2, 256, 256, generator=g) < 0.1).long().cuda()
    state = {k: v.clone() for k, v in m.state_dict().items()}
    seen0, seen1 = set(), set()
    out0, g0 = _grads(m, x, t, {}, seen0)
    m.load_state_dict(state)
    out1, g1 = _grads(m, x, t, {"UNET_NO_ACT_OUT": "1"}, seen1)
    from unet._hip import lib as L
    plain, act = f"wgrad3:src0kind={L.SRC_PLAIN}", f"wgrad3:src0kind={L.SRC_ACT}"
    assert plain in seen0 and act in seen1, (sorted(seen0), sorted(seen1))
    assert torch.equal(out0, out1)
    names = dict(m.named_parameters())
    for n in g0:
        if names[n].dim() == 4 and names[n].shape[-1] == 3:
            rel = float((g0[n] - g1[n]).double().norm() / g1[n].double().norm())
            assert rel <= 1e-5, (n, rel)
        else:
            assert torch.equal(g0[n], g1[n]), n


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("kind", ["attention", "unet"])
def test_outconv_bn_backward_fused(prec, kind):
    """OutConv's backward fused with the BN backward of its input (unet_outconv_bwd_bn + unet_bn_bwd_apply_oc:
    the activation gradient W^T dl is recomputed, never stored) against the stored-gradient path
    (UNET_NO_OC_FUSE): the same sums in another order, so equal up to fp32 rounding (fp32 mode), and up to
    the 16-bit rounding of the dgrad operand that this reorder can flip (bf16 mode)."""
    from unet.models import AttentionUNet, UNet
    torch.manual_seed(7)
    m = (AttentionUNet(1, 2, base_features=16) if kind == "attention" else UNet(1, 2, base_features=16)).cuda().train()
    m.hip_precision = prec
    g = torch.Generator().manual_seed(8)
    x = (torch.rand(2, 1, 96, 128, generator=g) * 2 - 1).cuda()
    t = (torch.rand(2, 96, 128, generator=g) < 0.1).long().cuda()
    state = {k: v.clone() for k, v in m.state_dict().items()}
    seen0, seen1 = set(), set()
    out0, g0 = _grads(m, x, t, {}, seen0)
    m.load_state_dict(state)
    out1, g1 = _grads(m, x, t, {"UNET_NO_OC_FUSE": "1"}, seen1)
    assert "unet_outconv_bwd_bn" in seen0 and "unet_bn_bwd_apply_oc" in seen0
    assert "unet_outconv_bwd_bn" not in seen1
    assert torch.equal(out0, out1)
    if prec == "fp32":
        for n in g0:
            a, b = g0[n].double(), g1[n].double()
            rel = float((a - b).norm() / (b.norm() + 1e-30))
            assert rel <= 1e-4, (n, rel)
    else:
        # 16-bit: a reordered BN sum can flip the rounding of a 16-bit dgrad operand, and the attention psi
        # BatchNorm's scalar parameters are sums with heavy cancellation (the BN-sums fusion's own test sees
        # the same: all params rel-L2 6e-3, worst tensor 5e-2) — gate the whole gradient and each tensor's
        # largest deviation
        a = torch.cat([g0[n].double().flatten() for n in g0])
        b = torch.cat([g1[n].double().flatten() for n in g0])
        assert float((a - b).norm() / b.norm()) <= 1e-2
        for n in g0:
            if g0[n].numel() < 16:
                # a 1-channel BN's gamma / beta gradient (psi): ONE sum over all pixels, whose relative change
                # under a 16-bit rounding flip upstream is unbounded where the sum cancels (0.19 on up1's psi gamma
                # at 16^2 once round 5 moved a BN-statistics summation order); the all-parameter rel-L2 covers it
                continue
            d = float((g0[n].double() - g1[n].double()).abs().max() / (g1[n].double().abs().max() + 1e-30))
            assert d <= 0.1, (n, d)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("base,size", [(16, 96), (64, 128)])
def test_gate_vec_passes_equivalent(prec, base, size):
    """Attention-gate backward passes 2 / 3 in the coalesced form (gate_bwd2_vec / gate_bwd3_vec: 8 channels
    per lane) against the per-channel kernels (UNET_NO_GATE_VEC): pass 3 evaluates the same per-element
    expressions, pass 2 sums the same terms in another fixed order — equal up to fp32 rounding (fp32 mode),
    and up to the 16-bit roundings such a reorder can flip downstream (bf16 mode; gates as for the OutConv
    fusion above)."""
    from unet.models import AttentionUNet
    torch.manual_seed(9)
    m = AttentionUNet(1, 2, base_features=base).cuda().train()
    m.hip_precision = prec
    g = torch.Generator().manual_seed(10)
    x = (torch.rand(2, 1, size, size + 32, generator=g) * 2 - 1).cuda()
    t = (torch.rand(2, size, size + 32, generator=g) < 0.1).long().cuda()
    state = {k: v.clone() for k, v in m.state_dict().items()}
    out0, g0 = _grads(m, x, t, {})
    m.load_state_dict(state)
    out1, g1 = _grads(m, x, t, {"UNET_NO_GATE_VEC": "1"})
    assert torch.equal(out0, out1)
    if prec == "fp32":
        for n in g0:
            a, b = g0[n].double(), g1[n].double()
            rel = float((a - b).norm() / (b.norm() + 1e-30))
            assert rel <= 1e-4, (n, rel)
    else:
        a = torch.cat([g0[n].double().flatten() for n in g0])
        b = torch.cat([g1[n].double().flatten() for n in g0])
        assert float((a - b).norm() / b.norm()) <= 1e-2
        for n in g0:
            if g0[n].numel() < 16:
                # a 1-channel BN's gamma / beta gradient (psi): ONE sum over all pixels, whose relative change
                # under a 16-bit rounding flip upstream is unbounded where the sum cancels (0.19 on up1's psi gamma
                # at 16^2 once round 5 moved a BN-statistics summation order); the all-parameter rel-L2 covers it
                continue
            d = float((g0[n].double() - g1[n].double()).abs().max() / (g1[n].double().abs().max() + 1e-30))
            assert d <= 0.1, (n, d)
