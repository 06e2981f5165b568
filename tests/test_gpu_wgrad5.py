"""wgrad5 (csrc/wgrad5.hip): the LDS-DMA-pipelined 3x3 weight gradient, through the C-ABI
(`unet_conv_wgrad`), against torch's conv2d_weight on the same 16-bit operands — and wgrad2 on the same
cases, so the two paths the dispatcher chooses between (UNET_WGRAD5) are pinned to the same reference.

Reference op: the weight half of convolution_backward of nn.Conv2d(k=3, pad=1, bias=False)
(/root/reference/unet/models/layers.py:32,35).  Operands are exactly representable in the kernel's 16-bit
type, so a plain source leaves only the fp32 summation order (rel-L2 <= 1e-4); a BN-activation / gated
source is rounded to 16 bits once by the kernel, as by the forward, which can differ from torch's rounding
of the same fp32 value by one ulp (rel-L2 <= 2e-3)."""

import pytest
import torch

pytestmark = pytest.mark.gpu

DT = {"bf16": torch.bfloat16, "fp16": torch.float16}
SHAPES = [(4, 512, 512, 64, 64), (4, 256, 256, 128, 128), (2, 66, 70, 128, 64), (4, 32, 32, 512, 512),
          (1, 24, 40, 64, 128), (4, 128, 128, 256, 256), (1, 17, 45, 64, 64)]


def _lib():
    from unet._hip import lib as L
    return L


def _rt():
    from unet._hip import runtime as R
    return R


def _case(shape, kind, dt, seed=16):
    """(sources, the conv input x as fp32 NHWC, dy) for a plain / BN-activation / gated-concat input"""
    L = _lib()
    N, H, W, cin, cout = shape
    g = torch.Generator(device="cuda").manual_seed(seed)
    rnd = lambda *s: torch.randn(*s, device="cuda", generator=g)
    dy = rnd(N, H, W, cout).to(dt)

    def act(y, ab):
        s = L.Src()
        s.kind, s.C, s.H, s.W, s.data = L.SRC_ACT, y.shape[3], H, W, y.data_ptr()
        s.scale, s.shift, s.relu = ab[0].data_ptr(), ab[1].data_ptr(), 1
        return s

    def plain(y):
        s = L.Src()
        s.kind, s.C, s.H, s.W, s.data = L.SRC_PLAIN, y.shape[3], H, W, y.data_ptr()
        return s

    keep = []
    if kind == "plain":
        y = rnd(N, H, W, cin).to(dt)
        keep.append(y)
        return [plain(y)], y.float(), dy, keep
    if kind == "act":
        y = rnd(N, H, W, cin).to(dt)
        ab = torch.stack([rnd(cin), rnd(cin) * 0.2])
        keep += [y, ab]
        return [act(y, ab)], torch.relu(y.float() * ab[0] + ab[1]).to(dt).float(), dy, keep
    cs = cin // 2     # "gated+plain": the attention up-block concat [x * s, up]
    skip = rnd(N, H, W, cs).to(dt)
    ab = torch.stack([torch.rand(cs, device="cuda", generator=g) + 0.5, rnd(cs) * 0.2])
    p = rnd(N, H, W)
    pab = torch.tensor([0.7, -0.1], device="cuda")
    up = rnd(N, H, W, cin - cs).to(dt)
    s0 = act(skip, ab)
    s0.gate_p, s0.gate_ab = p.data_ptr(), pab.data_ptr()
    keep += [skip, ab, p, pab, up]
    xs = torch.relu(skip.float() * ab[0] + ab[1]) * torch.sigmoid(p * 0.7 - 0.1)[..., None]
    return [s0, plain(up)], torch.cat([xs.to(dt).float(), up.float()], -1), dy, keep


def _wgrad(srcs, dy, shape, dt):
    L, R = _lib(), _rt()
    N, H, W, cin, cout = shape
    wd = L.WgradDesc()
    wd.dtype = L.BF16 if dt == torch.bfloat16 else L.F16
    wd.N, wd.H, wd.W, wd.Cin, wd.Cout, wd.ksize, wd.nsrc = N, H, W, cin, cout, 3, len(srcs)
    for i, s in enumerate(srcs):
        wd.src[i] = s
    wd.dy = dy.data_ptr()
    dw = torch.empty(cout, cin, 3, 3, device="cuda")
    wd.dw = dw.data_ptr()
    ws = torch.empty(max(L.load().unet_wgrad_workspace(wd), 16), dtype=torch.uint8, device="cuda")
    wd.workspace = ws.data_ptr()
    name = R.wgrad_kernel_name(wd)
    L.call("unet_conv_wgrad", wd, R.stream())
    torch.cuda.synchronize()
    return dw, name


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("kind", ["plain", "act", "gated+plain"])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("path", ["wgrad5", "wgrad2"])
def test_wgrad_paths_vs_torch(path, prec, kind, shape, monkeypatch):
    if path == "wgrad5" and kind == "gated+plain" and shape[3] % 128:
        pytest.skip("wgrad5 takes a concat whose sources hold multiples of 64 channels (the network's: 64+64 ...)")
    monkeypatch.setenv("UNET_WGRAD5", "1" if path == "wgrad5" else "0")
    dt = DT[prec]
    srcs, x, dy, keep = _case(shape, kind, dt)
    N, H, W, cin, cout = shape
    ref = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2), (cout, cin, 3, 3), dy.float().permute(0, 3, 1, 2),
                                      padding=1)
    dw, name = _wgrad(srcs, dy, shape, dt)
    assert name.startswith(f"{path}_kernel<{'fp16' if prec == 'fp16' else 'bf16'}"), name
    rel = float((dw - ref).double().norm() / ref.double().norm())
    assert rel <= (1e-4 if kind == "plain" else 2e-3), (name, rel)


@pytest.mark.parametrize("shape", [(4, 512, 512, 64, 64), (2, 66, 70, 128, 64)], ids=lambda s: "x".join(map(str, s)))
def test_wgrad5_deterministic(shape, monkeypatch):
    """fixed-order split-K: two runs of the same wgrad are bit-identical"""
    monkeypatch.setenv("UNET_WGRAD5", "1")
    srcs, x, dy, keep = _case(shape, "act", torch.bfloat16, seed=5)
    a, name = _wgrad(srcs, dy, shape, torch.bfloat16)
    b, _ = _wgrad(srcs, dy, shape, torch.bfloat16)
    assert name.startswith("wgrad5_kernel"), name
    assert torch.equal(a, b)


def test_wgrad5_default_policy_at_bench_sizes(monkeypatch):
    """the default dispatch (UNET_WGRAD5 unset) at the bench's sizes: stored sources (the forward's act_out,
    materialised pool / upsample), BN activations (gated or not) and >= 128 output channels all go to wgrad5"""
    monkeypatch.delenv("UNET_WGRAD5", raising=False)
    L, R = _lib(), _rt()
    for shape, kind, want in [((4, 512, 512, 64, 64), "plain", "wgrad5"), ((4, 512, 512, 128, 64), "plain", "wgrad5"),
                              ((4, 256, 256, 128, 128), "gated+plain", "wgrad5"),
                              ((4, 512, 512, 64, 64), "act", "wgrad5"), ((4, 512, 512, 128, 64), "gated+plain", "wgrad5")]:
        srcs, x, dy, keep = _case(shape, kind, torch.bfloat16)
        N, H, W, cin, cout = shape
        wd = L.WgradDesc()
        wd.dtype, wd.N, wd.H, wd.W, wd.Cin, wd.Cout, wd.ksize, wd.nsrc = L.BF16, N, H, W, cin, cout, 3, len(srcs)
        for i, s in enumerate(srcs):
            wd.src[i] = s
        wd.dy = dy.data_ptr()
        assert R.wgrad_kernel_name(wd).startswith(f"{want}_kernel<bf16"), (shape, kind)


@pytest.mark.parametrize("kind", ["act", "gated+plain"])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_conv5_act_out_matches_transform(prec, kind):
    """unet_conv act_out (conv5 forward, y mode): the stored map is the transformed src[0] — the weight
    gradient on [plain(act_out), src1] equals the one on the BN-activation sources up to fp32 summation order"""
    L, R = _lib(), _rt()
    dt = DT[prec]
    shape = (4, 256, 256, 128, 64)     # conv5 needs >= 256 output tiles
    N, H, W, cin, cout = shape
    srcs, x, dy, keep = _case(shape, kind, dt, seed=8)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") * 0.05).to(dt).float()
    wp = R.pack_weight(w, R._PRECISIONS[prec], transpose=False)
    d = L.ConvDesc()
    d.dtype = L.BF16 if dt == torch.bfloat16 else L.F16
    d.N, d.H, d.W, d.Cin, d.Cout, d.ksize, d.nsrc = N, H, W, cin, cout, 3, len(srcs)
    for i, s in enumerate(srcs):
        d.src[i] = s
    y = torch.empty(N, H, W, cout, dtype=dt, device="cuda")
    d.weight, d.out_mode, d.out = wp.data_ptr(), L.OUT_Y, y.data_ptr()
    assert L.load().unet_conv_act_out_ok(d) == 1
    act = torch.full((N, H, W, srcs[0].C), float("nan"), dtype=dt, device="cuda")
    d.act_out = act.data_ptr()
    L.call("unet_conv", d, R.stream())
    torch.cuda.synchronize()
    assert not torch.isnan(act.float()).any()          # every pixel written
    c0 = srcs[0].C
    assert (act.float() - x[..., :c0]).abs().max() <= 2 ** -7 * (1 + x[..., :c0].abs().max())
    ps = L.Src()
    ps.kind, ps.C, ps.H, ps.W, ps.data = L.SRC_PLAIN, c0, H, W, act.data_ptr()
    a, na = _wgrad(srcs, dy, shape, dt)
    b, nb = _wgrad([ps] + srcs[1:], dy, shape, dt)
    # the same 16-bit operands; the dispatcher may pick another kernel for the stored source (wgrad5 with 4-row
    # stages for a 64-channel output block vs wgrad2 for the BN-activation source): the same fp32 products
    # summed in another order
    rel = float((a - b).double().norm() / b.double().norm())
    assert rel <= 1e-5, rel
