"""GPU op-level numerics: each HIP entry point (through the C-ABI) against a plain PyTorch fp32
reference of the same op, on operands that are exactly representable in the kernel's operand type
(bf16-rounded for the bf16 kernels), so the only difference left is the summation order.
Shapes are chosen to hit every tile configuration of csrc/conv.hip and csrc/wgrad2.hip, including
partial tiles and channel counts that are not multiples of the tile sizes."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DT = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}
TN = {"fp32": "fp32", "bf16": "bf16", "fp16": "fp16"}   # kernel-name spelling


def _lib():
    from unet._hip import lib as L
    return L


def _rt():
    from unet._hip import runtime as R
    return R


def _rand(*shape, dt, scale=1.0):
    return (torch.randn(*shape, device="cuda") * scale).to(dt)


def _act_src(y, ab, relu=True, kind=None):
    L = _lib()
    s = L.Src()
    s.kind = L.SRC_ACT if kind is None else kind
    _, s.H, s.W, s.C = y.shape
    s.data = y.data_ptr()
    s.scale = ab[0].data_ptr()
    s.shift = ab[1].data_ptr()
    s.relu = int(relu)
    return s


def _act_ref(y, ab, relu=True):
    a = y.float() * ab[0] + ab[1]
    return a.clamp_min(0) if relu else a


def _conv(prec, srcs, N, H, W, cin, w, k, out_mode, **kw):
    L, R = _lib(), _rt()
    P = R._PRECISIONS[prec]
    transpose = kw.pop("transpose", False)
    cout = w.shape[1] if transpose else w.shape[0]
    wp = R.pack_weight(w, P, transpose=transpose)
    d = L.ConvDesc()
    d.dtype = P.code
    d.N, d.H, d.W, d.Cin, d.Cout, d.ksize = N, H, W, cin, cout, k
    d.nsrc = len(srcs)
    for i, s in enumerate(srcs):
        d.src[i] = s
    d.weight = wp.data_ptr()
    d.out_mode = out_mode
    for key, v in kw.items():
        setattr(d, key, v)
    ws = L.attach_workspace(d, "cuda")   # the split-K form where d has one (kept set on d: the row queries)
    L.call("unet_conv", d, R.stream())
    torch.cuda.synchronize()
    del ws
    return d


CONV_SHAPES = [  # (N, H, W, Cin, Cout) — tile configs: BN 32/64/128, TH 8/16, partial tiles
    (2, 16, 16, 32, 32), (1, 24, 40, 64, 64), (2, 33, 20, 96, 128), (4, 64, 64, 64, 128), (1, 8, 24, 128, 256),
    (2, 20, 36, 40, 48),
]


@pytest.mark.parametrize("prec", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("shape", CONV_SHAPES)
@pytest.mark.parametrize("k", [3, 1])
def test_conv_fwd_act(prec, shape, k):
    L = _lib()
    N, H, W, cin, cout = shape
    dt = DT[prec]
    torch.manual_seed(0)
    y = _rand(N, H, W, cin, dt=dt)
    ab = torch.stack([torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.2])
    w = (torch.randn(cout, cin, k, k, device="cuda") * 0.1).to(dt).float()
    out = torch.empty(N, H, W, cout, dtype=dt, device="cuda")
    st = torch.zeros(2, 4096, cout, device="cuda")
    d = _conv(prec, [_act_src(y, ab)], N, H, W, cin, w, k, L.OUT_Y, out=out.data_ptr(), stats=st.data_ptr())
    x = _act_ref(y, ab).to(dt).float().permute(0, 3, 1, 2)
    ref = F.conv2d(x, w, padding=k // 2).permute(0, 2, 3, 1)
    tol = 2e-2 if prec != "fp32" else 1e-4
    assert (out.float() - ref).abs().max() <= tol * (1 + ref.abs().max()), (out.float() - ref).abs().max()
    # BN partial sums ([2][Cout][rows], from the fp32 accumulators)
    rows = L.load().unet_conv_stats_rows(d)
    sums = st.flatten()[:2 * cout * rows].view(2, cout, rows).double().sum(-1)
    r = ref.double().reshape(-1, cout)
    P = r.shape[0]
    assert ((sums[0] - r.sum(0)).abs() <= tol * P ** 0.5 * (1 + r.abs().mean(0))).all()
    assert ((sums[1] - (r * r).sum(0)).abs() <= 4 * tol * (r * r).sum(0) + 1e-3).all()


@pytest.mark.parametrize("prec", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("shape", [(2, 16, 16, 32, 64), (1, 21, 30, 64, 128), (2, 8, 8, 128, 64)])
def test_conv_fwd_pool_and_up_concat(prec, shape):
    """down.0 (max-pool of ACT) and up.0 ([gated skip, pad(up(ACT))]) loaders."""
    L = _lib()
    N, H, W, cin, cout = shape
    dt = DT[prec]
    torch.manual_seed(1)
    # pool
    ys = _rand(N, 2 * H + 1, 2 * W, cin, dt=dt)
    ab = torch.stack([torch.randn(cin, device="cuda"), torch.randn(cin, device="cuda") * 0.2])
    w = (torch.randn(cout, cin, 3, 3, device="cuda") * 0.1).to(dt).float()
    out = torch.empty(N, H, W, cout, dtype=dt, device="cuda")
    _conv(prec, [_act_src(ys, ab, kind=L.SRC_POOL_ACT)], N, H, W, cin, w, 3, L.OUT_Y, out=out.data_ptr())
    x = F.max_pool2d(_act_ref(ys, ab).permute(0, 3, 1, 2), 2)
    ref = F.conv2d(x.to(dt).float(), w, padding=1).permute(0, 2, 3, 1)
    tol = 2e-2 if prec != "fp32" else 1e-4
    assert (out.float() - ref).abs().max() <= tol * (1 + ref.abs().max())
    # concat [skip * sigmoid(gate), pad(up(act(dec)))]
    cs = cin // 2
    skip = _rand(N, H, W, cs, dt=dt)
    abs_ = torch.stack([torch.rand(cs, device="cuda") + 0.5, torch.randn(cs, device="cuda") * 0.1])
    dec = _rand(N, (H - 1) // 2, W // 2, cin - cs, dt=dt)
    abd = torch.stack([torch.rand(cin - cs, device="cuda") + 0.5, torch.randn(cin - cs, device="cuda") * 0.1])
    p = torch.randn(N, H, W, device="cuda")
    pab = torch.tensor([0.7, -0.1], device="cuda")
    s0 = _act_src(skip, abs_)
    s0.gate_p, s0.gate_ab = p.data_ptr(), pab.data_ptr()
    up_h, up_w = 2 * dec.shape[1], 2 * dec.shape[2]
    s1 = _act_src(dec, abd, kind=L.SRC_UP_ACT)
    R = _rt()
    s1.up_h, s1.up_w, s1.pad_t, s1.pad_l = up_h, up_w, (H - up_h) // 2, (W - up_w) // 2
    s1.sh, s1.sw = R.up_scale(dec.shape[1], up_h), R.up_scale(dec.shape[2], up_w)
    _conv(prec, [s0, s1], N, H, W, cin, w, 3, L.OUT_Y, out=out.data_ptr())
    xs = _act_ref(skip, abs_).permute(0, 3, 1, 2) * torch.sigmoid(p * 0.7 - 0.1)[:, None]
    xu = F.interpolate(_act_ref(dec, abd).permute(0, 3, 1, 2), size=(up_h, up_w), mode="bilinear", align_corners=True)
    dyy, dxx = H - up_h, W - up_w
    xu = F.pad(xu, [dxx // 2, dxx - dxx // 2, dyy // 2, dyy - dyy // 2])
    ref = F.conv2d(torch.cat([xs, xu], 1).to(dt).float(), w, padding=1).permute(0, 2, 3, 1)
    assert (out.float() - ref).abs().max() <= tol * (1 + ref.abs().max())


@pytest.mark.parametrize("prec", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("shape", [(2, 16, 16, 64, 32), (1, 24, 40, 128, 64), (2, 18, 20, 64, 128)])
def test_conv_dgrad_split_and_pool(prec, shape):
    L = _lib()
    N, H, W, cin, cout = shape     # forward conv cin -> cout; dgrad maps dy[cout] -> dx[cin]
    dt = DT[prec]
    torch.manual_seed(2)
    dy = _rand(N, H, W, cout, dt=dt)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") * 0.1).to(dt).float()
    ref = F.conv_transpose2d(dy.float().permute(0, 3, 1, 2), w, padding=1).permute(0, 2, 3, 1)
    src = L.Src()
    src.kind, src.C, src.H, src.W, src.data = L.SRC_PLAIN, cout, H, W, dy.data_ptr()
    split = cin // 4 * 2
    o1 = torch.full((N, H, W, split), 1.0, device="cuda")
    o2 = torch.empty(N, H, W, cin - split, device="cuda")
    _conv(prec, [src], N, H, W, cout, w, 3, L.OUT_F32, transpose=True, out=o1.data_ptr(), out2=o2.data_ptr(),
          split=split, accum=1, accum2=0)
    tol = 2e-2 if prec != "fp32" else 1e-4
    got = torch.cat([o1 - 1.0, o2], -1)
    assert (got - ref).abs().max() <= tol * (1 + ref.abs().max())
    # pool-bwd routing: gradient of maxpool(act(ys)) at the pooled resolution
    ys = _rand(N, 2 * H, 2 * W + 1, cin, dt=dt)
    ab = torch.stack([torch.randn(cin, device="cuda"), torch.randn(cin, device="cuda") * 0.2])
    da = torch.zeros(N, 2 * H, 2 * W + 1, cin, device="cuda")
    _conv(prec, [src], N, H, W, cout, w, 3, L.OUT_POOL_BWD, transpose=True, out=da.data_ptr(),
          pool_src=_act_src(ys, ab))
    a = _act_ref(ys, ab).permute(0, 3, 1, 2).requires_grad_(True)
    F.max_pool2d(a, 2).backward(ref.permute(0, 3, 1, 2))
    assert (da.permute(0, 3, 1, 2) - a.grad).abs().max() <= tol * (1 + ref.abs().max())


@pytest.mark.parametrize("prec", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("shape", [(2, 16, 16, 64, 64), (1, 24, 40, 32, 128), (2, 40, 36, 128, 256),
                                   (4, 32, 32, 96, 64), (4, 128, 128, 64, 64)])   # last: >32 split-K slabs
@pytest.mark.parametrize("k", [3, 1])
@pytest.mark.parametrize("kind", ["act", "pool"])
def test_conv_wgrad(prec, shape, k, kind):
    L, R = _lib(), _rt()
    P = R._PRECISIONS[prec]
    N, H, W, cin, cout = shape
    dt = DT[prec]
    torch.manual_seed(3)
    dy = _rand(N, H, W, cout, dt=dt)
    ab = torch.stack([torch.randn(cin, device="cuda"), torch.randn(cin, device="cuda") * 0.2])
    if kind == "act":
        y = _rand(N, H, W, cin, dt=dt)
        src = _act_src(y, ab)
        x = _act_ref(y, ab).permute(0, 3, 1, 2)
    else:
        y = _rand(N, 2 * H, 2 * W, cin, dt=dt)
        src = _act_src(y, ab, kind=L.SRC_POOL_ACT)
        x = F.max_pool2d(_act_ref(y, ab).permute(0, 3, 1, 2), 2)
    x = x.to(dt).float()
    ref = torch.nn.grad.conv2d_weight(x, (cout, cin, k, k), dy.float().permute(0, 3, 1, 2), padding=k // 2)
    wd = L.WgradDesc()
    wd.dtype = P.code
    wd.N, wd.H, wd.W, wd.Cin, wd.Cout, wd.ksize, wd.nsrc = N, H, W, cin, cout, k, 1
    wd.src[0] = src
    wd.dy = dy.data_ptr()
    dw = torch.empty(cout, cin, k, k, device="cuda")
    wd.dw = dw.data_ptr()
    ws = torch.empty(max(L.load().unet_wgrad_workspace(wd), 16), dtype=torch.uint8, device="cuda")
    wd.workspace = ws.data_ptr()
    L.call("unet_conv_wgrad", wd, R.stream())
    torch.cuda.synchronize()
    tol = 1e-3 if prec != "fp32" else 1e-4
    assert (dw - ref).abs().max() <= tol * (1 + ref.abs().max()), float((dw - ref).abs().max())


@pytest.mark.parametrize("prec", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("shape", [(2, 1, 40, 36, 64), (1, 3, 33, 50, 16), (4, 1, 64, 64, 8),
                                   (2, 3, 70, 100, 64), (4, 1, 512, 512, 64), (1, 2, 9, 130, 64)])
def test_first_conv_nchw_input(prec, shape):
    """inc.0: the fp32 NCHW model input read directly (csrc/smallcin.hip), fwd + BN sums + wgrad.  16-bit,
    64 output channels: the MFMA forward (x split into two 16-bit halves); otherwise the VALU kernel."""
    L, R = _lib(), _rt()
    P = R._PRECISIONS[prec]
    N, cin, H, W, cout = shape
    dt = DT[prec]
    torch.manual_seed(4)
    x = torch.rand(N, cin, H, W, device="cuda") * 2 - 1
    w = (torch.randn(cout, cin, 3, 3, device="cuda") * 0.3).to(dt).float()
    src = L.Src()
    src.kind, src.C, src.H, src.W, src.data = L.SRC_NCHW_F32, cin, H, W, x.data_ptr()
    out = torch.empty(N, H, W, cout, dtype=dt, device="cuda")
    d = L.ConvDesc()
    d.dtype, d.N, d.H, d.W, d.Cin, d.Cout, d.ksize, d.nsrc = P.code, N, H, W, cin, cout, 3, 1
    d.src[0] = src
    rows = L.load().unet_conv_stats_rows(d)
    st = torch.empty(2, cout, rows, device="cuda")   # [2][Cout][rows] partial sums
    wp = R.pack_weight(w, P, transpose=False)
    d.weight, d.out_mode, d.out, d.stats = wp.data_ptr(), L.OUT_Y, out.data_ptr(), st.data_ptr()
    L.call("unet_conv", d, R.stream())
    torch.cuda.synchronize()
    want = "smallcin_fwd_mfma_kernel" if prec != "fp32" and cout == 64 else "smallcin_fwd_kernel"
    assert _variant(d).startswith(want), _variant(d)
    xr = x.to(dt).float() if prec != "fp32" else x
    ref = F.conv2d(x, w, padding=1).permute(0, 2, 3, 1)
    tol = 1e-2 if prec != "fp32" else 1e-5
    assert (out.float() - ref).abs().max() <= tol * (1 + ref.abs().max())
    assert torch.allclose(st[0].sum(1), ref.sum((0, 1, 2)), rtol=1e-4, atol=1e-2)
    assert torch.allclose(st[1].sum(1), (ref * ref).sum((0, 1, 2)), rtol=1e-4, atol=1e-2)
    # weight gradient
    dy = _rand(N, H, W, cout, dt=dt)
    refw = torch.nn.grad.conv2d_weight(x, (cout, cin, 3, 3), dy.float().permute(0, 3, 1, 2), padding=1)
    wd = L.WgradDesc()
    wd.dtype, wd.N, wd.H, wd.W, wd.Cin, wd.Cout, wd.ksize, wd.nsrc = P.code, N, H, W, cin, cout, 3, 1
    wd.src[0] = src
    wd.dy = dy.data_ptr()
    dw = torch.empty(cout, cin, 3, 3, device="cuda")
    wd.dw = dw.data_ptr()
    ws = torch.empty(max(L.load().unet_wgrad_workspace(wd), 16), dtype=torch.uint8, device="cuda")
    wd.workspace = ws.data_ptr()
    L.call("unet_conv_wgrad", wd, R.stream())
    torch.cuda.synchronize()
    assert (dw - refw).abs().max() <= 1e-4 * (1 + refw.abs().max())
    del xr


@pytest.mark.parametrize("prec", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("shape", [(2, 8, 8, 64, 32, 0, 0), (1, 12, 20, 128, 64, 1, 2), (2, 5, 7, 32, 16, 0, 1)])
def test_conv_transpose_k2s2(prec, shape):
    """Up(bilinear=False): ConvTranspose2d(k=2, s=2, bias) as a 1x1 conv with the SHUFFLE2 epilogue,
    and its backward (space-to-depth prep + bias colsum + 1x1 wgrad + 1x1 dgrad), vs torch fp32."""
    from unet._hip.stages import ConvTStage, Grads
    R = _rt()
    P = R._PRECISIONS[prec]
    N, h, w, cin, ct, pt, pl = shape
    dt = DT[prec]
    torch.manual_seed(5)
    m = torch.nn.ConvTranspose2d(cin, ct, 2, 2).cuda()
    with torch.no_grad():
        m.weight.copy_(m.weight.to(dt).float())
    y = _rand(N, h, w, cin, dt=dt)
    ab = torch.stack([torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.2])
    a = R.Act(y, ab, True)
    st = ConvTStage(m)
    u = st.forward(P, a)
    x = _act_ref(y, ab).to(dt).float().permute(0, 3, 1, 2).requires_grad_(True)
    ref = m(x)
    tol = 2e-2 if prec != "fp32" else 1e-4
    assert (u.data.float().permute(0, 3, 1, 2) - ref).abs().max() <= tol * (1 + ref.abs().max())
    # backward through a padded placement
    Hp, Wp = 2 * h + pt + 1, 2 * w + pl + 2
    d_up = torch.zeros(N, Hp, Wp, ct, device="cuda")
    g = torch.randn(N, 2 * h, 2 * w, ct, device="cuda").to(dt).float()
    d_up[:, pt:pt + 2 * h, pl:pl + 2 * w] = g
    grads = Grads()
    st.backward(P, d_up, pt, pl, grads)
    torch.cuda.synchronize()
    ref.backward(g.permute(0, 3, 1, 2))
    gw, gb = grads[m.weight], grads[m.bias]
    assert gw.shape == m.weight.shape
    tw = 1e-3 if prec != "fp32" else 1e-4
    assert (gw - m.weight.grad).abs().max() <= tw * (1 + m.weight.grad.abs().max())
    assert (gb - m.bias.grad).abs().max() <= 1e-4 * (1 + m.bias.grad.abs().max())
    gx = x.grad.permute(0, 2, 3, 1)
    assert (a.grad - gx).abs().max() <= tol * (1 + gx.abs().max())


# pointwise (1x1) path of csrc/pw.hip: taken for bf16 1x1 convs over >= 32768 pixels (the attention-gate
# projections at 128^2..512^2); shapes include a pixel count that is not a multiple of the 256-pixel block
PW_SHAPES = [(4, 128, 128, 64, 32), (4, 181, 183, 64, 64), (4, 128, 256, 128, 64), (8, 128, 128, 256, 128),
             (4, 200, 170, 32, 64)]


def _pw_var(L, d):
    import ctypes
    buf = ctypes.create_string_buffer(128)
    L.load().unet_conv_variant(d, buf, 128)
    return buf.value.decode()


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("shape", PW_SHAPES)
@pytest.mark.parametrize("gate", [False, True])
def test_pw_fwd_stats(shape, gate, prec):
    L = _lib()
    N, H, W, cin, cout = shape
    dt = DT[prec]
    torch.manual_seed(5)
    y = _rand(N, H, W, cin, dt=dt)
    ab = torch.stack([torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.2])
    src = _act_src(y, ab)
    x = _act_ref(y, ab)
    if gate:
        p = torch.randn(N, H, W, device="cuda")
        pab = torch.tensor([0.7, -0.1], device="cuda")
        src.gate_p, src.gate_ab = p.data_ptr(), pab.data_ptr()
        x = x * torch.sigmoid(p * 0.7 - 0.1)[..., None]
    w = (torch.randn(cout, cin, 1, 1, device="cuda") * 0.1).to(dt).float()
    out = torch.empty(N, H, W, cout, dtype=dt, device="cuda")
    st = torch.zeros(2, cout, 8192, device="cuda")
    d = _conv(prec, [src], N, H, W, cin, w, 1, L.OUT_Y, out=out.data_ptr(), stats=st.data_ptr())
    assert _pw_var(L, d).startswith("pw_conv_kernel"), _pw_var(L, d)
    ref = F.conv2d(x.to(dt).float().permute(0, 3, 1, 2), w).permute(0, 2, 3, 1)
    assert (out.float() - ref).abs().max() <= 2e-2 * (1 + ref.abs().max())
    rows = L.load().unet_conv_stats_rows(d)
    sums = st.flatten()[:2 * cout * rows].view(2, cout, rows).double().sum(-1)
    r = ref.double().reshape(-1, cout)
    assert torch.allclose(sums[0], r.sum(0), rtol=1e-3, atol=1e-1)
    assert torch.allclose(sums[1], (r * r).sum(0), rtol=1e-3, atol=1e-1)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("shape", PW_SHAPES)
def test_pw_dgrad_split_accum(shape, prec):
    L = _lib()
    N, H, W, cin, cout = shape     # forward 1x1 conv cin -> cout; dgrad dy[cout] -> dx[cin]
    dt = DT[prec]
    torch.manual_seed(6)
    dy = _rand(N, H, W, cout, dt=dt)
    w = (torch.randn(cout, cin, 1, 1, device="cuda") * 0.1).to(dt).float()
    ref = F.conv_transpose2d(dy.float().permute(0, 3, 1, 2), w).permute(0, 2, 3, 1)
    src = L.Src()
    src.kind, src.C, src.H, src.W, src.data = L.SRC_PLAIN, cout, H, W, dy.data_ptr()
    split = cin // 2
    o1 = torch.full((N, H, W, split), 1.0, device="cuda")
    o2 = torch.full((N, H, W, cin - split), float("nan"), device="cuda")
    d = _conv(prec, [src], N, H, W, cout, w, 1, L.OUT_F32, transpose=True, out=o1.data_ptr(), out2=o2.data_ptr(),
              split=split, accum=1, accum2=0)
    if cout % 32 == 0:
        assert _pw_var(L, d).startswith("pw_conv_kernel"), _pw_var(L, d)
    got = torch.cat([o1 - 1.0, o2], -1)
    assert (got - ref).abs().max() <= 2e-2 * (1 + ref.abs().max())


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("shape", PW_SHAPES)
@pytest.mark.parametrize("gate", [False, True])
def test_pw_wgrad(shape, gate, prec):
    L, R = _lib(), _rt()
    N, H, W, cin, cout = shape
    dt = DT[prec]
    torch.manual_seed(7)
    dy = _rand(N, H, W, cout, dt=dt)
    ab = torch.stack([torch.randn(cin, device="cuda"), torch.randn(cin, device="cuda") * 0.2])
    y = _rand(N, H, W, cin, dt=dt)
    src = _act_src(y, ab)
    x = _act_ref(y, ab)
    if gate:
        p = torch.randn(N, H, W, device="cuda")
        pab = torch.tensor([0.7, -0.1], device="cuda")
        src.gate_p, src.gate_ab = p.data_ptr(), pab.data_ptr()
        x = x * torch.sigmoid(p * 0.7 - 0.1)[..., None]
    x = x.to(dt).float().permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(x, (cout, cin, 1, 1), dy.float().permute(0, 3, 1, 2))
    wd = L.WgradDesc()
    wd.dtype = R._PRECISIONS[prec].code
    wd.N, wd.H, wd.W, wd.Cin, wd.Cout, wd.ksize, wd.nsrc = N, H, W, cin, cout, 1, 1
    wd.src[0] = src
    wd.dy = dy.data_ptr()
    dw = torch.full((cout, cin, 1, 1), 3.0, device="cuda")
    wd.dw = dw.data_ptr()
    wd.accum = 1
    ws = torch.empty(max(L.load().unet_wgrad_workspace(wd), 16), dtype=torch.uint8, device="cuda")
    wd.workspace = ws.data_ptr()
    L.call("unet_conv_wgrad", wd, R.stream())
    torch.cuda.synchronize()
    assert ((dw - 3.0) - ref).abs().max() <= 1e-3 * (1 + ref.abs().max()), float(((dw - 3.0) - ref).abs().max())


@pytest.mark.parametrize("shape", [(2, 64, 64, 64), (1, 37, 50, 16), (2, 32, 48, 128)])
@pytest.mark.parametrize("accum", [0, 1])
def test_outconv_bwd_vec(shape, accum):
    """OutConv (1x1 + bias, layers.py:109-123) backward on a BN+ReLU source: dx, dW, db (bf16 operands)."""
    L = _lib()
    N, H, W, C = shape
    K = 2
    dt = torch.bfloat16
    torch.manual_seed(8)
    y = _rand(N, H, W, C, dt=dt)
    ab = torch.stack([torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.2])
    w = torch.randn(K, C, device="cuda") * 0.1
    dl = torch.randn(N, K, H, W, device="cuda")
    a = _act_ref(y, ab)                                   # NHWC fp32
    ref_dx = torch.einsum("nkhw,kc->nhwc", dl, w)
    ref_dw = torch.einsum("nkhw,nhwc->kc", dl, a)
    ref_db = dl.sum((0, 2, 3))
    P = N * H * W
    rows = L.load().unet_outconv_rows(P)
    part = torch.zeros(rows, K + 1, max(C, K), device="cuda")
    da = torch.full((N, H, W, C), 2.0, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    L.call("unet_outconv_bwd", L.BF16, N, H, W, C, K, y.data_ptr(), ab[0].data_ptr(), ab[1].data_ptr(), 1,
           w.data_ptr(), dl.data_ptr(), da.data_ptr(), accum, part.data_ptr(), s)
    dw, db = torch.empty(K, C, device="cuda"), torch.empty(K, device="cuda")
    L.call("unet_outconv_bwd_finalize", part.data_ptr(), rows, C, K, dw.data_ptr(), db.data_ptr(), 0, s)
    torch.cuda.synchronize()
    assert ((da - 2.0 * accum) - ref_dx).abs().max() <= 1e-5 * (1 + ref_dx.abs().max())
    assert (dw - ref_dw).abs().max() <= 1e-4 * (1 + ref_dw.abs().max())
    assert (db - ref_db).abs().max() <= 1e-4 * (1 + ref_db.abs().max())


@pytest.mark.parametrize("geo", [(2, 32, 32, 64, 64, 64), (1, 16, 20, 33, 41, 32), (2, 7, 9, 14, 18, 8),
                                 (1, 25, 17, 50, 34, 12), (4, 256, 256, 512, 512, 64), (2, 32, 32, 64, 64, 512),
                                 (1, 13, 37, 27, 75, 48)])
@pytest.mark.parametrize("accum", [0, 1])
def test_upsample_bwd(geo, accum):
    """Adjoint of bilinear x2 (align_corners=True) + F.pad into the skip's frame (layers.py:78,98-102),
    incl. the bench's 256^2 -> 512^2 x 64-channel case, against torch's adjoint in fp64"""
    L, R = _lib(), _rt()
    N, h, w, Hp, Wp, C = geo
    up_h, up_w = 2 * h, 2 * w
    pt, pl = (Hp - up_h) // 2, (Wp - up_w) // 2
    torch.manual_seed(9)
    g = torch.randn(N, Hp, Wp, C, device="cuda")
    # reference: torch's adjoint in fp64 (its fp32 form scatters with atomics: order-dependent rounding)
    x = torch.randn(N, C, h, w, device="cuda", dtype=torch.float64, requires_grad=True)
    u = F.interpolate(x, size=(up_h, up_w), mode="bilinear", align_corners=True)
    u = F.pad(u, [pl, Wp - up_w - pl, pt, Hp - up_h - pt])
    u.backward(g.double().permute(0, 3, 1, 2))
    ref = x.grad.permute(0, 2, 3, 1)
    dx = torch.full((N, h, w, C), 1.5, device="cuda")
    L.call("unet_upsample_bwd", N, C, h, w, up_h, up_w, pt, pl, Hp, Wp, R.up_scale(h, up_h), R.up_scale(w, up_w),
           g.data_ptr(), dx.data_ptr(), accum, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    err = float(((dx - 1.5 * accum).double() - ref).abs().max())
    assert err <= 1e-5 * (1 + float(ref.abs().max())), err


# ------------------------------------------------------------------------------------------------
# The conv3 instantiations the benchmark runs (csrc/conv.hip pick_cfg: tiles16 = N*ceil(H/16)*ceil(W/16)
# >= 256 selects the 4-wave w4 tiles for the y epilogue and the 8-wave MI=8 tiles for the fp32 dgrad and
# pool-routing epilogues).  Bench-sized maps, so that M tiles outnumber the persistent grid and every
# workgroup runs the multi-tile loop (next tile staged during the last chunk).  Reference: torch fp32
# conv on the same bf16-rounded operands; gates: rel-L2 <= 4e-3 (bf16 output rounding is ~1e-3) and
# max-abs <= 2e-2 * (1 + max|ref|).
# ------------------------------------------------------------------------------------------------

def _variant(d):
    import ctypes
    buf = ctypes.create_string_buffer(128)
    _lib().load().unet_conv_variant(d, buf, 128)
    return buf.value.decode()


def _close_bf16(got, ref, what):
    got, ref = got.double(), ref.double()
    rel = float((got - ref).norm() / (ref.norm() + 1e-30))
    mx = float((got - ref).abs().max())
    assert rel <= 4e-3, (what, rel)
    assert mx <= 2e-2 * (1 + float(ref.abs().max())), (what, mx)


def _persistent(N, H, W, TH, cout, BN, w4):
    """M tiles per workgroup of launch_conv3's grid (> 1: the persistent multi-tile loop runs)."""
    mt = N * ((H + TH - 1) // TH) * ((W + 15) // 16)
    gy = (cout + BN - 1) // BN
    gx = min(mt, ((512 if w4 else 256) + gy - 1) // gy)
    return mt / gx


# (N, H, W, Cin, Cout, expected variant) — forward / y epilogue (+ BN partial sums)
Y_BENCH = [
    (4, 512, 512, 64, 64, "conv3_kernel<bf16,3,1,4,1,8,1>"),     # inc.3 / up4.conv.3
    (4, 256, 256, 64, 128, "conv3_kernel<bf16,3,1,4,2,8,1>"),    # down1.0
    (4, 256, 256, 128, 128, "conv3_kernel<bf16,3,1,4,2,8,1>"),   # down1.3
    (4, 128, 128, 256, 256, "conv3_kernel<bf16,3,1,4,2,8,1>"),   # down2.3
    (3, 200, 328, 64, 128, "conv3_kernel<bf16,3,1,4,2,8,1>"),    # partial tiles in both directions
]


@pytest.mark.parametrize("shape", Y_BENCH, ids=lambda s: "x".join(map(str, s[:5])))
@pytest.mark.parametrize("stats", [True, False])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_conv3_bench_tiles_y(prec, shape, stats, monkeypatch):
    monkeypatch.setenv("UNET_CONV5", "0")
    L = _lib()
    N, H, W, cin, cout, want = shape
    dt = DT[prec]
    torch.manual_seed(11)
    y = _rand(N, H, W, cin, dt=dt)
    ab = torch.stack([torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.2])
    w = (torch.randn(cout, cin, 3, 3, device="cuda") * (2.0 / (9 * cin)) ** 0.5).to(dt).float()
    out = torch.empty(N, H, W, cout, dtype=dt, device="cuda")
    L.load()
    kw = {"out": out.data_ptr()}
    st = None
    if stats:
        d0 = L.ConvDesc()
        d0.dtype, d0.N, d0.H, d0.W, d0.Cin, d0.Cout, d0.ksize, d0.nsrc = _rt()._PRECISIONS[prec].code, N, H, W, cin, cout, 3, 1
        d0.src[0] = _act_src(y, ab)
        ws0 = L.attach_workspace(d0, "cuda")
        rows = L.load().unet_conv_stats_rows(d0)
        st = torch.empty(2, cout, rows, device="cuda")
        kw["stats"] = st.data_ptr()
    d = _conv(prec, [_act_src(y, ab)], N, H, W, cin, w, 3, L.OUT_Y, **kw)
    assert _variant(d) == want.replace("bf16", TN[prec]), _variant(d)
    assert _persistent(N, H, W, 8, cout, 64 if cout <= 64 else 128, True) > 1
    x = _act_ref(y, ab).to(dt).float().permute(0, 3, 1, 2)
    ref = F.conv2d(x, w, padding=1).permute(0, 2, 3, 1)
    _close_bf16(out.float(), ref, "y")
    if stats:
        r = ref.double().reshape(-1, cout)
        s = st.double().sum(-1)
        # the sums come from the fp32 accumulators (before bf16 rounding of y)
        assert ((s[0] - r.sum(0)).abs() <= 1e-3 * r.abs().sum(0) + 1e-2).all()
        assert ((s[1] - (r * r).sum(0)).abs() <= 1e-2 * (r * r).sum(0) + 1e-2).all()


# dgrad of a forward conv cin -> cout: dy[cout] -> dx[cin] (the dgrad conv has Cout = cin)
DGRAD_BENCH = [
    (4, 512, 512, 128, 64, "conv3_kernel<bf16,3,2,4,2,8,1>"),    # up4.conv.0 dgrad, split skip / up
    (4, 256, 256, 256, 128, "conv3_kernel<bf16,3,2,4,2,8,1>"),   # up3.conv.0 dgrad
    (4, 512, 512, 64, 64, "conv3_kernel<bf16,3,2,4,1,8,1>"),
    (3, 200, 328, 128, 64, "conv3_kernel<bf16,3,2,4,2,8,1>"),
]


@pytest.mark.parametrize("shape", DGRAD_BENCH, ids=lambda s: "x".join(map(str, s[:5])))
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_conv3_bench_tiles_dgrad_f32(prec, shape, monkeypatch):
    monkeypatch.setenv("UNET_CONV5", "0")
    L = _lib()
    N, H, W, cin, cout, want = shape
    dt = DT[prec]
    torch.manual_seed(12)
    dy = _rand(N, H, W, cout, dt=dt)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") * (2.0 / (9 * cin)) ** 0.5).to(dt).float()
    ref = F.conv_transpose2d(dy.float().permute(0, 3, 1, 2), w, padding=1).permute(0, 2, 3, 1)
    src = L.Src()
    src.kind, src.C, src.H, src.W, src.data = L.SRC_PLAIN, cout, H, W, dy.data_ptr()
    split = cin // 2
    o1 = torch.full((N, H, W, split), 0.5, device="cuda")
    o2 = torch.full((N, H, W, cin - split), float("nan"), device="cuda")
    d = _conv(prec, [src], N, H, W, cout, w, 3, L.OUT_F32, transpose=True, out=o1.data_ptr(), out2=o2.data_ptr(),
              split=split, accum=1, accum2=0)
    assert _variant(d) == want.replace("bf16", TN[prec]), _variant(d)
    assert _persistent(N, H, W, 16, cin, 128 if cin > 64 else 64, False) > 1
    got = torch.cat([o1 - 0.5, o2], -1)
    _close_bf16(got, ref, "dgrad f32")


@pytest.mark.parametrize("shape", [(4, 512, 512, 64, 64), (4, 256, 256, 128, 128), (3, 200, 328, 64, 64)],
                         ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_conv3_bench_tiles_dgrad_y(prec, shape, monkeypatch):
    """bf16 gradient of a DoubleConv's middle activation (the y epilogue without BN sums)."""
    monkeypatch.setenv("UNET_CONV5", "0")
    L = _lib()
    N, H, W, cin, cout = shape
    dt = DT[prec]
    torch.manual_seed(13)
    dy = _rand(N, H, W, cout, dt=dt)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") * (2.0 / (9 * cin)) ** 0.5).to(dt).float()
    ref = F.conv_transpose2d(dy.float().permute(0, 3, 1, 2), w, padding=1).permute(0, 2, 3, 1)
    src = L.Src()
    src.kind, src.C, src.H, src.W, src.data = L.SRC_PLAIN, cout, H, W, dy.data_ptr()
    out = torch.empty(N, H, W, cin, dtype=dt, device="cuda")
    d = _conv(prec, [src], N, H, W, cout, w, 3, L.OUT_Y, transpose=True, out=out.data_ptr())
    assert _variant(d).startswith(f"conv3_kernel<{TN[prec]},3,1,4,"), _variant(d)
    _close_bf16(out.float(), ref, "dgrad y")


# pool-routed dgrad: dy at the pooled map -> dx into the 2x map through the recorded argmax
POOL_BENCH = [
    (4, 256, 256, 64, 128, "conv3_kernel<bf16,3,2,4,1,8,1>"),    # down1.0 dgrad -> inc output (512^2)
    (4, 128, 128, 128, 256, "conv3_kernel<bf16,3,2,4,2,8,1>"),   # down2.0 dgrad -> down1 output
    (3, 130, 166, 64, 128, "conv3_kernel<bf16,3,2,4,1,8,1>"),   # tiles16 = 297, partial tiles
]


@pytest.mark.parametrize("shape", POOL_BENCH, ids=lambda s: "x".join(map(str, s[:5])))
@pytest.mark.parametrize("with_code", [True, False])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_conv3_bench_tiles_pool_bwd(prec, shape, with_code):
    L, R = _lib(), _rt()
    N, H, W, cin, cout, want = shape
    dt = DT[prec]
    torch.manual_seed(14)
    dy = _rand(N, H, W, cout, dt=dt)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") * (2.0 / (9 * cin)) ** 0.5).to(dt).float()
    ref = F.conv_transpose2d(dy.float().permute(0, 3, 1, 2), w, padding=1).permute(0, 2, 3, 1)
    ys = _rand(N, 2 * H, 2 * W, cin, dt=dt)
    ab = torch.stack([torch.randn(cin, device="cuda"), torch.randn(cin, device="cuda") * 0.2])
    psrc = _act_src(ys, ab, kind=L.SRC_POOL_ACT)
    kw = {}
    if with_code:
        pooled = torch.empty(N, H, W, cin, dtype=dt, device="cuda")
        code = torch.empty(N, H, W, cin, dtype=torch.uint8, device="cuda")
        L.call("unet_materialize_pool", _rt()._PRECISIONS[prec].code, psrc, N, H, W, pooled.data_ptr(), code.data_ptr(), R.stream())
        kw["pool_code"] = code.data_ptr()
    src = L.Src()
    src.kind, src.C, src.H, src.W, src.data = L.SRC_PLAIN, cout, H, W, dy.data_ptr()
    da = torch.zeros(N, 2 * H, 2 * W, cin, device="cuda")
    d = _conv(prec, [src], N, H, W, cout, w, 3, L.OUT_POOL_BWD, transpose=True, out=da.data_ptr(),
              pool_src=_act_src(ys, ab), **kw)
    assert _variant(d) == want.replace("bf16", TN[prec]), _variant(d)
    a = _act_ref(ys, ab).permute(0, 3, 1, 2).requires_grad_(True)
    F.max_pool2d(a, 2).backward(ref.permute(0, 3, 1, 2))
    _close_bf16(da.permute(0, 3, 1, 2), a.grad, "pool bwd")


@pytest.mark.parametrize("shape", [(4, 512, 512, 64, 64), (4, 256, 256, 64, 128), (4, 64, 64, 512, 512)],
                         ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_wgrad_bench_sizes(prec, shape):
    """3x3 weight gradients at the benchmark's sizes (wgrad2, split-K slabs + fixed-order reduction)."""
    L, R = _lib(), _rt()
    N, H, W, cin, cout = shape
    dt = DT[prec]
    torch.manual_seed(15)
    dy = _rand(N, H, W, cout, dt=dt)
    ab = torch.stack([torch.randn(cin, device="cuda"), torch.randn(cin, device="cuda") * 0.2])
    y = _rand(N, H, W, cin, dt=dt)
    x = _act_ref(y, ab).to(dt).float().permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(x, (cout, cin, 3, 3), dy.float().permute(0, 3, 1, 2), padding=1)
    wd = L.WgradDesc()
    wd.dtype = _rt()._PRECISIONS[prec].code
    wd.N, wd.H, wd.W, wd.Cin, wd.Cout, wd.ksize, wd.nsrc = N, H, W, cin, cout, 3, 1
    wd.src[0] = _act_src(y, ab)
    wd.dy = dy.data_ptr()
    dw = torch.empty(cout, cin, 3, 3, device="cuda")
    wd.dw = dw.data_ptr()
    ws = torch.empty(max(L.load().unet_wgrad_workspace(wd), 16), dtype=torch.uint8, device="cuda")
    wd.workspace = ws.data_ptr()
    L.call("unet_conv_wgrad", wd, R.stream())
    torch.cuda.synchronize()
    rel = float((dw - ref).double().norm() / ref.double().norm())
    assert rel <= 1e-4, rel     # fp32 accumulation of exact bf16 products: only the summation order differs


@pytest.mark.parametrize("shape", [(4, 128, 128, 64, 128), (2, 66, 70, 128, 64), (4, 256, 256, 128, 64)],
                         ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("kind", ["plain", "act", "gated+plain"])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_wgrad_source_kinds(prec, shape, kind):
    """wgrad2's compile-time source-kind staging (plain map / BN+ReLU source / the up-block concat of a
    gated skip and the stored upsampled map) vs torch's conv2d_weight on the same activation."""
    L, R = _lib(), _rt()
    N, H, W, cin, cout = shape
    dt = DT[prec]
    torch.manual_seed(16)
    dy = _rand(N, H, W, cout, dt=dt)
    if kind == "plain":
        y = _rand(N, H, W, cin, dt=dt)
        src = L.Src()
        src.kind, src.C, src.H, src.W, src.data = L.SRC_PLAIN, cin, H, W, y.data_ptr()
        srcs, x = [src], y.float()
    elif kind == "act":
        y = _rand(N, H, W, cin, dt=dt)
        ab = torch.stack([torch.randn(cin, device="cuda"), torch.randn(cin, device="cuda") * 0.2])
        srcs, x = [_act_src(y, ab)], _act_ref(y, ab).to(dt).float()
    else:
        cs = cin // 2
        skip = _rand(N, H, W, cs, dt=dt)
        ab = torch.stack([torch.rand(cs, device="cuda") + 0.5, torch.randn(cs, device="cuda") * 0.2])
        p = torch.randn(N, H, W, device="cuda")
        pab = torch.tensor([0.7, -0.1], device="cuda")
        s0 = _act_src(skip, ab)
        s0.gate_p, s0.gate_ab = p.data_ptr(), pab.data_ptr()
        up = _rand(N, H, W, cin - cs, dt=dt)
        s1 = L.Src()
        s1.kind, s1.C, s1.H, s1.W, s1.data = L.SRC_PLAIN, cin - cs, H, W, up.data_ptr()
        xs = _act_ref(skip, ab) * torch.sigmoid(p * 0.7 - 0.1)[..., None]
        srcs, x = [s0, s1], torch.cat([xs.to(dt).float(), up.float()], -1)
    ref = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2), (cout, cin, 3, 3), dy.float().permute(0, 3, 1, 2),
                                      padding=1)
    wd = L.WgradDesc()
    wd.dtype = _rt()._PRECISIONS[prec].code
    wd.N, wd.H, wd.W, wd.Cin, wd.Cout, wd.ksize, wd.nsrc = N, H, W, cin, cout, 3, len(srcs)
    for i, s in enumerate(srcs):
        wd.src[i] = s
    wd.dy = dy.data_ptr()
    dw = torch.empty(cout, cin, 3, 3, device="cuda")
    wd.dw = dw.data_ptr()
    ws = torch.empty(max(L.load().unet_wgrad_workspace(wd), 16), dtype=torch.uint8, device="cuda")
    wd.workspace = ws.data_ptr()
    L.call("unet_conv_wgrad", wd, R.stream())
    torch.cuda.synchronize()
    rel = float((dw - ref).double().norm() / ref.double().norm())
    assert rel <= 2e-3, rel    # the gate / activation rounding to bf16 can differ by one ulp from torch's


@pytest.mark.parametrize("path", ["conv5", "conv3"])
@pytest.mark.parametrize("regime", ["centered", "offset"])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("shape", [(4, 256, 256, 64, 64), (4, 128, 128, 128, 128), (2, 64, 64, 256, 256),
                                   (1, 24, 40, 64, 64), (2, 20, 36, 36, 20), (3, 33, 20, 96, 128),
                                   (4, 64, 64, 256, 128)],   # conv5's MI = 2 form without split-K
                         ids=lambda s: "x".join(map(str, s)))
def test_dgrad_y_bn_backward_sums(prec, shape, regime, path, monkeypatch):
    """The dgrad y epilogue's fused BatchNorm-backward reduction (unet_conv_desc.bnb_*): per channel
    Σg and Σg·(y-mean)·invstd of the STORED gradient g, masked by the activation's ReLU, against torch
    on the same stored values (conv3 / conv2 epilogues and the fallback reduction of the other paths).
    regime "offset": y = 50 + N(0, 1) with mean ≈ 50 (|mean| >> std), where the epilogue's
    invstd·(Σg·y − mean·Σg) form cancels; its error must stay at fp32 summation-noise level relative to
    Σ|g·(y − mean)·invstd|."""
    monkeypatch.setenv("UNET_CONV5", "1" if path == "conv5" else "0")
    L, R = _lib(), _rt()
    N, H, W, cmid, cout = shape     # the conv cmid -> cout; its dgrad writes the cmid-channel gradient
    dt = DT[prec]
    torch.manual_seed(21)
    dy = _rand(N, H, W, cout, dt=dt)
    w = (torch.randn(cout, cmid, 3, 3, device="cuda") * (2.0 / (9 * cmid)) ** 0.5).to(dt).float()
    sc = torch.rand(cmid, device="cuda") + 0.5
    if regime == "offset":
        y1 = (50.0 + torch.randn(N, H, W, cmid, device="cuda")).to(dt)
        mean = 50.0 + torch.randn(cmid, device="cuda") * 0.1
        sf = -sc * 50.0 + torch.randn(cmid, device="cuda") * 0.3     # the ReLU keeps about half
    else:
        y1 = _rand(N, H, W, cmid, dt=dt)
        mean = torch.randn(cmid, device="cuda") * 0.1
        sf = torch.randn(cmid, device="cuda") * 0.3
    ab = torch.stack([sc, sf])
    invstd = torch.rand(cmid, device="cuda") + 0.5
    src = L.Src()
    src.kind, src.C, src.H, src.W, src.data = L.SRC_PLAIN, cout, H, W, dy.data_ptr()
    g = torch.empty(N, H, W, cmid, dtype=dt, device="cuda")
    P = R._PRECISIONS[prec]
    wp = R.pack_weight(w, P, transpose=True)
    d = L.ConvDesc()
    d.dtype = P.code
    d.N, d.H, d.W, d.Cin, d.Cout, d.ksize, d.nsrc = N, H, W, cout, cmid, 3, 1
    d.src[0] = src
    d.weight = wp.data_ptr()
    d.out_mode = L.OUT_Y
    d.out = g.data_ptr()
    d.bnb_y, d.bnb_scale, d.bnb_shift, d.bnb_relu = y1.data_ptr(), ab[0].data_ptr(), ab[1].data_ptr(), 1
    d.bnb_mean, d.bnb_invstd = mean.data_ptr(), invstd.data_ptr()
    ws = L.attach_workspace(d, "cuda")
    rows = L.load().unet_conv_stats_rows(d)
    part = torch.full((2, rows, cmid), float("nan"), device="cuda")
    d.bnb_stats = part.data_ptr()
    L.call("unet_conv", d, R.stream())
    torch.cuda.synchronize()
    ref = F.conv_transpose2d(dy.float().permute(0, 3, 1, 2), w, padding=1).permute(0, 2, 3, 1)
    _close_bf16(g.float(), ref, "dgrad y")
    gs = g.double().reshape(-1, cmid)
    yv = y1.double().reshape(-1, cmid)
    mask = (yv * sc.double() + sf.double()) > 0
    gm = torch.where(mask, gs, torch.zeros_like(gs))
    s1 = gm.sum(0)
    s2 = (gm * (yv - mean.double()) * invstd.double()).sum(0)
    got = part.double().sum(1)
    assert torch.isfinite(got).all(), _variant(d)
    for k, (a, b) in enumerate(((got[0], s1), (got[1], s2))):
        scale = gm.abs().sum(0) * (1 if k == 0 else float((yv - mean.double()).abs().max() * invstd.max()))
        assert ((a - b).abs() <= 1e-5 * scale + 1e-4).all(), (k, float((a - b).abs().max()), _variant(d))
    # against the natural scale of the second sum (the sum of its absolute terms)
    nat = (gm * (yv - mean.double()) * invstd.double()).abs().sum(0)
    rel = float(((got[1] - s2).abs() / (nat + 1e-30)).max())
    print(f" {regime}: Σg·x̂ max error / Σ|g·x̂| = {rel:.2e} ({_variant(d)})")
    assert rel <= 2e-5, (rel, _variant(d))


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("shape", [(2, 64, 64, 512, 512, 256), (2, 96, 80, 64, 64, 32), (1, 33, 47, 128, 128, 64)],
                         ids=lambda s: "x".join(map(str, s)))
def test_gate_psi_eval_single_pass(prec, shape):
    """unet_gate_psi_eval (the eval-mode AttentionGate in one pass, layers.py:171-192 with running-stat
    BN) against torch fp32 on the same 16-bit inputs: p = wpsi . relu(bn_g(W_g g) + bn_x(W_x relu(bn(y))))."""
    L, R = _lib(), _rt()
    N, H, W, cg, cx, ci = shape
    dt = DT[prec]
    torch.manual_seed(31)
    g = _rand(N, H, W, cg, dt=dt)
    y = _rand(N, H, W, cx, dt=dt)
    xab = torch.stack([torch.rand(cx, device="cuda") + 0.5, torch.randn(cx, device="cuda") * 0.2])
    wg = (torch.randn(ci, cg, 1, 1, device="cuda") * cg ** -0.5).to(dt).float()
    wx = (torch.randn(ci, cx, 1, 1, device="cuda") * cx ** -0.5).to(dt).float()
    gab = torch.stack([torch.rand(ci, device="cuda") + 0.5, torch.randn(ci, device="cuda") * 0.2])
    pab = torch.stack([torch.rand(ci, device="cuda") + 0.5, torch.randn(ci, device="cuda") * 0.2])
    wpsi = torch.randn(ci, device="cuda") * ci ** -0.5
    P = R._PRECISIONS[prec]
    wgp, wxp = R.pack_weight(wg, P, transpose=False), R.pack_weight(wx, P, transpose=False)
    p = torch.full((N, H, W), float("nan"), device="cuda")
    L.call("unet_gate_psi_eval", P.code, N * H * W, cg, cx, ci, g.data_ptr(), y.data_ptr(), xab[0].data_ptr(),
           xab[1].data_ptr(), 1, wgp.data_ptr(), wxp.data_ptr(), gab.data_ptr(), pab.data_ptr(), wpsi.data_ptr(),
           p.data_ptr(), R.stream())
    torch.cuda.synchronize()
    x = (y.float() * xab[0] + xab[1]).clamp_min(0).to(dt).float()      # the kernel feeds 16-bit x to the MFMA
    a = (g.float() @ wg.view(ci, cg).t()) * gab[0] + gab[1] + (x @ wx.view(ci, cx).t()) * pab[0] + pab[1]
    ref = a.clamp_min(0) @ wpsi
    rel = float((p - ref).norm() / ref.norm())
    assert torch.isfinite(p).all() and rel <= 1e-4, rel     # fp32 accumulation: summation order only


@pytest.mark.parametrize("prec", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("shape", [(4, 512, 512, 64), (2, 21, 20, 64), (3, 34, 19, 128), (1, 6, 7, 1024)],
                         ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("with_da", [True, False])
def test_bn_backward_pooled_gradient(prec, shape, with_da):
    """unet_bn_bwd_reduce_pool / _apply_pool (a Down block's MaxPool2d backward folded into the producer's
    BatchNorm backward) against the plain passes on the explicitly routed full-resolution gradient
    da + unpool(g2, code) — the same fp32 additions in the same order, so bit-identical; odd H / W
    leave the last row / column without a pooled contribution (MaxPool2d floors)."""
    L, R = _lib(), _rt()
    N, H, W, C = shape
    dt = DT[prec]
    ph, pw = H // 2, W // 2
    torch.manual_seed(23)
    y = _rand(N, H, W, C, dt=dt)
    da = torch.randn(N, H, W, C, device="cuda") if with_da else None
    g2 = torch.randn(N, ph, pw, C, device="cuda")
    code = torch.randint(0, 4, (N, ph, pw, C), dtype=torch.uint8, device="cuda")
    sc = torch.rand(C, device="cuda") + 0.5
    sf = torch.randn(C, device="cuda") * 0.3
    ab = torch.stack([sc, sf]).contiguous()
    mean = torch.randn(C, device="cuda") * 0.1
    invstd = torch.rand(C, device="cuda") + 0.5
    # the routed reference gradient
    full = da.clone() if with_da else torch.zeros(N, H, W, C, device="cuda")
    for q in range(4):
        a, b = q >> 1, q & 1
        sl = full[:, a:2 * ph:2, b:2 * pw:2, :]
        sl += torch.where(code == q, g2, torch.zeros_like(g2))
    P = N * H * W
    pc = R._PRECISIONS[prec].code
    rows = L.load().unet_bn_bwd_reduce_rows(P, C)
    part_ref = torch.empty(2, rows, C, device="cuda")
    part = torch.empty(2, rows, C, device="cuda")
    vp = R.vp
    L.call("unet_bn_bwd_reduce", pc, L.F32, P, C, vp(full), vp(y), vp(ab[0]), vp(ab[1]), 1, vp(mean), vp(invstd),
           vp(part_ref), R.stream())
    L.call("unet_bn_bwd_reduce_pool", pc, N, H, W, C, vp(da) if with_da else None, vp(g2), vp(code), ph, pw, vp(y),
           vp(ab[0]), vp(ab[1]), 1, vp(mean), vp(invstd), vp(part), R.stream())
    coef = torch.randn(3, C, device="cuda")
    dy_ref = torch.empty(N, H, W, C, dtype=dt, device="cuda")
    dy = torch.empty_like(dy_ref)
    L.call("unet_bn_bwd_apply", pc, L.F32, P, C, vp(full), vp(y), vp(ab[0]), vp(ab[1]), 1, vp(coef), vp(dy_ref),
           R.stream())
    L.call("unet_bn_bwd_apply_pool", pc, N, H, W, C, vp(da) if with_da else None, vp(g2), vp(code), ph, pw, vp(y),
           vp(ab[0]), vp(ab[1]), 1, vp(coef), vp(dy), R.stream())
    torch.cuda.synchronize()
    assert torch.equal(part, part_ref)
    assert torch.equal(dy, dy_ref)


@pytest.mark.parametrize("shape", [(4, 128, 128, 64, 32), (4, 181, 183, 64, 64), (4, 200, 170, 32, 64)],
                         ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("accum", [0, 1])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_pw_dgrad_gated(shape, accum, prec):
    """UNET_OUT_F32_GATED: the attention gate's W_x input gradient with the x*s term fused in,
    out (+)= sigmoid(p*a+b) * d(x*s) + W_x^T dy (layers.py:171-192), against torch; the pass-1 kernel then
    writes no dx (unet_gate_bwd1 with dx = NULL)."""
    L, R = _lib(), _rt()
    N, H, W, cin, cout = shape     # forward 1x1 conv cin (= Cx) -> cout (= Ci); dgrad dy[cout] -> dx[cin]
    dt = DT[prec]
    torch.manual_seed(7)
    dy = _rand(N, H, W, cout, dt=dt)
    w = (torch.randn(cout, cin, 1, 1, device="cuda") * 0.1).to(dt).float()
    dxs = torch.randn(N, H, W, cin, device="cuda")
    p = torch.randn(N, H, W, device="cuda")
    ab = torch.tensor([0.7, -0.2], device="cuda")
    old = torch.randn(N, H, W, cin, device="cuda")
    out = old.clone()
    src = L.Src()
    src.kind, src.C, src.H, src.W, src.data = L.SRC_PLAIN, cout, H, W, dy.data_ptr()
    ps = L.Src()
    ps.kind, ps.C, ps.H, ps.W = L.SRC_PLAIN, cin, H, W
    ps.data, ps.gate_p, ps.gate_ab = dxs.data_ptr(), p.data_ptr(), ab.data_ptr()
    d = _conv(prec, [src], N, H, W, cout, w, 1, L.OUT_F32_GATED, transpose=True, out=out.data_ptr(),
              split=cin, accum=accum, pool_src=ps)
    assert _pw_var(L, d).startswith("pw_conv_kernel"), _pw_var(L, d)
    s = torch.sigmoid(p * ab[0] + ab[1]).unsqueeze(-1)
    ref = F.conv_transpose2d(dy.float().permute(0, 3, 1, 2), w).permute(0, 2, 3, 1) + dxs * s
    if accum:
        ref = ref + old
    assert (out - ref).abs().max() <= 2e-2 * (1 + ref.abs().max())
    # pass 1 without dx: dq and the psi-BN sums unchanged, nothing written to dx
    R_ = _rt()
    y = _rand(N, H, W, cin, dt=dt)
    sc, sf = torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.1
    pm, pi = torch.zeros(1, device="cuda"), torch.ones(1, device="cuda")
    P = N * H * W
    rows = L.load().unet_gate_psi_rows(P)
    dq1, dq2 = torch.empty(P, device="cuda"), torch.empty(P, device="cuda")
    part1, part2 = torch.empty(2, rows, device="cuda"), torch.empty(2, rows, device="cuda")
    dx = torch.empty(N, H, W, cin, device="cuda")
    vp = R_.vp
    L.call("unet_gate_bwd1", R_._PRECISIONS[prec].code, P, cin, vp(dxs), vp(y), vp(sc), vp(sf), 1, vp(p), vp(ab), vp(pm), vp(pi), vp(dx),
           0, vp(dq1), vp(part1), R_.stream())
    L.call("unet_gate_bwd1", R_._PRECISIONS[prec].code, P, cin, vp(dxs), vp(y), vp(sc), vp(sf), 1, vp(p), vp(ab), vp(pm), vp(pi), None,
           0, vp(dq2), vp(part2), R_.stream())
    torch.cuda.synchronize()
    assert torch.equal(dq1, dq2) and torch.equal(part1, part2)
    assert torch.allclose(dx, dxs * s, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_pack_weights_batched_matches_single(prec):
    """unet_pack_weights (one launch, LDS-tiled coalesced reads: csrc/pack.hip) writes exactly the packed
    operands of the per-tensor unet_pack_weight for every job: 3x3 / 1x1, forward / transposed (dgrad), odd
    channel counts (row padding to 128, partial 32-column chunks)"""
    import ctypes
    L, R = _lib(), _rt()
    P = R._PRECISIONS[prec]
    torch.manual_seed(21)
    # round 6: 16-byte source loads for in-range tiles with 16-byte-aligned segments (Cin * taps % 4 == 0), the
    # scalar path for the rest (partial tiles, Cin = 62 / 33 / 1), padded LDS layouts for both
    shapes = [(64, 64, 3), (40, 24, 3), (130, 64, 3), (32, 64, 1), (256, 512, 1), (1024, 512, 3), (64, 1, 3), (8, 33, 3),
              (128, 36, 3), (96, 62, 1), (256, 128, 1), (48, 128, 3)]
    jobs, outs, refs = [], [], []
    for co, ci, k in shapes:
        w = torch.randn(co, ci, k, k, device="cuda")
        for tr in (0, 1):
            n = L.load().unet_packed_weight_elems(P.code, co, ci, k, tr)
            o = torch.full((n,), 7.0, dtype=DT[prec], device="cuda")
            r = R.pack_weight(w, P, transpose=bool(tr))
            j = L.PackJob()
            j.w, j.packed, j.Cout, j.Cin, j.ksize, j.transpose = w.data_ptr(), o.data_ptr(), co, ci, k, tr
            jobs.append(j); outs.append((o, w)); refs.append(r)
    arr = (L.PackJob * len(jobs))(*jobs)
    L.call("unet_pack_weights", P.code, len(jobs), arr, R.stream())
    torch.cuda.synchronize()
    for (o, _), r in zip(outs, refs):
        assert torch.equal(o.view(torch.int16), r.view(torch.int16))


def test_bn_finalize_multi_matches_single():
    """unet_bn_finalize_multi / unet_bn_bwd_finalize_multi (round 5: the attention gate's two projections
    finalized in one launch) against one unet_bn_finalize / unet_bn_bwd_finalize call per job: bit-identical,
    running statistics and num_batches_tracked included; the column-sum job against fp64 (unet_colsum's role)."""
    L, R = _lib(), _rt()
    torch.manual_seed(5)
    dev = "cuda"
    shapes = [(32, 2048, 4 * 512 * 512), (64, 1024, 4 * 256 * 256), (3, 7, 100)]
    fwd = {}
    for mode in ("single", "multi"):
        outs, jobs, keep = [], [], []
        for k, (C, rows, cnt) in enumerate(shapes):
            g = torch.Generator(device="cpu").manual_seed(100 + k)
            stats = torch.stack([torch.randn(C, rows, generator=g) * 3 + 1,
                                 torch.rand(C, rows, generator=g) * 10 + 5]).to(dev)
            gamma, beta = torch.randn(C, generator=g).to(dev), torch.randn(C, generator=g).to(dev)
            rm, rv = torch.randn(C, generator=g).to(dev), torch.rand(C, generator=g).to(dev) + 0.5
            nbt = torch.tensor([3], dtype=torch.int64, device=dev)
            o = [torch.empty(C, device=dev) for _ in range(4)]
            keep += [stats, gamma, beta]
            mom = 0.1 if k != 1 else -1.0     # momentum=None: the cumulative average reads num_batches_tracked
            if mode == "single":
                L.call("unet_bn_finalize", stats.data_ptr(), rows, C, cnt, gamma.data_ptr(), beta.data_ptr(),
                       rm.data_ptr(), rv.data_ptr(), nbt.data_ptr(), mom, 1e-5, o[0].data_ptr(), o[1].data_ptr(),
                       o[2].data_ptr(), o[3].data_ptr(), R.stream())
            else:
                j = L.BnFinJob()
                j.stats, j.rows, j.C, j.count, j.gamma, j.beta = stats.data_ptr(), rows, C, cnt, gamma.data_ptr(), beta.data_ptr()
                j.running_mean, j.running_var, j.num_batches_tracked = rm.data_ptr(), rv.data_ptr(), nbt.data_ptr()
                j.momentum, j.eps = mom, 1e-5
                j.mean, j.invstd, j.scale, j.shift = (t.data_ptr() for t in o)
                jobs.append(j)
            outs.append(o + [rm, rv, nbt])
        if mode == "multi":
            L.call("unet_bn_finalize_multi", len(jobs), (L.BnFinJob * len(jobs))(*jobs), R.stream())
        torch.cuda.synchronize()
        fwd[mode] = outs
    for a, b in zip(fwd["single"], fwd["multi"]):
        for x, y in zip(a, b):
            assert torch.equal(x, y)
    # backward: two BN jobs (as the gate's) and a column sum
    C, rows, P = 32, 2048, 4 * 512 * 512
    g = torch.Generator(device="cpu").manual_seed(7)
    part = (torch.randn(4, rows, C, generator=g) * 2).to(dev)
    gam = [torch.randn(C, generator=g).to(dev) for _ in range(2)]
    mu = [torch.randn(C, generator=g).to(dev) for _ in range(2)]
    ist = [torch.rand(C, generator=g).to(dev) + 0.5 for _ in range(2)]
    res = {}
    for mode in ("single", "multi"):
        o = [[torch.empty(C, device=dev), torch.empty(C, device=dev), torch.empty(3, C, device=dev)] for _ in range(2)]
        cs = torch.empty(C, device=dev)
        if mode == "single":
            for k in range(2):
                L.call("unet_bn_bwd_finalize", part[0].data_ptr(), part[1 + k].data_ptr(), rows, C, P, gam[k].data_ptr(),
                       mu[k].data_ptr(), ist[k].data_ptr(), o[k][0].data_ptr(), o[k][1].data_ptr(), 0, o[k][2].data_ptr(),
                       R.stream())
            L.call("unet_colsum", part[3].data_ptr(), rows, C, cs.data_ptr(), 0, R.stream())
        else:
            jobs = []
            for k in range(2):
                j = L.BnBwdFinJob()
                j.sum_g, j.sum_gx, j.rows, j.C, j.count = part[0].data_ptr(), part[1 + k].data_ptr(), rows, C, P
                j.gamma, j.mean, j.invstd = gam[k].data_ptr(), mu[k].data_ptr(), ist[k].data_ptr()
                j.dgamma, j.dbeta, j.accum, j.coef = o[k][0].data_ptr(), o[k][1].data_ptr(), 0, o[k][2].data_ptr()
                jobs.append(j)
            j = L.BnBwdFinJob()
            j.sum_g, j.sum_gx, j.rows, j.C, j.count, j.dbeta = part[3].data_ptr(), None, rows, C, 0, cs.data_ptr()
            jobs.append(j)
            L.call("unet_bn_bwd_finalize_multi", len(jobs), (L.BnBwdFinJob * len(jobs))(*jobs), R.stream())
        torch.cuda.synchronize()
        res[mode] = (o, cs)
    for k in range(2):
        for x, y in zip(res["single"][0][k], res["multi"][0][k]):
            assert torch.equal(x, y)
    ref = part[3].double().sum(0)
    for cs in (res["single"][1], res["multi"][1]):
        assert ((cs.double() - ref).abs() <= 1e-6 * part[3].double().abs().sum(0) + 1e-6).all()
