"""conv5 (csrc/conv5.hip: the LDS-DMA 3x3 conv on v_mfma_f32_32x32x16, the default path on large maps)
against torch fp32 on the same 16-bit operands, for every epilogue and source kind they serve, at bench sizes (the persistent multi-tile loop runs) and with
partial tiles in both directions.  Reference ops: nn.Conv2d(k=3, pad=1, bias=False) forward
(unet/models/layers.py:32,35) and its input gradient; BatchNorm2d forward partial sums / backward sums of
the DoubleConv (layers.py:33,36).  Gates as the conv3 bench-tile tests: rel-L2 <= 4e-3, max-abs <= 2e-2 (1 +
max|ref|); sums against fp64 sums of the same stored values."""

import pytest
import torch
import torch.nn.functional as F

from test_gpu_ops import DT, TN, _act_ref, _act_src, _close_bf16, _conv, _lib, _rand, _rt, _variant

pytestmark = pytest.mark.gpu

Y_SHAPES = [(4, 512, 512, 64, 64), (4, 256, 256, 64, 128), (4, 256, 256, 128, 128), (4, 128, 128, 256, 256),
            (3, 200, 328, 64, 128), (8, 258, 98, 96, 64),
            (2, 128, 128, 1024, 256)]   # a 1024-channel (C5_CMAX) activation: the scale / shift table's padding


PATH = {"conv5": {"UNET_CONV5": "1"}}


def _wide(N, H, W, cin, cout, mode="y", src="plain"):
    """conv5w (csrc/conv5w.hip, round 6) serves, by default, the BN-activation forwards with >= 256 input channels
    and >= 128 output channels whose 16 x 32 x 128 tiles (or else 8 x 32 x 128: ",4") fill the chip (conv5w_ok)"""
    if not (mode == "y" and src != "plain" and cin >= 256 and cout % 128 == 0):
        return None
    for mi, suffix in ((8, ""), (4, ",4")):
        if N * -(-W // 32) * -(-H // (2 * mi)) * (cout // 128) >= 256:
            return suffix
    return None


def _want(prec, cout, path, shape=None, mode="y", src="plain"):
    if shape is not None:
        w = _wide(shape[0], shape[1], shape[2], shape[3], cout, mode, src)
        if w is not None:
            return f"conv5w_kernel<{TN[prec]}{w}>"
    return f"conv5_kernel<{TN[prec]},4>"


@pytest.fixture(params=["conv5"])
def path(request, monkeypatch):
    for k, v in PATH[request.param].items():
        monkeypatch.setenv(k, v)
    return request.param


@pytest.mark.parametrize("shape", Y_SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("src", ["plain", "act", "act_gate", "concat"])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_conv5_y_stats(prec, src, shape, path):
    L, R = _lib(), _rt()
    N, H, W, cin, cout = shape
    dt = DT[prec]
    torch.manual_seed(31)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") * (2.0 / (9 * cin)) ** 0.5).to(dt).float()
    if src == "concat":
        c0 = cin // 2 if (cin // 2) % 16 == 0 else 32
        y0 = _rand(N, H, W, c0, dt=dt)
        ab0 = torch.stack([torch.rand(c0, device="cuda") + 0.5, torch.randn(c0, device="cuda") * 0.2])
        up = _rand(N, H, W, cin - c0, dt=dt)
        s1 = L.Src()
        s1.kind, s1.C, s1.H, s1.W, s1.data = L.SRC_PLAIN, cin - c0, H, W, up.data_ptr()
        srcs = [_act_src(y0, ab0), s1]
        x = torch.cat([_act_ref(y0, ab0).to(dt).float(), up.float()], -1)
    else:
        y = _rand(N, H, W, cin, dt=dt)
        if src == "plain":
            s = L.Src()
            s.kind, s.C, s.H, s.W, s.data = L.SRC_PLAIN, cin, H, W, y.data_ptr()
            x = y.float()
        else:
            ab = torch.stack([torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.2])
            s = _act_src(y, ab)
            a = _act_ref(y, ab)
            if src == "act_gate":
                p = torch.randn(N, H, W, device="cuda")
                pab = torch.tensor([0.7, -0.1], device="cuda")
                s.gate_p, s.gate_ab = p.data_ptr(), pab.data_ptr()
                a = a * torch.sigmoid(p * 0.7 - 0.1)[..., None]
            x = a.to(dt).float()
        srcs = [s]
    d0 = L.ConvDesc()
    d0.dtype, d0.N, d0.H, d0.W, d0.Cin, d0.Cout, d0.ksize, d0.nsrc = R._PRECISIONS[prec].code, N, H, W, cin, cout, 3, len(srcs)
    for i, s in enumerate(srcs):
        d0.src[i] = s
    ws0 = L.attach_workspace(d0, "cuda")   # (the split-K forms' row count: ask with a workspace, as _conv launches)
    rows = L.load().unet_conv_stats_rows(d0)
    st = torch.full((2, cout, rows), float("nan"), device="cuda")
    out = torch.empty(N, H, W, cout, dtype=dt, device="cuda")
    d = _conv(prec, srcs, N, H, W, cin, w, 3, L.OUT_Y, out=out.data_ptr(), stats=st.data_ptr())
    assert _variant(d) == _want(prec, cout, path, shape, "y", src), _variant(d)
    ref = F.conv2d(x.permute(0, 3, 1, 2), w, padding=1).permute(0, 2, 3, 1)
    _close_bf16(out.float(), ref, "y")
    r = ref.double().reshape(-1, cout)
    sm = st.double().sum(-1)
    assert torch.isfinite(sm).all()
    assert ((sm[0] - r.sum(0)).abs() <= 1e-3 * r.abs().sum(0) + 1e-2).all()
    assert ((sm[1] - (r * r).sum(0)).abs() <= 1e-2 * (r * r).sum(0) + 1e-2).all()


DGRAD_SHAPES = [(4, 512, 512, 128, 64), (4, 512, 512, 64, 64), (4, 256, 256, 256, 128), (4, 256, 256, 64, 128),
                (3, 200, 328, 128, 64), (8, 258, 98, 64, 96)]


@pytest.mark.parametrize("shape", DGRAD_SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_conv5_dgrad_f32_split_accum(prec, shape, path):
    """dgrad of a forward conv cin -> cout: dy[cout] -> dx[cin], fp32, split across the concat with the first
    part accumulated (UNET_OUT_F32)."""
    L = _lib()
    N, H, W, cin, cout = shape
    dt = DT[prec]
    torch.manual_seed(32)
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
    assert _variant(d) == _want(prec, cin, path, shape, "f32"), _variant(d)
    _close_bf16(torch.cat([o1 - 0.5, o2], -1), ref, "dgrad f32")
    # unsplit, stored
    o = torch.full((N, H, W, cin), float("nan"), device="cuda")
    _conv(prec, [src], N, H, W, cout, w, 3, L.OUT_F32, transpose=True, out=o.data_ptr(), split=cin)
    _close_bf16(o, ref, "dgrad f32 stored")


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_conv5_matches_conv3(prec, path, monkeypatch):
    """The 32x32x16 kernels and conv3 on the same inputs agree to fp32 summation-order noise."""
    L = _lib()
    N, H, W, cin, cout = 4, 256, 256, 128, 128
    dt = DT[prec]
    torch.manual_seed(33)
    y = _rand(N, H, W, cin, dt=dt)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") * (2.0 / (9 * cin)) ** 0.5).to(dt).float()
    outs = []
    for flag in ("1", "0"):
        for k, v in PATH[path].items():
            monkeypatch.setenv(k, v if flag == "1" else "0")
        o = torch.full((N, H, W, cout), float("nan"), device="cuda")
        src = L.Src()
        src.kind, src.C, src.H, src.W, src.data = L.SRC_PLAIN, cout, H, W, y.data_ptr()
        d = _conv(prec, [src], N, H, W, cin, w, 3, L.OUT_F32, transpose=True, out=o.data_ptr(), split=cin)
        outs.append((_variant(d), o))
    (v4, o4), (v3, o3) = outs
    assert v4.startswith(path) and v3.startswith("conv3_kernel"), (v4, v3)
    rel = float((o4 - o3).double().norm() / o3.double().norm())
    assert rel <= 1e-5, rel


# ---- small maps (round 5): maps whose 16 x 32 x 64 tiles do not fill the chip (down4 at 32^2, up1.conv.3 at 64^2):
# split-K over the input channels, and the 8-row (MI = 2) tiles, which halve the splits or need none.
# mi2 "0": the MI = 4 split-K form alone (UNET_CONV5_MI2=0); "1": the default (MI = 2, split where still needed)
SPLIT_SHAPES = [(4, 32, 32, 512, 512), (4, 64, 64, 512, 256), (2, 16, 16, 256, 128), (2, 16, 24, 64, 64)]


def _small_map_form(v, prec, mi2):
    if mi2 == "0":
        return v.startswith(f"conv5_kernel<{TN[prec]},4>+splitk")
    return v.startswith(f"conv5_kernel<{TN[prec]},2>")


@pytest.mark.parametrize("mi2", ["0", "1"])
@pytest.mark.parametrize("shape", SPLIT_SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("src", ["plain", "act", "act_gate", "concat"])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_conv5_splitk_y_stats(prec, src, shape, mi2, monkeypatch):
    """The small-map forms against torch fp32 on the same operands: y and the BN partial sums (same gates as the
    persistent form), and bit-identical across two runs (split-K slabs are added in a fixed order)."""
    monkeypatch.setenv("UNET_CONV5_MI2", mi2)
    L, R = _lib(), _rt()
    N, H, W, cin, cout = shape
    dt = DT[prec]
    torch.manual_seed(41)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") * (2.0 / (9 * cin)) ** 0.5).to(dt).float()
    if src == "concat":
        c0 = cin // 2
        y0 = _rand(N, H, W, c0, dt=dt)
        ab0 = torch.stack([torch.rand(c0, device="cuda") + 0.5, torch.randn(c0, device="cuda") * 0.2])
        up = _rand(N, H, W, cin - c0, dt=dt)
        s1 = L.Src()
        s1.kind, s1.C, s1.H, s1.W, s1.data = L.SRC_PLAIN, cin - c0, H, W, up.data_ptr()
        srcs = [_act_src(y0, ab0), s1]
        x = torch.cat([_act_ref(y0, ab0).to(dt).float(), up.float()], -1)
    else:
        y = _rand(N, H, W, cin, dt=dt)
        if src == "plain":
            s = L.Src()
            s.kind, s.C, s.H, s.W, s.data = L.SRC_PLAIN, cin, H, W, y.data_ptr()
            x = y.float()
        else:
            ab = torch.stack([torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.2])
            s = _act_src(y, ab)
            a = _act_ref(y, ab)
            if src == "act_gate":
                p = torch.randn(N, H, W, device="cuda")
                pab = torch.tensor([0.7, -0.1], device="cuda")
                s.gate_p, s.gate_ab = p.data_ptr(), pab.data_ptr()
                a = a * torch.sigmoid(p * 0.7 - 0.1)[..., None]
            x = a.to(dt).float()
        srcs = [s]
    d0 = L.ConvDesc()
    d0.dtype, d0.N, d0.H, d0.W, d0.Cin, d0.Cout, d0.ksize, d0.nsrc = R._PRECISIONS[prec].code, N, H, W, cin, cout, 3, len(srcs)
    for i, s in enumerate(srcs):
        d0.src[i] = s
    ws0 = L.attach_workspace(d0, "cuda")   # (the split-K forms' row count: ask with a workspace, as _conv launches)
    rows = L.load().unet_conv_stats_rows(d0)
    outs = []
    for _ in range(2):
        st = torch.full((2, cout, rows), float("nan"), device="cuda")
        out = torch.full((N, H, W, cout), float("nan"), dtype=dt, device="cuda")
        d = _conv(prec, srcs, N, H, W, cin, w, 3, L.OUT_Y, out=out.data_ptr(), stats=st.data_ptr())
        outs.append((out, st))
    v = _variant(d)
    assert _small_map_form(v, prec, mi2), v
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])   # deterministic
    out, st = outs[0]
    ref = F.conv2d(x.permute(0, 3, 1, 2), w, padding=1).permute(0, 2, 3, 1)
    _close_bf16(out.float(), ref, "y")
    r = ref.double().reshape(-1, cout)
    sm = st.double().sum(-1)
    assert torch.isfinite(sm).all()
    assert ((sm[0] - r.sum(0)).abs() <= 1e-3 * r.abs().sum(0) + 1e-2).all()
    assert ((sm[1] - (r * r).sum(0)).abs() <= 1e-2 * (r * r).sum(0) + 1e-2).all()


@pytest.mark.parametrize("prec", ["bf16"])
def test_conv5_small_map_without_workspace(prec, monkeypatch):
    """a descriptor without a workspace (a zero-initialised C caller) on a split-K shape runs the unsplit
    form — correct y and BN sums, and unet_conv_stats_rows asked the same way agrees with what the launch writes."""
    monkeypatch.setenv("UNET_CONV5_MI2", "1")
    L, R = _lib(), _rt()
    N, H, W, cin, cout = 4, 32, 32, 512, 512
    dt = DT[prec]
    torch.manual_seed(43)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") * (2.0 / (9 * cin)) ** 0.5).to(dt).float()
    y = _rand(N, H, W, cin, dt=dt)
    s = L.Src()
    s.kind, s.C, s.H, s.W, s.data = L.SRC_PLAIN, cin, H, W, y.data_ptr()
    P = R._PRECISIONS[prec]
    d = L.ConvDesc()
    d.dtype, d.N, d.H, d.W, d.Cin, d.Cout, d.ksize, d.nsrc = P.code, N, H, W, cin, cout, 3, 1
    d.src[0] = s
    assert L.load().unet_conv_workspace(d) > 0          # the shape has a split-K form
    wp = R.pack_weight(w, P, transpose=False)
    rows = L.load().unet_conv_stats_rows(d)
    st = torch.full((2, cout, rows), float("nan"), device="cuda")
    out = torch.full((N, H, W, cout), float("nan"), dtype=dt, device="cuda")
    d.weight, d.out_mode, d.out, d.stats = wp.data_ptr(), L.OUT_Y, out.data_ptr(), st.data_ptr()
    assert "splitk" not in _variant(d), _variant(d)
    L.call("unet_conv", d, R.stream())
    torch.cuda.synchronize()
    ref = F.conv2d(y.float().permute(0, 3, 1, 2), w, padding=1).permute(0, 2, 3, 1)
    _close_bf16(out.float(), ref, "y")
    r = ref.double().reshape(-1, cout)
    sm = st.double().sum(-1)
    assert torch.isfinite(sm).all()
    assert ((sm[0] - r.sum(0)).abs() <= 1e-3 * r.abs().sum(0) + 1e-2).all()


SPLIT_DGRAD_SHAPES = [(4, 32, 32, 512, 512), (4, 32, 32, 256, 512), (2, 16, 16, 256, 128), (2, 16, 24, 64, 64),
                      (4, 64, 64, 256, 512)]   # the last: MI = 2 without split-K (the network's 64^2 512 -> 256 dgrad form)


@pytest.mark.parametrize("mi2", ["0", "1"])
@pytest.mark.parametrize("shape", SPLIT_DGRAD_SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_conv5_splitk_dgrad_f32_split_accum(prec, shape, mi2, monkeypatch):
    """The small-map fp32 dgrad epilogues: split across the concat, the first part accumulated, and unsplit."""
    monkeypatch.setenv("UNET_CONV5_MI2", mi2)
    L = _lib()
    N, H, W, cin, cout = shape
    dt = DT[prec]
    torch.manual_seed(42)
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
    v = _variant(d)
    assert _small_map_form(v, prec, mi2), v
    _close_bf16(torch.cat([o1 - 0.5, o2], -1), ref, "dgrad f32")
    o = torch.full((N, H, W, cin), float("nan"), device="cuda")
    _conv(prec, [src], N, H, W, cout, w, 3, L.OUT_F32, transpose=True, out=o.data_ptr(), split=cin)
    _close_bf16(o, ref, "dgrad f32 stored")
