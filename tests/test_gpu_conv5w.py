"""conv5w (csrc/conv5w.hip, round 6: 16 rows x 32 px x 128 output channels per workgroup) against conv5 on the same
descriptors.  Both issue, per output element, the same v_mfma_f32_32x32x16 sequence (16-channel chunks in order, tap
columns dx, then rows dy), so y, act_out and the fp32 gradients must be BIT-identical; the BatchNorm partial sums are
partitioned differently (8-row wave tiles, other tiles per workgroup), so their totals agree to fp32 summation order.
Reference ops: nn.Conv2d(k=3, pad=1, bias=False) forward (unet/models/layers.py:32,35) and its input gradient; the
absolute accuracy against torch is test_gpu_conv5.py's (test_conv5_y_stats / test_conv5_dgrad_f32_split_accum run
these shapes through conv5w)."""

import pytest
import torch

from test_gpu_ops import DT, TN, _act_ref, _act_src, _conv, _lib, _rand, _rt, _variant

pytestmark = pytest.mark.gpu

SHAPES = [(4, 256, 256, 64, 128), (4, 256, 256, 128, 128), (4, 128, 128, 256, 256), (3, 200, 328, 64, 128),
          (4, 128, 128, 1024, 256), (4, 256, 256, 256, 128), (4, 100, 150, 128, 384)]   # (partial tiles both ways)
# the 8-row form (MI = 4: BN-activation y outputs on maps whose 16-row tiles do not fill the chip)
SHAPES4 = [(4, 64, 64, 1024, 512), (4, 64, 64, 512, 512), (4, 60, 90, 256, 512)]


def _srcs(L, src, N, H, W, cin, dt):
    if src == "concat":
        c0 = cin // 2
        y0 = _rand(N, H, W, c0, dt=dt)
        ab0 = torch.stack([torch.rand(c0, device="cuda") + 0.5, torch.randn(c0, device="cuda") * 0.2])
        up = _rand(N, H, W, cin - c0, dt=dt)
        s1 = L.Src()
        s1.kind, s1.C, s1.H, s1.W, s1.data = L.SRC_PLAIN, cin - c0, H, W, up.data_ptr()
        s0 = _act_src(y0, ab0)
        keep = [y0, ab0, up]
        if True:   # the network's up-block conv0: the skip is attention-gated
            p = torch.randn(N, H, W, device="cuda")
            pab = torch.tensor([0.7, -0.1], device="cuda")
            s0.gate_p, s0.gate_ab = p.data_ptr(), pab.data_ptr()
            keep += [p, pab]
        return [s0, s1], keep
    y = _rand(N, H, W, cin, dt=dt)
    if src == "plain":
        s = L.Src()
        s.kind, s.C, s.H, s.W, s.data = L.SRC_PLAIN, cin, H, W, y.data_ptr()
        return [s], [y]
    ab = torch.stack([torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.2])
    s = _act_src(y, ab)
    keep = [y, ab]
    if src == "act_gate":
        p = torch.randn(N, H, W, device="cuda")
        pab = torch.tensor([0.7, -0.1], device="cuda")
        s.gate_p, s.gate_ab = p.data_ptr(), pab.data_ptr()
        keep += [p, pab]
    return [s], keep


@pytest.mark.parametrize("shape", SHAPES + SHAPES4, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("src", ["plain", "act", "act_gate", "concat"])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_conv5w_y_matches_conv5(prec, src, shape, monkeypatch):
    if shape in SHAPES4 and src == "plain":
        pytest.skip("the 8-row form serves BN-activation sources only")
    mi = ",4" if shape in SHAPES4 else ""
    L, R = _lib(), _rt()
    N, H, W, cin, cout = shape
    dt = DT[prec]
    torch.manual_seed(51)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") * (2.0 / (9 * cin)) ** 0.5).to(dt).float()
    srcs, keep = _srcs(L, src, N, H, W, cin, dt)
    monkeypatch.setenv("UNET_CONV5", "1")
    res = {}
    for wide in ("1", "0"):
        monkeypatch.setenv("UNET_CONV5W", wide)
        d0 = L.ConvDesc()
        d0.dtype, d0.N, d0.H, d0.W, d0.Cin, d0.Cout, d0.ksize, d0.nsrc = R._PRECISIONS[prec].code, N, H, W, cin, cout, 3, len(srcs)
        for i, s in enumerate(srcs):
            d0.src[i] = s
        act = src != "plain"
        ao = torch.full((N, H, W, srcs[0].C), float("nan"), dtype=dt, device="cuda") if act else None
        if act:
            d0.act_out = ao.data_ptr()
            assert L.load().unet_conv_act_out_ok(d0)
        rows = L.load().unet_conv_stats_rows(d0)
        st = torch.full((2, cout, rows), float("nan"), device="cuda")
        out = torch.full((N, H, W, cout), float("nan"), dtype=dt, device="cuda")
        kw = {"out": out.data_ptr(), "stats": st.data_ptr()}
        if act:
            kw["act_out"] = ao.data_ptr()
        d = _conv(prec, srcs, N, H, W, cin, w, 3, L.OUT_Y, **kw)
        res[wide] = (_variant(d), out, st.double().sum(-1), ao)
    v1, y1, s1, a1 = res["1"]
    v0, y0, s0, a0 = res["0"]
    assert v1 == f"conv5w_kernel<{TN[prec]}{mi}>" and v0.startswith("conv5_kernel"), (v1, v0)
    assert torch.isfinite(y1.float()).all()
    assert torch.equal(y1, y0), float((y1.float() - y0.float()).abs().max())
    if a1 is not None:
        assert torch.equal(a1, a0)
    assert torch.isfinite(s1).all()
    assert ((s1 - s0).abs() <= 1e-5 * s0.abs() + 1e-3).all(), float((s1 - s0).abs().max())


@pytest.mark.parametrize("shape", [(4, 512, 512, 128, 64), (4, 256, 256, 256, 128), (4, 256, 256, 128, 64),
                                   (3, 200, 328, 128, 64)], ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("split", ["whole", "half"])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_conv5w_dgrad_f32_matches_conv5(prec, split, shape, monkeypatch):
    """dgrad of a forward conv cin -> cout (dy[cout] -> dx[cin], cin >= 128), fp32 stores, whole or split in two
    outputs (the concat gradient), no accumulation."""
    L = _lib()
    N, H, W, cin, cout = shape
    dt = DT[prec]
    torch.manual_seed(52)
    dy = _rand(N, H, W, cout, dt=dt)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") * (2.0 / (9 * cin)) ** 0.5).to(dt).float()
    src = L.Src()
    src.kind, src.C, src.H, src.W, src.data = L.SRC_PLAIN, cout, H, W, dy.data_ptr()
    monkeypatch.setenv("UNET_CONV5", "1")
    res = {}
    for wide in ("1", "0"):
        monkeypatch.setenv("UNET_CONV5W", wide)
        sp = cin if split == "whole" else cin // 2
        o1 = torch.full((N, H, W, sp), float("nan"), device="cuda")
        o2 = torch.full((N, H, W, max(cin - sp, 1)), float("nan"), device="cuda")
        kw = {"out": o1.data_ptr(), "split": sp}
        if sp < cin:
            kw.update(out2=o2.data_ptr(), accum=0, accum2=0)
        d = _conv(prec, [src], N, H, W, cout, w, 3, L.OUT_F32, transpose=True, **kw)
        res[wide] = (_variant(d), o1, o2)
    (v1, a1, b1), (v0, a0, b0) = res["1"], res["0"]
    assert v1 == f"conv5w_kernel<{TN[prec]}>" and v0.startswith("conv5_kernel"), (v1, v0)
    assert torch.isfinite(a1).all()
    assert torch.equal(a1, a0) and (split == "whole" or torch.equal(b1, b0))


@pytest.mark.parametrize("shape", [(4, 256, 256, 128, 128), (4, 256, 256, 64, 128), (4, 128, 128, 256, 256),
                                   (3, 200, 328, 64, 128)], ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("relu", [1, 0])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_conv5w_dgrad_bnb_matches_conv5(prec, relu, shape, monkeypatch):
    """The middle-activation dgrad with the BN-backward sums in its epilogue (dy[cout] -> g[cmid], cmid >= 128):
    g bit-identical to conv5's, the per-row sums' totals equal to fp32 summation order."""
    L, R = _lib(), _rt()
    N, H, W, cout, cmid = shape     # the dgrad conv: Cin = cout (dy channels), Cout = cmid
    dt = DT[prec]
    torch.manual_seed(53)
    dy = _rand(N, H, W, cout, dt=dt)
    y1 = _rand(N, H, W, cmid, dt=dt)
    ab = torch.stack([torch.rand(cmid, device="cuda") + 0.5, torch.randn(cmid, device="cuda") * 0.2])
    mean = torch.randn(cmid, device="cuda") * 0.1
    invstd = torch.rand(cmid, device="cuda") + 0.5
    w = (torch.randn(cout, cmid, 3, 3, device="cuda") * (2.0 / (9 * cmid)) ** 0.5).to(dt).float()
    P = R._PRECISIONS[prec]
    wp = R.pack_weight(w, P, transpose=True)
    src = L.Src()
    src.kind, src.C, src.H, src.W, src.data = L.SRC_PLAIN, cout, H, W, dy.data_ptr()
    monkeypatch.setenv("UNET_CONV5", "1")
    res = {}
    for wide in ("1", "0"):
        monkeypatch.setenv("UNET_CONV5W", wide)
        g = torch.full((N, H, W, cmid), float("nan"), dtype=dt, device="cuda")
        d = L.ConvDesc()
        d.dtype = P.code
        d.N, d.H, d.W, d.Cin, d.Cout, d.ksize, d.nsrc = N, H, W, cout, cmid, 3, 1
        d.src[0] = src
        d.weight = wp.data_ptr()
        d.out_mode = L.OUT_Y
        d.out = g.data_ptr()
        d.bnb_y, d.bnb_scale, d.bnb_shift, d.bnb_relu = y1.data_ptr(), ab[0].data_ptr(), ab[1].data_ptr(), relu
        d.bnb_mean, d.bnb_invstd = mean.data_ptr(), invstd.data_ptr()
        ws = L.attach_workspace(d, "cuda")
        rows = L.load().unet_conv_stats_rows(d)
        part = torch.full((2, rows, cmid), float("nan"), device="cuda")
        d.bnb_stats = part.data_ptr()
        L.call("unet_conv", d, R.stream())
        torch.cuda.synchronize()
        res[wide] = (_variant(d), g, part.double().sum(1))
        del ws
    (v1, g1, s1), (v0, g0, s0) = res["1"], res["0"]
    assert v1 == f"conv5w_kernel<{TN[prec]}>" and v0.startswith("conv5_kernel"), (v1, v0)
    assert torch.isfinite(g1.float()).all()
    assert torch.equal(g1, g0)
    # reference sums of the stored gradient (fp64): sum g' and sum g' * (y1 - mean) * invstd, g' = g masked by ReLU
    gg = g0.double()
    if relu:
        gg = torch.where(y1.double() * ab[0].double() + ab[1].double() > 0, gg, torch.zeros_like(gg))
    ref0 = gg.reshape(-1, cmid).sum(0)
    ref1 = (gg * (y1.double() - mean.double()) * invstd.double()).reshape(-1, cmid).sum(0)
    for got, ref in ((s1[0], ref0), (s1[1], ref1), (s0[0], ref0), (s0[1], ref1)):
        assert torch.isfinite(got).all()
        assert ((got - ref).abs() <= 1e-4 * gg.abs().reshape(-1, cmid).sum(0) + 1e-3).all(), float((got - ref).abs().max())
