"""Op test of `unet_materialize` (csrc/misc.hip: the LDS-tiled Up-block kernel since round 5 for 16-bit maps, the
packed-fp32 per-element kernel otherwise and under UNET_MAT_TILE=0): the
bilinear x2 upsample (align_corners=True) of relu?(y * scale + shift), placed with the skip-size padding —
the decoder input of every Up block (reference unet/models/layers.py:78,183 `nn.Upsample(scale_factor=2,
mode='bilinear', align_corners=True)` + the pad of :98-102) — against F.interpolate / F.pad in fp64.

Bound, per output element, derived a priori (not fitted): the kernel forms a_i = relu(fma(y_i, s, b)) in fp32
(one rounding: <= 2^-24 |a_i|), blends the four corners with fp32 weights whose source coordinate o * (in-1)/(out-1)
is rounded once in fp32 (weight error <= 2^-24 * 2 * in_size, times the corner spread <= 2 max|a_i|), with a few
fp32 roundings in the blend (<= 8 * 2^-24 * sum w_i |a_i|), and rounds once to the output type (half an ulp of
the computed value).  So |out - exact| <= 0.5 ulp_T(|exact| + e) + e with
e = 2^-24 (8 sum w_i|a_i| + 4 in_size max|a_i|).  Where the exact value is not a cancellation this is within
half an output ulp (plus the tiny fp32 term); tools/mat_diag.py printed the same comparison in round 4."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DT = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}
MANT = {"bf16": 7, "fp16": 10, "fp32": 23}

# (N, h, w, C, H, W): source map and output (skip) size; H = 2h / W = 2w except the padded cases
SHAPES = [(4, 32, 32, 512, 64, 64), (4, 64, 64, 256, 128, 128), (4, 128, 128, 128, 256, 256),
          (4, 256, 256, 64, 512, 512), (2, 3, 5, 64, 6, 10), (2, 17, 64, 128, 34, 128),
          (2, 17, 24, 64, 37, 49)]


def _ulp(x, prec):
    """spacing of the output type at |x| (normal range; the subnormal spacing below it)"""
    fi = torch.finfo(DT[prec])
    m, e = torch.frexp(x.abs().clamp_min(fi.tiny))
    return torch.ldexp(torch.ones_like(x), (e - 1 - MANT[prec]).to(torch.int32)).clamp_min(fi.tiny * fi.eps)


def _corner_terms(a, H, W, pad_t, pad_l, h, w):
    """fp64 sum_i w_i |a_i| and max_i |a_i| over the four corners of every output pixel (zeros in the padding)"""
    uh, uw = 2 * h, 2 * w

    def axis(n_out, n_in, pad, n_up):
        o = torch.arange(n_out, device=a.device, dtype=torch.float64) - pad
        s = o * ((n_in - 1) / (n_up - 1) if n_up > 1 else 0.0)
        i0 = s.floor().clamp(0, n_in - 1).long()
        i1 = (i0 + 1).clamp(max=n_in - 1)
        lam = (s - i0).clamp(0, 1)
        inside = (o >= 0) & (o < n_up)
        return i0, i1, lam, inside

    y0, y1, ly, iy = axis(H, h, pad_t, uh)
    x0, x1, lx, ix = axis(W, w, pad_l, uw)
    aa = a.abs()
    c = [aa[:, y0][:, :, x0], aa[:, y0][:, :, x1], aa[:, y1][:, :, x0], aa[:, y1][:, :, x1]]
    wy = [(1 - ly)[None, :, None, None], ly[None, :, None, None]]
    wx = [(1 - lx)[None, None, :, None], lx[None, None, :, None]]
    S = wy[0] * wx[0] * c[0] + wy[0] * wx[1] * c[1] + wy[1] * wx[0] * c[2] + wy[1] * wx[1] * c[3]
    M = torch.maximum(torch.maximum(c[0], c[1]), torch.maximum(c[2], c[3]))
    mask = (iy[None, :, None, None] & ix[None, None, :, None]).double()
    return S * mask, M * mask


@pytest.mark.parametrize("relu", [True, False])
@pytest.mark.parametrize("prec", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_materialize_vs_fp64_interpolate(shape, prec, relu):
    from unet._hip import lib as L
    from unet._hip import runtime as R
    N, h, w, C, H, W = shape
    pad_t, pad_l = (H - 2 * h) // 2, (W - 2 * w) // 2        # layers.py:98-102: diff // 2 before, the rest after
    torch.manual_seed(23)
    y = torch.randn(N, h, w, C, device="cuda").to(DT[prec])
    ab = torch.stack([torch.randn(C, device="cuda"), torch.randn(C, device="cuda") * 0.2])
    s = L.Src()
    s.kind, s.H, s.W, s.C, s.data = L.SRC_UP_ACT, h, w, C, y.data_ptr()
    s.scale, s.shift, s.relu = ab[0].data_ptr(), ab[1].data_ptr(), int(relu)
    s.up_h, s.up_w, s.pad_t, s.pad_l = 2 * h, 2 * w, pad_t, pad_l
    s.sh, s.sw = R.up_scale(h, 2 * h), R.up_scale(w, 2 * w)
    o = torch.full((N, H, W, C), float("nan"), dtype=DT[prec], device="cuda")
    L.call("unet_materialize", R._PRECISIONS[prec].code, s, N, H, W, o.data_ptr(), R.stream())
    torch.cuda.synchronize()
    a = y.double() * ab[0].double() + ab[1].double()
    a = torch.relu(a) if relu else a
    ref = F.interpolate(a.permute(0, 3, 1, 2), scale_factor=2, mode="bilinear", align_corners=True)
    ref = F.pad(ref, [pad_l, W - 2 * w - pad_l, pad_t, H - 2 * h - pad_t]).permute(0, 2, 3, 1)
    S, M = _corner_terms(a, H, W, pad_t, pad_l, h, w)
    e32 = 2.0 ** -24 * (8 * S + 4 * max(h, w) * M)
    tol = 0.5 * _ulp(ref.abs() + e32, prec) + e32
    err = (o.double() - ref).abs()
    assert not o.isnan().any()
    bad = err > tol
    inside = torch.zeros(H, W, dtype=torch.bool, device="cuda")
    inside[pad_t:pad_t + 2 * h, pad_l:pad_l + 2 * w] = True
    assert bool((o[:, ~inside] == 0).all()), "the padding must be exact zeros"
    half = float((err <= 0.5 * _ulp(ref.abs(), prec)).double().mean())
    print(f"\n{prec} relu={int(relu)} {shape}: max|err| {float(err.max()):.3e}, max err/tol {float((err / tol).max()):.3f}, "
          f"fraction within half an output ulp of the exact value {half:.6f}")
    assert not bool(bad.any()), (int(bad.sum()), float((err / tol).max()))


@pytest.mark.parametrize("relu", [True, False])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("shape", SHAPES + [(1, 9, 7, 8, 23, 20), (3, 11, 40, 16, 22, 85), (2, 8, 8, 24, 16, 16)],
                         ids=lambda s: "x".join(map(str, s)))
def test_materialize_tile_bit_identical_to_per_pixel(shape, prec, relu, monkeypatch):
    """The tiled form (materialize_up_tile_kernel) stages the source span once and blends from LDS with the same
    tap indices, weights and fma order as the per-pixel form: the two maps are bit-identical (C = 8 / 16 / 24:
    one and two channel vectors per block, and a channel count the tiled form leaves to the per-pixel one)."""
    from unet._hip import lib as L
    from unet._hip import runtime as R
    N, h, w, C, H, W = shape
    pad_t, pad_l = (H - 2 * h) // 2, (W - 2 * w) // 2
    torch.manual_seed(29)
    y = torch.randn(N, h, w, C, device="cuda").to(DT[prec])
    ab = torch.stack([torch.randn(C, device="cuda"), torch.randn(C, device="cuda") * 0.2])
    s = L.Src()
    s.kind, s.H, s.W, s.C, s.data = L.SRC_UP_ACT, h, w, C, y.data_ptr()
    s.scale, s.shift, s.relu = ab[0].data_ptr(), ab[1].data_ptr(), int(relu)
    s.up_h, s.up_w, s.pad_t, s.pad_l = 2 * h, 2 * w, pad_t, pad_l
    s.sh, s.sw = R.up_scale(h, 2 * h), R.up_scale(w, 2 * w)
    outs = []
    for tile in ("1", "0"):
        monkeypatch.setenv("UNET_MAT_TILE", tile)
        o = torch.full((N, H, W, C), float("nan"), dtype=DT[prec], device="cuda")
        L.call("unet_materialize", R._PRECISIONS[prec].code, s, N, H, W, o.data_ptr(), R.stream())
        outs.append(o)
    torch.cuda.synchronize()
    assert not outs[0].isnan().any()
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))
