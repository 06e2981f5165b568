"""Diagnostic: unet_materialize (bilinear x2 of relu?(bn(x)), per-element kernel) against F.interpolate in fp64,
per case: max abs error and the error in output-type ulps.  Not part of the product or the tests."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "unet-segment-pytorch_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from unet._hip import lib as L  # noqa: E402
from unet._hip import runtime as R  # noqa: E402

DT = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}
for prec in ("bf16", "fp32"):
    for relu in (True, False):
        for (N, h, w, C) in ((2, 3, 5, 64), (4, 32, 32, 512), (4, 32, 32, 64), (2, 17, 64, 128), (4, 64, 64, 256)):
            torch.manual_seed(23)
            y = (torch.randn(N, h, w, C, device="cuda")).to(DT[prec])
            ab = torch.stack([torch.randn(C, device="cuda"), torch.randn(C, device="cuda") * 0.2])
            s = L.Src()
            s.kind, s.H, s.W, s.C, s.data = L.SRC_UP_ACT, h, w, C, y.data_ptr()
            s.scale, s.shift, s.relu = ab[0].data_ptr(), ab[1].data_ptr(), int(relu)
            s.up_h, s.up_w, s.pad_t, s.pad_l = 2 * h, 2 * w, 0, 0
            s.sh, s.sw = R.up_scale(h, 2 * h), R.up_scale(w, 2 * w)
            o = torch.full((N, 2 * h, 2 * w, C), float("nan"), dtype=DT[prec], device="cuda")
            L.call("unet_materialize", R._PRECISIONS[prec].code, s, N, 2 * h, 2 * w, o.data_ptr(), R.stream())
            torch.cuda.synchronize()
            a = y.double() * ab[0].double() + ab[1].double()
            a = torch.relu(a) if relu else a
            ref = F.interpolate(a.permute(0, 3, 1, 2), scale_factor=2, mode="bilinear", align_corners=True)
            ref = ref.permute(0, 2, 3, 1)
            err = (o.double() - ref).abs()
            spacing = torch.finfo(DT[prec]).eps * ref.abs().clamp_min(torch.finfo(DT[prec]).tiny)
            print(f"{prec} relu={int(relu)} {N}x{h}x{w}x{C}: nan={int(o.isnan().sum())} max|err|={float(err.max()):.3e} "
                  f"max err/eps|ref|={float((err / spacing).max()):.2f} worst at {tuple(int(i) for i in (err == err.max()).nonzero()[0])}")
