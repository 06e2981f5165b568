"""Interleaved same-process timing of the 1x1 weight gradients (pw_wgrad) of the bench step under several values
of an environment switch read per call (e.g. UNET_PWW_BLOCKS 256 512 768 1024).  Diagnostic only.
usage: python tools/pww_ab.py VAR v1 v2 ... """
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "unet-segment-pytorch_amd"))
import torch  # noqa: E402

from unet._hip import lib as L  # noqa: E402
from unet._hip import runtime as R  # noqa: E402

# (N, H, W, Cin, Cout, act) of the step's pw_wgrad calls (AttentionUNet 4 x 512^2 gate projections)
SHAPES = [(4, 512, 512, 64, 32, False), (4, 512, 512, 64, 32, True), (4, 256, 256, 128, 64, False),
          (4, 256, 256, 128, 64, True)]


def desc(N, H, W, cin, cout, act):
    dt = torch.bfloat16
    x = torch.randn(N, H, W, cin, device="cuda").to(dt)
    dy = torch.randn(N, H, W, cout, device="cuda").to(dt)
    ab = torch.stack([torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.3])
    d = L.WgradDesc()
    d.dtype = R._PRECISIONS["bf16"].code
    d.N, d.H, d.W, d.Cin, d.Cout, d.ksize, d.nsrc = N, H, W, cin, cout, 1, 1
    s = L.Src()
    s.kind, s.C, s.H, s.W, s.data = (L.SRC_ACT if act else L.SRC_PLAIN), cin, H, W, x.data_ptr()
    if act:
        s.scale, s.shift, s.relu = ab[0].data_ptr(), ab[1].data_ptr(), 1
    d.src[0] = s
    d.dy = dy.data_ptr()
    dw = torch.empty(cout, cin, device="cuda")
    d.dw = dw.data_ptr()
    return d, [x, dy, ab, dw]


def timed(d, keep, k=5):
    st = R.stream()
    ws = torch.empty(max(L.load().unet_wgrad_workspace(d), 16), dtype=torch.uint8, device="cuda")
    d.workspace = ws.data_ptr()
    keep.append(ws)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        L.call("unet_conv_wgrad", d, st)
    e1.record()
    torch.cuda.synchronize()
    keep.pop()
    return e0.elapsed_time(e1) * 1e3 / k


def main():
    var, vals = sys.argv[1], sys.argv[2:]
    for shp in SHAPES:
        d, keep = desc(*shp)
        res = {v: [] for v in vals}
        for v in vals:
            os.environ[var] = v
            timed(d, keep, 2)
        for _ in range(10):
            for v in vals:
                os.environ[var] = v
                res[v].append(timed(d, keep))
        print(f"{'x'.join(map(str, shp)):28s} " + "  ".join(f"{var}={v}: {statistics.median(res[v]):6.1f}" for v in vals),
              flush=True)


if __name__ == "__main__":
    main()
