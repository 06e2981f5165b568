"""Interleaved same-process A/B of an environment switch on the network's BN-backward-sums dgrads (conv y with
bnb_* set: the dgrad of a DoubleConv's second conv, which writes the first conv's gradient and its BatchNorm-
backward sums).  Diagnostic only.
usage: python tools/bnb_ab.py VAR A B [reps]   (e.g. UNET_C5_BNB_PIPE 0 1); the switch must be read per call."""
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "unet-segment-pytorch_amd"))
import torch  # noqa: E402

from unet._hip import lib as L  # noqa: E402
from unet._hip import runtime as R  # noqa: E402

# (N, H, W, Cin = dy channels, Cout = gradient channels) of the bench step's BNB dgrads (AttentionUNet 4 x 512^2)
SHAPES = [(4, 512, 512, 64, 64), (4, 256, 256, 64, 128), (4, 256, 256, 128, 128), (4, 128, 128, 128, 256),
          (4, 128, 128, 256, 256), (4, 64, 64, 256, 512), (4, 64, 64, 512, 512)]


def desc(N, H, W, cin, cout):
    dt = torch.bfloat16
    dy = (torch.randn(N, H, W, cin, device="cuda") * 0.5).to(dt)
    w = torch.randn(cin, cout, 3, 3, device="cuda") * (2.0 / (9 * cout)) ** 0.5
    y1 = torch.randn(N, H, W, cout, device="cuda").to(dt)
    ab = torch.stack([torch.rand(cout, device="cuda") + 0.5, torch.randn(cout, device="cuda") * 0.3])
    mean, invstd = torch.randn(cout, device="cuda") * 0.1, torch.rand(cout, device="cuda") + 0.5
    g = torch.empty(N, H, W, cout, dtype=dt, device="cuda")
    P = R._PRECISIONS["bf16"]
    wp = R.pack_weight(w, P, transpose=True)
    d = L.ConvDesc()
    d.dtype = P.code
    d.N, d.H, d.W, d.Cin, d.Cout, d.ksize, d.nsrc = N, H, W, cin, cout, 3, 1
    s = L.Src()
    s.kind, s.C, s.H, s.W, s.data = L.SRC_PLAIN, cin, H, W, dy.data_ptr()
    d.src[0] = s
    d.weight = wp.data_ptr()
    d.out_mode = L.OUT_Y
    d.out = g.data_ptr()
    d.bnb_y, d.bnb_scale, d.bnb_shift, d.bnb_relu = y1.data_ptr(), ab[0].data_ptr(), ab[1].data_ptr(), 1
    d.bnb_mean, d.bnb_invstd = mean.data_ptr(), invstd.data_ptr()
    part = torch.empty(2, L.load().unet_conv_stats_rows(d), cout, device="cuda")
    d.bnb_stats = part.data_ptr()
    return d, (dy, wp, y1, ab, mean, invstd, g, part)


def timed(d, k=5):
    st = R.stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        L.call("unet_conv", d, st)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / k


def main():
    var, a, b = sys.argv[1:4]
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    tot = {a: 0.0, b: 0.0}
    for shp in SHAPES:
        d, keep = desc(*shp)
        res = {a: [], b: []}
        for v in (a, b):
            os.environ[var] = v
            timed(d, 2)
        for _ in range(reps):
            for v in (a, b):
                os.environ[var] = v
                res[v].append(timed(d))
        ma, mb = statistics.median(res[a]), statistics.median(res[b])
        tot[a] += ma
        tot[b] += mb
        print(f"{'x'.join(map(str, shp)):22s} {var}={a}: {ma:7.1f} us  {var}={b}: {mb:7.1f} us  ({100 * (mb / ma - 1):+.1f} %)",
              flush=True)
        del keep
    print(f"total {var}={a}: {tot[a]:.1f} us  {var}={b}: {tot[b]:.1f} us")


if __name__ == "__main__":
    main()
