"""Run one full-size bf16 3x3 weight-gradient launch repeatedly (PMC / timing target, diagnostic).
usage: python tools/wgrad_one.py [N H W Cin Cout] [reps]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "unet-segment-pytorch_amd"))
import torch  # noqa: E402

from unet._hip import lib as L  # noqa: E402
from unet._hip.runtime import stream  # noqa: E402

a = [int(v) for v in sys.argv[1:6]] if len(sys.argv) > 5 else [4, 512, 512, 64, 64]
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 20
N, H, W, cin, cout = a
dev = "cuda"
y = torch.randn(N, H, W, cin, device=dev).to(torch.bfloat16)
ab = torch.stack([torch.rand(cin, device=dev) + 0.5, torch.randn(cin, device=dev) * 0.1]).contiguous()
dy = torch.randn(N, H, W, cout, device=dev).to(torch.bfloat16)
wd = L.WgradDesc()
wd.dtype = L.BF16
wd.N, wd.H, wd.W, wd.Cin, wd.Cout, wd.ksize, wd.nsrc = N, H, W, cin, cout, 3, 1
s = wd.src[0]
import os  # noqa: E402
if os.environ.get("WG_KIND", "act") == "plain":
    s.kind, s.C, s.H, s.W, s.data = L.SRC_PLAIN, cin, H, W, y.data_ptr()
else:
    s.kind, s.C, s.H, s.W, s.data = L.SRC_ACT, cin, H, W, y.data_ptr()
    s.scale, s.shift, s.relu = ab[0].data_ptr(), ab[1].data_ptr(), 1
wd.dy = dy.data_ptr()
dw = torch.empty(cout, cin, 3, 3, device=dev)
wd.dw = dw.data_ptr()
ws = torch.empty(max(L.load().unet_wgrad_workspace(wd), 16), dtype=torch.uint8, device=dev)
wd.workspace = ws.data_ptr()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for i in range(reps):
    if i == reps // 2:
        ev[0].record()
    L.call("unet_conv_wgrad", wd, stream())
ev[1].record()
torch.cuda.synchronize()
us = ev[0].elapsed_time(ev[1]) * 1e3 / (reps - reps // 2)
fl = 2.0 * N * H * W * cin * cout * 9
from unet._hip.runtime import wgrad_kernel_name  # noqa: E402
print(f"{wgrad_kernel_name(wd)} {os.environ.get('WG_KIND', 'act')} {N}x{H}x{W} {cin}->{cout}: {us:.1f} us/launch (incl. reduce), {fl / us / 1e6:.1f} TF/s")
