"""Ablation timing of conv5_kernel (csrc/conv5.hip, bf16 y mode) on full-size layers (diagnostic, GPU).
Modes (bits): 1 no in-loop halo DMA; 2 no in-loop weight DMA; 4 no epilogue stores / sums; 8 no per-chunk
barrier; 16 no BN transform.  Times are medians of 10 launches; results are garbage for modes != 0.
--split: the split-K form on the small maps (the split kernel alone with the same bits; mode -1 = its y + BN-stats
finisher alone)."""
import ctypes
import os
os.environ["UNET_CONV5"] = "1"
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "unet-segment-pytorch_amd"))
import torch  # noqa: E402

from unet._hip import lib as L  # noqa: E402
from unet._hip.runtime import pack_weight, BF16, f32  # noqa: E402

lib = L.load()
lib.unet_diag_conv5_ablate.argtypes = [ctypes.POINTER(L.ConvDesc), ctypes.c_int, ctypes.c_void_p]
if "--conv5" in sys.argv:     # accepted for older command lines
    sys.argv.remove("--conv5")
lib.unet_diag_conv5_split_ablate.argtypes = [ctypes.POINTER(L.ConvDesc), ctypes.c_int, ctypes.c_void_p]
SPLIT = "--split" in sys.argv
if SPLIT:
    sys.argv.remove("--split")
FN = lib.unet_diag_conv5_split_ablate if SPLIT else lib.unet_diag_conv5_ablate


def layer(N, H, W, cin, cout, kind):
    dev = "cuda"
    x = torch.randn(N, H, W, cin, device=dev).to(torch.bfloat16)
    w = torch.randn(cout, cin, 3, 3, device=dev) * 0.05
    wp = pack_weight(w, BF16, transpose=False)
    ab = torch.stack([torch.rand(cin, device=dev) + 0.5, torch.randn(cin, device=dev) * 0.1]).contiguous()
    d = L.ConvDesc()
    d.dtype = L.BF16
    d.N, d.H, d.W, d.Cin, d.Cout, d.ksize, d.nsrc = N, H, W, cin, cout, 3, 1
    s = d.src[0]
    s.kind = kind
    s.C, s.H, s.W = cin, H, W
    s.data = x.data_ptr()
    s.scale, s.shift, s.relu = ab[0].data_ptr(), ab[1].data_ptr(), 1
    d.weight = wp.data_ptr()
    y = torch.empty(N, H, W, cout, dtype=torch.bfloat16, device=dev)
    d.out_mode = L.OUT_Y
    d.out = y.data_ptr()
    ws = torch.empty(max(lib.unet_conv_workspace(ctypes.byref(d)), 16), dtype=torch.uint8, device=dev)
    d.workspace = ws.data_ptr()
    rows = lib.unet_conv_stats_rows(d)
    st = f32(2, cout, rows, device=dev)
    d.stats = st.data_ptr()
    return d, (x, w, wp, ab, y, st, ws)


def main():
    modes = [int(m) for m in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3,4,8,7,15,16,31").split(",")]
    layers = [(4, 512, 512, 64, 64, L.SRC_ACT), (4, 512, 512, 64, 64, L.SRC_PLAIN),
              (4, 256, 256, 128, 128, L.SRC_ACT), (4, 128, 128, 256, 256, L.SRC_PLAIN)]
    if SPLIT:
        layers = [(4, 32, 32, 512, 512, L.SRC_ACT), (4, 32, 32, 512, 512, L.SRC_PLAIN), (4, 64, 64, 512, 256, L.SRC_ACT)]
    for (N, H, W, cin, cout, kind) in layers:
        d, keep = layer(N, H, W, cin, cout, kind)
        fl = 2.0 * N * H * W * cin * cout * 9
        stream = torch.cuda.current_stream().cuda_stream
        times = {m: [] for m in modes}
        for rep in range(12):
            for m in modes:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                rc = FN(ctypes.byref(d), m, stream)
                e.record()
                assert rc == 0, rc
                e.synchronize()
                if rep >= 2:
                    times[m].append(s.elapsed_time(e) * 1e3)
        print(f"layer {N}x{H}x{W} {cin}->{cout} {'act' if kind == L.SRC_ACT else 'plain'}:", flush=True)
        for m in modes:
            us = statistics.median(times[m])
            print(f"   mode {m:2d}: {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
