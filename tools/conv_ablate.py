"""Ablation timing of the conv3 (4,2,4) kernel on full-size layers (diagnostic, GPU).
Modes: 0 full; 1 weights from one L1-resident fragment; 2 no next-chunk halo staging; 3 = 1+2;
4 one barrier per block; 8 no epilogue stores; 11 = 1+2+8; 15 = everything off but the MFMA/LDS loop."""
import ctypes
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "unet-segment-pytorch_amd"))
import torch  # noqa: E402

from unet._hip import lib as L  # noqa: E402
from unet._hip.runtime import pack_weight, BF16, f32  # noqa: E402

lib = L.load()
lib.unet_diag_conv3_ablate.argtypes = [ctypes.POINTER(L.ConvDesc), ctypes.c_int, ctypes.c_void_p]


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
    rows = lib.unet_conv_stats_rows(d)
    st = f32(2, rows, cout, device=dev)
    d.stats = st.data_ptr()
    return d, (x, w, wp, ab, y, st)


def main():
    modes = [int(m) for m in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3,8,15,100,101,102,103,108,115").split(",")]
    for (N, H, W, cin, cout) in [(4, 256, 256, 128, 128), (4, 64, 64, 512, 512), (4, 128, 128, 256, 256)]:
        d, keep = layer(N, H, W, cin, cout, L.SRC_ACT)
        fl = 2.0 * N * H * W * cin * cout * 9
        stream = torch.cuda.current_stream().cuda_stream
        times = {m: [] for m in modes}
        for rep in range(12):
            for m in modes:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                rc = lib.unet_diag_conv3_ablate(ctypes.byref(d), m, stream)
                e.record()
                assert rc == 0, rc
                e.synchronize()
                if rep >= 2:
                    times[m].append(s.elapsed_time(e) * 1e3)
        print(f"layer {N}x{H}x{W} {cin}->{cout}:")
        for m in modes:
            us = statistics.median(times[m])
            print(f"   mode {m:2d}: {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s")


if __name__ == "__main__":
    main()
