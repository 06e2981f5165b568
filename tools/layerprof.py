"""Per-launch timing of one full training step (every C-ABI call bracketed by HIP events).

usage: python tools/layerprof.py [--model attention_unet|unet] [--batch 4] [--size 512] [--prec bf16]
Prints one line per conv fwd / dgrad / wgrad launch (geometry, source kinds, variant, us, TFLOP/s), one
per HBM-bound launch of the bench line's hbm block (algorithmic bytes, GB/s) and a per-entry-point summary.  Diagnostic only (not part of the product or the tests)."""
import argparse
import collections
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "unet-segment-pytorch_amd"))

import torch  # noqa: E402

from unet._hip import lib as L  # noqa: E402
from unet._hip.runtime import conv_kernel_name, wgrad_kernel_name  # noqa: E402

sys.path.insert(0, str(ROOT))
from bench import _hbm_bytes  # noqa: E402  (the algorithmic bytes of the bench line's hbm block)

KIND = {0: "plain", 1: "act", 2: "pool", 3: "up", 4: "nchw", 5: "upplain"}
OUT = {0: "y", 1: "f32", 2: "poolbwd", 3: "shuf2", 4: "f32gate"}

_orig = L.call
_rec = []
_on = [False]


def _desc_info(name, d):
    srcs = "+".join(f"{KIND[d.src[i].kind]}{d.src[i].C}" for i in range(d.nsrc))
    fl = 2.0 * d.N * d.H * d.W * d.Cin * d.Cout * d.ksize ** 2
    if name == "unet_conv":
        tag = f"conv {OUT[d.out_mode]:7s}"
        var = conv_kernel_name(d)
    else:
        tag = "wgrad       "
        var = wgrad_kernel_name(d)
    return f"{tag} {d.N}x{d.H}x{d.W} {d.Cin:4d}->{d.Cout:4d} k{d.ksize} [{srcs}] {var}", fl


def _call(name, *args):
    if not _on[0]:
        return _orig(name, *args)
    info, fl = (_desc_info(name, args[0]) if name in ("unet_conv", "unet_conv_wgrad") else (name, 0.0))
    hb = _hbm_bytes(name, args)
    if hb is not None and name not in ("unet_conv", "unet_conv_wgrad"):
        info = f"{name} {hb[1] / 1e6:.1f} MB"
        fl = -hb[1]          # negative: algorithmic bytes (HBM-bound line)
    elif hb is not None:
        info += f" | {hb[1] / 1e6:.1f} MB"
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    r = _orig(name, *args)
    e.record()
    _rec.append((name, info, fl, s, e))
    return r


L.call = _call


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="attention_unet")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--prec", default="bf16")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from unet.models import AttentionUNet, UNet
    from unet.utils.loss import DiceBCELoss
    torch.manual_seed(0)
    m = (AttentionUNet(1, 2) if a.model == "attention_unet" else UNet(1, 2)).cuda().train()
    m.hip_precision = a.prec
    x = torch.rand(a.batch, 1, a.size, a.size, device="cuda") * 2 - 1
    t = (torch.rand(a.batch, a.size, a.size, device="cuda") < 0.004).long()
    crit = DiceBCELoss()
    for _ in range(3):
        crit(m(x), t).backward()
    torch.cuda.synchronize()
    per = collections.defaultdict(list)
    order = []
    for rep in range(a.reps):
        _rec.clear()
        _on[0] = True
        crit(m(x), t).backward()
        _on[0] = False
        torch.cuda.synchronize()
        for i, (name, info, fl, s, e) in enumerate(_rec):
            key = (i, info)
            if rep == 0:
                order.append((key, name, fl))
            per[key].append(s.elapsed_time(e) * 1e3)
    tot = collections.defaultdict(float)
    for key, name, fl in order:
        us = min(per[key])
        tot[name] += us
        if fl > 0:
            print(f"{us:9.1f} us {fl / us / 1e6:8.1f} TF/s  {key[1]}")
        elif fl < 0:
            print(f"{us:9.1f} us {-fl / us / 1e3:8.1f} GB/s   {key[1]}")
    print("---- per entry point (us/step, min over reps) ----")
    for n, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"{v:10.1f}  {n}")
    print(f"{sum(tot.values()):10.1f}  total (sum of bracketed launches)")


if __name__ == "__main__":
    main()
