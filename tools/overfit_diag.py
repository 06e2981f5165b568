"""Overfit-loop numerics diagnostic (not a test): scripts/overfit_test.py:126-205 as the reference runs
it for BASELINE C1 — AttentionUNet(1, 2, deep_supervision=True), base 64, 2 x 1 x 512^2, Adam(lr=1e-3),
DeepSupervisionLoss(DiceBCELoss, [1, .4, .2, .1]), one step per epoch on the fixed batch, then an
eval-mode forward and Tumor Dice 2|P n G| / (|P| + |G|).  Runs the HIP path (fp32 operand mode) and the
oracle's ATen restatement in fp32 and fp64 on the GPU from the same initial weights, and prints the
per-epoch loss / Tumor-Dice trajectories and their spreads.

Usage: python tools/overfit_diag.py [epochs] [base] [size]"""

import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "unet-segment-pytorch_amd"))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT))

from oracle import unet_oracle as O  # noqa: E402


def batch(n, h, w, seed=5):
    g = torch.Generator().manual_seed(seed)
    t = torch.zeros(n, h, w, dtype=torch.int64)
    yy, xx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    for i in range(n):
        for _ in range(2):
            cy, cx = int(torch.randint(h // 5, h - h // 5, (1,), generator=g)), \
                int(torch.randint(w // 5, w - w // 5, (1,), generator=g))
            r = int(torch.randint(10, 20, (1,), generator=g))
            t[i][(yy - cy) ** 2 + (xx - cx) ** 2 <= r * r] = 1
    x = (torch.rand(n, 1, h, w, generator=g) * 2 - 1) * 0.5 + 0.8 * t[:, None].float()
    return x, t


def run_oracle(init, names, x, t, epochs, dtype):
    p = {}
    for k, v in init.items():
        v = v.detach().clone().cuda()
        if v.is_floating_point():
            v = v.to(dtype)
            if k in names:
                v.requires_grad_(True)
        p[k] = v
    xx, tt = x.cuda().to(dtype), t.cuda()
    opt = torch.optim.Adam([p[k] for k in names], lr=1e-3)
    hist = []
    for _ in range(epochs):
        opt.zero_grad()
        out = O.attention_unet_forward(p, xx, training=True, deep_supervision=True)
        loss = O.deep_supervision_loss(out, tt, O.dice_bce_loss)
        loss.backward()
        opt.step()
        with torch.no_grad():
            d = O.tumor_dice(O.attention_unet_forward(p, xx, training=False).argmax(1).cpu(), t)
        hist.append((float(loss.detach()), d))
    return hist


def run_hip(init, x, t, epochs, base, prec="fp32"):
    from unet.models import AttentionUNet
    from unet.utils.loss import DeepSupervisionLoss, DiceBCELoss
    m = AttentionUNet(1, 2, deep_supervision=True, base_features=base)
    m.load_state_dict(init)
    m = m.cuda().train()
    m.hip_precision = prec
    xx, tt = x.cuda(), t.cuda()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    crit = DeepSupervisionLoss(DiceBCELoss(), weights=[1.0, 0.4, 0.2, 0.1])
    hist = []
    for _ in range(epochs):
        opt.zero_grad()
        loss = crit(m(xx), tt)
        loss.backward()
        opt.step()
        m.eval()
        with torch.no_grad():
            d = O.tumor_dice(m(xx).argmax(1).cpu(), t)
        m.train()
        hist.append((float(loss.detach()), d))
    return hist


def main():
    epochs = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    base = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    size = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    torch.backends.cudnn.deterministic = True
    from unet.models import AttentionUNet
    torch.manual_seed(0)
    m = AttentionUNet(1, 2, deep_supervision=True, base_features=base)
    init = {k: v.clone() for k, v in m.state_dict().items()}
    names = [k for k, _ in m.named_parameters()]
    x, t = batch(2, size, size)
    print(f"tumour pixels per image: {[int(v) for v in t.sum((1, 2))]}", flush=True)
    res = {}
    for name, fn in [("hip32", lambda: run_hip(init, x, t, epochs, base)),
                     ("ora32", lambda: run_oracle(init, names, x, t, epochs, torch.float32)),
                     ("ora64", lambda: run_oracle(init, names, x, t, epochs, torch.float64))]:
        t0 = time.time()
        res[name] = fn()
        print(f"{name}: {time.time() - t0:.1f} s", flush=True)
    print("epoch  loss_hip32 loss_ora32 loss_ora64 | dice_hip32 dice_ora32 dice_ora64")
    for i in range(epochs):
        a, b, c = res["hip32"][i], res["ora32"][i], res["ora64"][i]
        print(f"{i:3d} {a[0]:.6f} {b[0]:.6f} {c[0]:.6f} | {a[1]:.6f} {b[1]:.6f} {c[1]:.6f}", flush=True)


if __name__ == "__main__":
    main()
