"""Overfit-loop numerics diagnostic (not a test): scripts/overfit_test.py:126-205 as the reference runs
it for BASELINE C1 — AttentionUNet(1, 2, deep_supervision=True), base 64, 2 x 1 x 512^2, Adam(lr=1e-3),
DeepSupervisionLoss(DiceBCELoss, [1, .4, .2, .1]), one step per epoch on the fixed batch, then an
eval-mode forward and Tumor Dice 2|P n G| / (|P| + |G|) on argmax(softmax(logits)) (:182-205).

Executions: the HIP path (fp32 operand mode) and the oracle's ATen restatement in fp32 and fp64 on the
GPU, all from the same initial weights.

Usage: python tools/overfit_diag.py MODE [args]
  traj [epochs] [base] [size]   per-epoch loss / Tumor-Dice of the three executions
  lockstep [epochs]             the three executions step by step, with the parameter and BN running-buffer
                                distances HIP-vs-fp64 and fp32-vs-fp64 at every epoch (where the trajectories part)
  ensemble K [epochs] [K64]     K executions each of HIP and reference fp32 (and K64 of fp64) from initial
                                weights perturbed by one ulp in a random half of their elements (the member-0 run
                                unperturbed): the distribution of the last-epoch Tumor-Dice under rounding noise
  pin [epochs...]               the HIP eval forward / train step from the oracle's own states at those epochs:
                                confusion counts vs the oracle's (near ties counted) and gradients vs fp64"""

import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "unet-segment-pytorch_amd"))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT))

from oracle import unet_oracle as O  # noqa: E402

DS_W = [1.0, 0.4, 0.2, 0.1]     # overfit_test.py:148


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


def setup(base=64, size=512):
    """The seeded C1 model state, its parameter names and the synthetic batch."""
    from unet.models import AttentionUNet
    torch.backends.cudnn.deterministic = True
    torch.manual_seed(0)
    m = AttentionUNet(1, 2, deep_supervision=True, base_features=base)
    init = {k: v.clone() for k, v in m.state_dict().items()}
    names = [k for k, _ in m.named_parameters()]
    x, t = batch(2, size, size)
    return init, names, x, t


def perturb(init, names, seed):
    """One-ulp perturbation (towards +-inf at random) of a random half of every parameter's elements: the
    size of the rounding difference another, equally correct, fp32 execution of the first step makes."""
    if seed == 0:
        return init
    g = torch.Generator().manual_seed(seed)
    out = dict(init)
    for k in names:
        v = init[k].float()
        sel = torch.rand(v.shape, generator=g) < 0.5
        up = torch.rand(v.shape, generator=g) < 0.5
        tgt = torch.where(up, torch.full_like(v, float("inf")), torch.full_like(v, float("-inf")))
        out[k] = torch.where(sel, torch.nextafter(v, tgt), v)
    return out


def tumor_dice_of_logits(z, t):
    """overfit_test.py:194-205: argmax of the softmax, then 2|P n G| / (|P| + |G|)."""
    return O.tumor_dice(torch.softmax(z.float(), 1).argmax(1).cpu(), t.cpu())


class Oracle:
    """The reference network as the oracle's ATen ops on the GPU in `dtype`, trained as overfit_test.py does."""

    def __init__(self, init, names, x, t, dtype):
        self.names, self.dtype = names, dtype
        self.p = {}
        for k, v in init.items():
            v = v.detach().clone().cuda()
            if v.is_floating_point():
                v = v.to(dtype)
                if k in names:
                    v.requires_grad_(True)
            self.p[k] = v
        self.x, self.t = x.cuda().to(dtype), t.cuda()
        self.opt = torch.optim.Adam([self.p[k] for k in names], lr=1e-3)

    def loss(self):
        out = O.attention_unet_forward(self.p, self.x, training=True, deep_supervision=True)
        return O.deep_supervision_loss(out, self.t, O.dice_bce_loss, DS_W)

    def step(self):
        self.opt.zero_grad()
        loss = self.loss()
        loss.backward()
        self.opt.step()
        return float(loss.detach())

    def eval_logits(self):
        with torch.no_grad():
            return O.attention_unet_forward(self.p, self.x, training=False)

    def epoch(self):
        loss = self.step()
        return loss, tumor_dice_of_logits(self.eval_logits(), self.t)

    def state(self):
        return {k: v.detach().double() for k, v in self.p.items() if v.is_floating_point()}


class Hip:
    """The HIP path (fp32 operand mode) trained the same way."""

    def __init__(self, init, x, t, base=64, prec="fp32"):
        from unet.models import AttentionUNet
        from unet.utils.loss import DeepSupervisionLoss, DiceBCELoss
        m = AttentionUNet(1, 2, deep_supervision=True, base_features=base)
        m.load_state_dict(init)
        self.m = m.cuda().train()
        self.m.hip_precision = prec
        self.x, self.t = x.cuda(), t.cuda()
        self.opt = torch.optim.Adam(self.m.parameters(), lr=1e-3)
        self.crit = DeepSupervisionLoss(DiceBCELoss(), weights=DS_W)

    def step(self):
        self.opt.zero_grad()
        loss = self.crit(self.m(self.x), self.t)
        loss.backward()
        self.opt.step()
        return float(loss.detach())

    def eval_logits(self):
        self.m.eval()
        with torch.no_grad():
            z = self.m(self.x)
        self.m.train()
        return z

    def epoch(self):
        loss = self.step()
        return loss, tumor_dice_of_logits(self.eval_logits(), self.t)

    def state(self):
        return {k: v.detach().double() for k, v in self.m.state_dict().items() if v.is_floating_point()}


def _progress(what, e, epochs):
    """a line every 25 epochs on the process's real stderr (past pytest's capture): long runs (the 200-epoch
    protocol is minutes per execution) keep writing, so a runner that watches for silence does not take
    them for hung"""
    if e % 25 == 0 or e == epochs:
        print(f"[overfit] {what}: epoch {e}/{epochs}", file=sys.__stderr__, flush=True)


def run_oracle(init, names, x, t, epochs, dtype, snap=()):
    """Per-epoch (loss, Tumor-Dice); with `snap`, also the oracle's full state (parameters + BN buffers, as
    fp32 CPU tensors keyed like the state_dict) after each of those epochs (1-based)."""
    o = Oracle(init, names, x, t, dtype)
    hist, snaps = [], {}
    for e in range(1, epochs + 1):
        hist.append(o.epoch())
        _progress(f"oracle {str(dtype).replace('torch.', '')}", e, epochs)
        if e in snap:
            snaps[e] = {k: (v.detach().float().cpu().clone() if v.is_floating_point() else v.cpu().clone())
                        for k, v in o.p.items()}
    return (hist, snaps) if snap else hist


def run_hip(init, x, t, epochs, base, prec="fp32"):
    h = Hip(init, x, t, base, prec)
    hist = []
    for e in range(1, epochs + 1):
        hist.append(h.epoch())
        _progress(f"HIP {prec}", e, epochs)
    return hist


def _dist(a, b, keys):
    num = sum(float((a[k] - b[k]).pow(2).sum()) for k in keys)
    den = sum(float(b[k].pow(2).sum()) for k in keys)
    return (num / max(den, 1e-300)) ** 0.5


def lockstep(init, names, x, t, epochs):
    """Where the trajectories part: per epoch, rel-L2 distances of all parameters and of all BN running
    buffers, HIP-vs-fp64 and fp32-vs-fp64, beside the three losses and Tumor-Dice values."""
    h, r32, r64 = Hip(init, x, t), Oracle(init, names, x, t, torch.float32), Oracle(init, names, x, t, torch.float64)
    bufs = [k for k in init if k.endswith("running_mean") or k.endswith("running_var")]
    rows = []
    print("epoch | loss hip r32 r64 | dice hip r32 r64 | params d(hip,64) d(32,64) | bn-buffers d(hip,64) d(32,64)",
          flush=True)
    for e in range(1, epochs + 1):
        a, b, c = h.epoch(), r32.epoch(), r64.epoch()
        sh, s32, s64 = h.state(), r32.state(), r64.state()
        row = (e, a[0], b[0], c[0], a[1], b[1], c[1], _dist(sh, s64, names), _dist(s32, s64, names),
               _dist(sh, s64, bufs), _dist(s32, s64, bufs))
        rows.append(row)
        print("%3d | %.6f %.6f %.6f | %.6f %.6f %.6f | %.3e %.3e | %.3e %.3e" % row, flush=True)
    return rows


def eval_pin(state, x, t, base=64):
    """The HIP fp32 eval forward of the oracle's own state vs the oracle's eval forward: (Tumor-Dice HIP,
    Tumor-Dice oracle, pixels whose label differs, of those the near ties |z1 - z0| < 1e-4, max |dz|)."""
    from unet.models import AttentionUNet
    m = AttentionUNet(1, 2, deep_supervision=True, base_features=base)
    m.load_state_dict(state)
    m = m.cuda().eval()
    m.hip_precision = "fp32"
    with torch.no_grad():
        zh = m(x.cuda()).float()
        p = {k: v.cuda() for k, v in state.items()}
        zo = O.attention_unet_forward(p, x.cuda(), training=False).float()
    lh = torch.softmax(zh, 1).argmax(1)
    lo = torch.softmax(zo, 1).argmax(1)
    diff = lh != lo
    tie = (zo[:, 1] - zo[:, 0]).abs() < 1e-4
    return (tumor_dice_of_logits(zh, t), tumor_dice_of_logits(zo, t), int(diff.sum()), int((diff & tie).sum()),
            float((zh - zo).abs().max()))


def step_pin(state, names, x, t, base=64):
    """One training forward + deep-supervision loss + backward from the oracle's state (train-mode BN) through
    HIP fp32, the oracle fp32 and the oracle fp64: (loss HIP, loss fp32, loss fp64, all-parameter gradient
    rel-L2 HIP-vs-fp64, fp32-vs-fp64, running-buffer rel-L2 after the step HIP-vs-fp64, fp32-vs-fp64)."""
    from unet.models import AttentionUNet
    from unet.utils.loss import DeepSupervisionLoss, DiceBCELoss
    m = AttentionUNet(1, 2, deep_supervision=True, base_features=base)
    m.load_state_dict(state)
    m = m.cuda().train()
    m.hip_precision = "fp32"
    lh = DeepSupervisionLoss(DiceBCELoss(), weights=DS_W)(m(x.cuda()), t.cuda())
    lh.backward()
    gh = {k: p.grad.double() for k, p in m.named_parameters()}
    bh = {k: v.double() for k, v in m.state_dict().items() if "running" in k}
    res = {}
    for dt in (torch.float32, torch.float64):
        o = Oracle(state, names, x, t, dt)
        loss = o.loss()
        loss.backward()
        res[dt] = (float(loss.detach()), {k: o.p[k].grad.double() for k in names},
                   {k: o.p[k].double() for k in bh})
    (l32, g32, b32), (l64, g64, b64) = res[torch.float32], res[torch.float64]
    bk = list(bh)
    return (float(lh.detach()), l32, l64, _dist(gh, g64, names), _dist(g32, g64, names),
            _dist(bh, b64, bk), _dist(b32, b64, bk))


def ensemble(init, names, x, t, k, epochs, k64):
    """Last-epoch Tumor-Dice (the reference's statistic, overfit_test.py:218,288) and the mean of the last 10
    epochs for k perturbed executions of HIP and of the reference in fp32 and k64 in fp64."""
    out = {"hip": [], "ref32": [], "ref64": []}
    for s in range(k):
        ini = perturb(init, names, s)
        for name, fn, n in [("hip", lambda: run_hip(ini, x, t, epochs, 64), k),
                            ("ref32", lambda: run_oracle(ini, names, x, t, epochs, torch.float32), k),
                            ("ref64", lambda: run_oracle(ini, names, x, t, epochs, torch.float64), k64)]:
            if s >= n:
                continue
            t0 = time.time()
            hist = fn()
            last, mean10 = hist[-1][1], sum(h[1] for h in hist[-10:]) / 10
            out[name].append((last, mean10))
            print(f"member {s} {name}: last-epoch dice {last:.6f}, mean of last 10 {mean10:.6f} "
                  f"({time.time() - t0:.1f} s)", flush=True)
    print("summary (last-epoch dice: mean +- std, min..max | mean of last 10 epochs: mean +- std)")
    for name, v in out.items():
        if not v:
            continue
        ls = torch.tensor([a for a, _ in v], dtype=torch.float64)
        ms = torch.tensor([b for _, b in v], dtype=torch.float64)
        sd = lambda z: float(z.std()) if len(z) > 1 else 0.0   # noqa: E731
        print(f"  {name:5s} n={len(v)}: {float(ls.mean()):.6f} +- {sd(ls):.6f}, {float(ls.min()):.6f}..{float(ls.max()):.6f}"
              f" | {float(ms.mean()):.6f} +- {sd(ms):.6f}", flush=True)
    return out


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "traj"
    args = [int(a) for a in sys.argv[2:]]
    if mode == "traj":
        epochs, base, size = (args + [40, 64, 512][len(args):])[:3]
        init, names, x, t = setup(base, size)
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
    elif mode == "lockstep":
        init, names, x, t = setup()
        lockstep(init, names, x, t, args[0] if args else 200)
    elif mode == "ensemble":
        init, names, x, t = setup()
        k = args[0] if args else 4
        ensemble(init, names, x, t, k, args[1] if len(args) > 1 else 200, args[2] if len(args) > 2 else 0)
    elif mode == "pin":
        init, names, x, t = setup()
        eps = args or [16, 100, 200]
        hist, snaps = run_oracle(init, names, x, t, max(eps), torch.float32, snap=set(eps))
        for e in eps:
            s = snaps[e]
            dh, do, nd, nt, dz = eval_pin(s, x, t)
            print(f"epoch {e}: oracle trajectory dice {hist[e - 1][1]:.6f}; eval forward of its state: HIP dice {dh:.6f}, "
                  f"oracle {do:.6f}, labels differing {nd} (near ties {nt}), max|dlogit| {dz:.2e}", flush=True)
            r = step_pin(s, names, x, t)
            print(f"  train step from it: loss HIP {r[0]:.7f} fp32 {r[1]:.7f} fp64 {r[2]:.7f}; grad rel-L2 vs fp64: "
                  f"HIP {r[3]:.3e}, oracle fp32 {r[4]:.3e}; running buffers vs fp64: HIP {r[5]:.3e}, fp32 {r[6]:.3e}",
                  flush=True)
    else:
        raise SystemExit(__doc__)


if __name__ == "__main__":
    main()
