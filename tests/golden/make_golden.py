"""Generate the golden fixtures by running the REAL reference (seagochen/unet-segment-pytorch).

Run in the build container only (the reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [/root/reference]

Outputs are plain tensors (torch.save of dicts of tensors, loadable with weights_only=True) under
tests/golden/.  No reference source or pickled reference object is stored.  The reference's own
repository has no tests or fixtures, so these vectors are what pins the oracle.

Status: the committed fixtures were produced by this script early in round 1.  Importing the
reference was refused later in that round, so this script is not to be re-run: it is
kept as the record of how the committed vectors were made.
"""

from __future__ import annotations

import os
import sys
from pathlib import Path

import torch

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = Path(__file__).resolve().parent
sys.dont_write_bytecode = True
sys.path.insert(0, REF)

from unet.models import UNet, AttentionUNet, DoubleConv, Down, Up, OutConv, AttentionGate, AttentionUp  # noqa: E402
from unet.utils.loss import DiceLoss, BalancedCELoss, DiceBCELoss, DeepSupervisionLoss  # noqa: E402
from unet.utils.metrics import SegmentationMetrics  # noqa: E402

torch.set_num_threads(8)
torch.use_deterministic_algorithms(False)


def disc_targets(n: int, h: int, w: int, seed: int) -> torch.Tensor:
    """1-3 discs per image, ~1-5 % foreground (scaled-down version of BASELINE's synthetic masks)."""
    g = torch.Generator().manual_seed(seed)
    t = torch.zeros(n, h, w, dtype=torch.int64)
    yy, xx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    for i in range(n):
        for _ in range(int(torch.randint(1, 4, (1,), generator=g))):
            cy = int(torch.randint(0, h, (1,), generator=g))
            cx = int(torch.randint(0, w, (1,), generator=g))
            r = int(torch.randint(max(2, h // 20), max(3, h // 8), (1,), generator=g))
            t[i][(yy - cy) ** 2 + (xx - cx) ** 2 <= r * r] = 1
    return t


def grads_of(m: torch.nn.Module):
    return {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}


def buffers_of(m: torch.nn.Module):
    return {k: b.detach().clone() for k, b in m.named_buffers()}


def model_case(kind: str, base: int, n: int, c: int, h: int, w: int, bilinear: bool, ds: bool,
               store_params: bool, seed: int = 0):
    torch.manual_seed(seed)
    if kind == "unet":
        m = UNet(n_channels=c, n_classes=2, bilinear=bilinear, base_features=base)
    else:
        m = AttentionUNet(n_channels=c, n_classes=2, bilinear=bilinear, base_features=base, deep_supervision=ds)
    init = {k: v.detach().clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.rand(n, c, h, w, generator=g) * 2 - 1
    t = disc_targets(n, h, w, seed + 2)
    m.train()
    out = m(x)
    crit = DiceBCELoss()
    if ds:
        crit = DeepSupervisionLoss(crit)
    loss = crit(out, t)
    loss.backward()
    rec = {
        "kind": kind, "base": base, "bilinear": bilinear, "deep_supervision": ds,
        "x": x, "t": t, "loss": loss.detach(),
        "outputs": [o.detach() for o in out] if isinstance(out, list) else [out.detach()],
        "grads": grads_of(m), "buffers_after": buffers_of(m),
        "keys": list(init.keys()), "shapes": {k: list(v.shape) for k, v in init.items()},
        "param_sums": {k: float(v.double().sum()) for k, v in init.items() if v.is_floating_point()},
        "num_params": sum(p.numel() for p in m.parameters()),
    }
    if store_params:
        rec["init"] = init
    # eval-mode forward after the train step (running stats updated once)
    m.eval()
    with torch.no_grad():
        rec["eval_logits"] = m(x).detach()
    return rec


def module_cases():
    recs = {}
    torch.manual_seed(10)
    g = torch.Generator().manual_seed(11)

    def run(name, mod, *inputs):
        ins = [i.clone().requires_grad_(True) for i in inputs]
        init = {k: v.detach().clone() for k, v in mod.state_dict().items()}
        mod.train()
        y = mod(*ins)
        gy = torch.randn(y.shape, generator=g)
        (y * gy).sum().backward()
        recs[name] = {"inputs": [i.detach() for i in inputs], "init": init, "out": y.detach(), "gout": gy,
                      "grad_inputs": [i.grad.detach() for i in ins], "grads": grads_of(mod),
                      "buffers_after": buffers_of(mod)}

    run("double_conv", DoubleConv(16, 32), torch.randn(2, 16, 20, 20, generator=g))
    run("double_conv_mid", DoubleConv(24, 8, 12), torch.randn(2, 24, 13, 17, generator=g))
    run("down", Down(16, 32), torch.randn(2, 16, 21, 20, generator=g))
    run("up_bilinear", Up(32, 8, bilinear=True), torch.randn(2, 16, 9, 10, generator=g),
        torch.randn(2, 16, 19, 21, generator=g))
    run("up_transposed", Up(32, 16, bilinear=False), torch.randn(2, 32, 10, 10, generator=g),
        torch.randn(2, 16, 20, 20, generator=g))
    run("out_conv", OutConv(16, 2), torch.randn(2, 16, 12, 12, generator=g))
    run("attention_gate", AttentionGate(16, 16), torch.randn(2, 16, 10, 10, generator=g),
        torch.randn(2, 16, 20, 20, generator=g))
    run("attention_gate_odd", AttentionGate(16, 8, 4), torch.randn(2, 16, 7, 9, generator=g),
        torch.randn(2, 8, 15, 17, generator=g))
    run("attention_up", AttentionUp(32, 8, bilinear=True), torch.randn(2, 16, 10, 10, generator=g),
        torch.randn(2, 16, 20, 20, generator=g))
    run("attention_up_transposed", AttentionUp(32, 16, bilinear=False), torch.randn(2, 32, 8, 8, generator=g),
        torch.randn(2, 16, 16, 16, generator=g))
    return recs


def loss_cases():
    g = torch.Generator().manual_seed(21)
    z = torch.randn(4, 2, 32, 32, generator=g) * 2
    t = disc_targets(4, 32, 32, 22)
    t[1].zero_()        # an image with no tumour
    t[2].fill_(1)       # an image with no background
    recs = {}
    for name, crit in [("dice_bce", DiceBCELoss()), ("dice", DiceLoss()), ("balanced_ce", BalancedCELoss()),
                       ("dice_bce_w", DiceBCELoss(ce_weight=0.7, dice_weight=1.3, class_weight=0.3))]:
        zz = z.clone().requires_grad_(True)
        loss = crit(zz, t)
        loss.backward()
        recs[name] = {"loss": loss.detach(), "grad": zz.grad.detach()}
    # 3-class case (general C path)
    z3 = torch.randn(2, 3, 16, 16, generator=g)
    t3 = torch.randint(0, 3, (2, 16, 16), generator=g)
    zz = z3.clone().requires_grad_(True)
    loss = DiceBCELoss()(zz, t3)
    loss.backward()
    recs["dice_bce_c3"] = {"loss": loss.detach(), "grad": zz.grad.detach(), "z": z3, "t": t3}
    return {"z": z, "t": t, "cases": recs}


def metric_cases():
    g = torch.Generator().manual_seed(31)
    z = torch.randn(2, 2, 24, 24, generator=g)
    t = disc_targets(2, 24, 24, 32)
    m = SegmentationMetrics(num_classes=2, class_names=["background", "tumor"])
    m.update(z, t)
    res = m.compute()
    return {"z": z, "t": t, "confusion": torch.tensor(m.confusion_matrix),
            "mean_dice": res["mean_dice"], "mean_iou": res["mean_iou"]}


def main():
    models = {
        "attention_unet_b8": model_case("attention_unet", 8, 2, 1, 64, 64, True, False, True),
        "unet_b8": model_case("unet", 8, 2, 1, 64, 64, True, False, True),
        "attention_unet_b4_ds": model_case("attention_unet", 4, 2, 1, 64, 64, True, True, False),
        "attention_unet_b4_odd": model_case("attention_unet", 4, 2, 1, 50, 44, True, False, False),
        "unet_b4_transposed": model_case("unet", 4, 2, 1, 48, 48, False, False, False),
        "attention_unet_b4_3ch_transposed": model_case("attention_unet", 4, 2, 3, 32, 32, False, False, False),
    }
    torch.save(models, OUT / "models.pt")
    torch.save(module_cases(), OUT / "modules.pt")
    torch.save(loss_cases(), OUT / "losses.pt")
    torch.save(metric_cases(), OUT / "metrics.pt")
    torch.manual_seed(0)
    full = AttentionUNet(1, 2)
    seeded = {"first_conv_sum": float(full.inc.double_conv[0].weight.detach().sum()),
              "num_params": sum(p.numel() for p in full.parameters()),
              "num_params_unet": sum(p.numel() for p in UNet(1, 2).parameters()),
              "keys_attention_unet": list(full.state_dict().keys())}
    torch.save(seeded, OUT / "seeded.pt")
    for f in sorted(OUT.glob("*.pt")):
        print(f.name, f.stat().st_size)


if __name__ == "__main__":
    main()
