"""CPU oracle for the Attention-U-Net forward/backward hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package (`unet-segment-pytorch_amd/unet`)
imports this module; only `tests/`, `__graft_entry__.smoke()` and the `cpu_baseline` leg of
`bench.py` may use it, and only as the checker / the timed CPU baseline.

What it is: a functional restatement, in plain PyTorch ATen ops on the CPU in fp32 NCHW, of the
reference's network and loss (seagochen/unet-segment-pytorch).  It works on a flat dict of
parameters/buffers keyed exactly like the reference's `state_dict()` so that a checkpoint (or a
seeded model of either implementation) can be fed to it.  Autograd on these ATen calls gives the
reference's gradients.

Pinning: `tests/golden/make_golden.py` imports the real reference (only in the build container)
and records fixtures; `tests/test_oracle_golden.py` checks this restatement against them.

Every function cites the reference line it restates.
"""

from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

Params = Dict[str, torch.Tensor]

BN_EPS = 1e-5        # nn.BatchNorm2d default (unet/models/layers.py:33,36)
BN_MOMENTUM = 0.1    # nn.BatchNorm2d default


def _bn(p: Params, prefix: str, x: torch.Tensor, training: bool) -> torch.Tensor:
    """nn.BatchNorm2d (affine, track_running_stats) — layers.py:33,36,153,159,165.

    Train mode normalises with the biased batch variance and updates the running buffers in place
    (running_var with the unbiased variance), exactly as nn.BatchNorm2d does.
    """
    if training:
        nbt = p.get(prefix + ".num_batches_tracked")
        if nbt is not None:
            nbt.add_(1)
    return F.batch_norm(x, p[prefix + ".running_mean"], p[prefix + ".running_var"],
                        p[prefix + ".weight"], p[prefix + ".bias"], training, BN_MOMENTUM, BN_EPS)


def double_conv(p: Params, prefix: str, x: torch.Tensor, training: bool) -> torch.Tensor:
    """DoubleConv: (conv3x3 pad1 no-bias -> BN -> ReLU) x 2 — layers.py:16-41."""
    y = F.conv2d(x, p[prefix + ".double_conv.0.weight"], None, 1, 1)
    y = F.relu(_bn(p, prefix + ".double_conv.1", y, training))
    y = F.conv2d(y, p[prefix + ".double_conv.3.weight"], None, 1, 1)
    return F.relu(_bn(p, prefix + ".double_conv.4", y, training))


def down(p: Params, prefix: str, x: torch.Tensor, training: bool) -> torch.Tensor:
    """Down: MaxPool2d(2) -> DoubleConv — layers.py:44-61."""
    return double_conv(p, prefix + ".maxpool_conv.1", F.max_pool2d(x, 2), training)


def _pad_to(x1: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    """Pad the upsampled decoder map to the skip size — layers.py:97-102 / 246-251."""
    dy = x2.size(2) - x1.size(2)
    dx = x2.size(3) - x1.size(3)
    return F.pad(x1, [dx // 2, dx - dx // 2, dy // 2, dy - dy // 2])


def _up(p: Params, prefix: str, x1: torch.Tensor, bilinear: bool) -> torch.Tensor:
    """self.up: bilinear x2 align_corners=True (layers.py:78) or ConvTranspose2d k2 s2 (layers.py:81)."""
    if bilinear:
        return F.interpolate(x1, scale_factor=2, mode="bilinear", align_corners=True)
    return F.conv_transpose2d(x1, p[prefix + ".up.weight"], p[prefix + ".up.bias"], stride=2)


def up(p: Params, prefix: str, x1: torch.Tensor, x2: torch.Tensor, bilinear: bool, training: bool) -> torch.Tensor:
    """Up: up(x1) -> pad -> cat([skip, up]) -> DoubleConv — layers.py:84-106."""
    u = _pad_to(_up(p, prefix, x1, bilinear), x2)
    return double_conv(p, prefix + ".conv", torch.cat([x2, u], dim=1), training)


def out_conv(p: Params, prefix: str, x: torch.Tensor) -> torch.Tensor:
    """OutConv: 1x1 conv with bias — layers.py:109-123."""
    return F.conv2d(x, p[prefix + ".conv.weight"], p[prefix + ".conv.bias"])


def attention_gate(p: Params, prefix: str, g: torch.Tensor, x: torch.Tensor, training: bool) -> torch.Tensor:
    """AttentionGate.forward — layers.py:171-192."""
    g_up = F.interpolate(g, size=x.shape[2:], mode="bilinear", align_corners=True)          # :183
    g1 = _bn(p, prefix + ".W_g.1", F.conv2d(g_up, p[prefix + ".W_g.0.weight"]), training)  # :186
    x1 = _bn(p, prefix + ".W_x.1", F.conv2d(x, p[prefix + ".W_x.0.weight"]), training)     # :187
    a = F.relu(g1 + x1)                                                                    # :188
    s = torch.sigmoid(_bn(p, prefix + ".psi.1", F.conv2d(a, p[prefix + ".psi.0.weight"]), training))  # :189
    return x * s                                                                           # :192


def attention_up(p: Params, prefix: str, x1: torch.Tensor, x2: torch.Tensor, bilinear: bool,
                 training: bool) -> torch.Tensor:
    """AttentionUp.forward — layers.py:229-255 (gate on the pre-upsample decoder map)."""
    x2a = attention_gate(p, prefix + ".attention", x1, x2, training)
    u = _pad_to(_up(p, prefix, x1, bilinear), x2a)
    return double_conv(p, prefix + ".conv", torch.cat([x2a, u], dim=1), training)


def unet_forward(p: Params, x: torch.Tensor, bilinear: bool = True, training: bool = True) -> torch.Tensor:
    """UNet.forward — unet.py:67-92."""
    x1 = double_conv(p, "inc", x, training)
    x2 = down(p, "down1", x1, training)
    x3 = down(p, "down2", x2, training)
    x4 = down(p, "down3", x3, training)
    x5 = down(p, "down4", x4, training)
    y = up(p, "up1", x5, x4, bilinear, training)
    y = up(p, "up2", y, x3, bilinear, training)
    y = up(p, "up3", y, x2, bilinear, training)
    y = up(p, "up4", y, x1, bilinear, training)
    return out_conv(p, "outc", y)


def attention_unet_forward(p: Params, x: torch.Tensor, bilinear: bool = True, training: bool = True,
                           deep_supervision: bool = False):
    """AttentionUNet.forward — unet.py:175-211 (DS heads :204-209, only in training)."""
    size = x.shape[2:]
    x1 = double_conv(p, "inc", x, training)
    x2 = down(p, "down1", x1, training)
    x3 = down(p, "down2", x2, training)
    x4 = down(p, "down3", x3, training)
    x5 = down(p, "down4", x4, training)
    d4 = attention_up(p, "up1", x5, x4, bilinear, training)
    d3 = attention_up(p, "up2", d4, x3, bilinear, training)
    d2 = attention_up(p, "up3", d3, x2, bilinear, training)
    d1 = attention_up(p, "up4", d2, x1, bilinear, training)
    logits = out_conv(p, "outc", d1)
    if deep_supervision and training:
        ds3 = F.interpolate(out_conv(p, "ds_out3", d4), size=size, mode="bilinear", align_corners=True)
        ds2 = F.interpolate(out_conv(p, "ds_out2", d3), size=size, mode="bilinear", align_corners=True)
        ds1 = F.interpolate(out_conv(p, "ds_out1", d2), size=size, mode="bilinear", align_corners=True)
        return [logits, ds1, ds2, ds3]
    return logits


# ----------------------------------------------------------------------------------------------
# losses — unet/utils/loss.py
# ----------------------------------------------------------------------------------------------

def dice_loss(z: torch.Tensor, t: torch.Tensor, smooth: float = 1.0, ignore_background: bool = True,
              reduction: str = "mean") -> torch.Tensor:
    """DiceLoss.forward — loss.py:45-85."""
    c = z.shape[1]
    pr = F.softmax(z, dim=1)
    oh = F.one_hot(t, num_classes=c).permute(0, 3, 1, 2).to(z.dtype)
    inter = (pr * oh).sum(dim=(2, 3))
    union = pr.sum(dim=(2, 3)) + oh.sum(dim=(2, 3))
    d = (2.0 * inter + smooth) / (union + smooth)
    if ignore_background and c > 1:
        d = d[:, 1:]
    if reduction == "mean":
        return 1.0 - d.mean()
    if reduction == "sum":
        return (1.0 - d).sum()
    return 1.0 - d


def balanced_ce_loss(z: torch.Tensor, t: torch.Tensor, class_weight: float = 0.5,
                     smooth: float = 1e-6) -> torch.Tensor:
    """BalancedCELoss.forward — loss.py:110-150 (weights only on labels 0 and 1)."""
    n = z.shape[0]
    ce = F.cross_entropy(z, t, reduction="none")
    w = torch.zeros_like(ce)
    for i in range(n):
        tm = t[i] == 1
        bm = t[i] == 0
        nt = tm.sum().to(z.dtype) + smooth
        nb = bm.sum().to(z.dtype) + smooth
        w[i][tm] = class_weight / nt
        w[i][bm] = (1 - class_weight) / nb
    return (ce * w).sum() / n


def dice_bce_loss(z: torch.Tensor, t: torch.Tensor, ce_weight: float = 1.0, dice_weight: float = 1.0,
                  class_weight: float = 0.5) -> torch.Tensor:
    """DiceBCELoss.forward — loss.py:184-191."""
    return ce_weight * balanced_ce_loss(z, t, class_weight) + dice_weight * dice_loss(z, t)


def deep_supervision_loss(preds, t: torch.Tensor, base, weights: Optional[List[float]] = None):
    """DeepSupervisionLoss.forward — loss.py:216-229."""
    weights = weights or [1.0, 0.4, 0.2, 0.1]
    if isinstance(preds, (list, tuple)):
        total = 0.0
        for pr, w in zip(preds, weights):
            total = total + w * base(pr, t)
        return total
    return base(preds, t)


# ----------------------------------------------------------------------------------------------
# metrics used as parity definitions (after threshold => integer arithmetic)
# ----------------------------------------------------------------------------------------------

def confusion_matrix(pred_labels: torch.Tensor, t: torch.Tensor, num_classes: int = 2) -> torch.Tensor:
    """SegmentationMetrics.update — metrics.py:55-84 (bincount form of the per-pixel loop)."""
    k = t.reshape(-1).long() * num_classes + pred_labels.reshape(-1).long()
    return torch.bincount(k, minlength=num_classes * num_classes).reshape(num_classes, num_classes)


def class_iou_dice(pred_labels: torch.Tensor, t: torch.Tensor, num_classes: int = 2, smooth: float = 1e-6):
    """compute_iou / compute_dice — metrics.py:178-192, 213-227: per class, boolean masks over every pixel
    (targets outside [0, K) included), float32 sums, (I + s) / (U + s) and (2I + s) / (|p| + |t| + s)."""
    iou, dice = [], []
    for c in range(num_classes):
        pc, tc = pred_labels == c, t == c
        inter = (pc & tc).float().sum()
        iou.append((inter + smooth) / ((pc | tc).float().sum() + smooth))
        dice.append((2.0 * (pc.float() * tc.float()).sum() + smooth) / (pc.float().sum() + tc.float().sum() + smooth))
    return torch.stack(iou), torch.stack(dice)


def segmentation_scores(cm: np.ndarray, class_names) -> dict:
    """SegmentationMetrics.compute — metrics.py:86-143: per class c, tp = cm[c, c], fp = column c minus tp,
    fn = row c minus tp; IoU = tp / (tp + fp + fn), Dice = 2 tp / (2 tp + fp + fn) (0 for a zero
    denominator); means over the classes whose score is non-zero; all zeros for an empty matrix."""
    total = cm.sum()
    iou, dice = {}, {}
    for c, name in enumerate(class_names):
        tp = cm[c, c]
        fp = cm[:, c].sum() - tp
        fn = cm[c, :].sum() - tp
        iou[name] = float(tp / (tp + fp + fn)) if total and tp + fp + fn > 0 else 0.0
        dice[name] = float(2 * tp / (2 * tp + fp + fn)) if total and 2 * tp + fp + fn > 0 else 0.0
    vi = [v for v in iou.values() if v > 0]
    vd = [v for v in dice.values() if v > 0]
    return {"pixel_accuracy": float(np.trace(cm) / total) if total else 0.0,
            "mean_iou": float(np.mean(vi)) if vi and total else 0.0,
            "mean_dice": float(np.mean(vd)) if vd and total else 0.0,
            "class_iou": iou, "class_dice": dice}


def tumor_dice(pred_labels: torch.Tensor, t: torch.Tensor) -> float:
    """Tumor Dice of scripts/overfit_test.py:196-205: 2|P∩G|/(|P|+|G|), no smoothing."""
    p1 = pred_labels == 1
    g1 = t == 1
    inter = (p1 & g1).sum().item()
    tot = p1.sum().item() + g1.sum().item()
    return 2.0 * inter / tot if tot > 0 else 0.0


# ----------------------------------------------------------------------------------------------
# helpers
# ----------------------------------------------------------------------------------------------

def params_from_module(m: torch.nn.Module, requires_grad: bool = True) -> Params:
    """Detached fp32 CPU copies of a model's parameters and buffers keyed like its state_dict."""
    out: Params = {}
    for k, v in m.state_dict().items():
        t = v.detach().cpu().clone()
        if t.is_floating_point():
            t = t.float()
            if requires_grad and not (k.endswith("running_mean") or k.endswith("running_var")):
                t.requires_grad_(True)
        out[k] = t
    return out
