"""Segmentation losses with the reference's API (unet/utils/loss.py of seagochen/unet-segment-pytorch).

DiceLoss, BalancedCELoss and DiceBCELoss run as one fused HIP reduction + gradient pass
(`unet_loss_*` in include/unet_hip.h): the reference's per-image Python loop with boolean-mask
indexing (loss.py:134-145) becomes device-side per-image reductions, with no host sync.
"""

from typing import Optional

import torch
import torch.nn as nn
from torch.autograd.function import once_differentiable

from .._hip import lib as L
from .._hip.runtime import f32, require_device, stream, vp

_RED = {"mean": 0, "sum": 1, "none": 2}


class _FusedLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, t, ce_w, dice_w, class_w, ce_smooth, dice_smooth, ignore_bg, reduction):
        N, K, H, W = z.shape
        zc = z.detach()
        if zc.dtype != torch.float32 or not zc.is_contiguous():
            zc = zc.float().contiguous()
        tc = t if (t.dtype == torch.int64 and t.is_contiguous()) else t.long().contiguous()
        HW = H * W
        rows = L.load().unet_loss_rows(HW)
        part = f32(N, rows, 4 + 3 * K, device=z.device)
        L.call("unet_loss_reduce", N, K, HW, vp(zc), vp(tc), vp(part), stream())
        coef = f32(N, 2 + 2 * K, device=z.device)
        nd = K - (1 if (ignore_bg and K > 1) else 0)
        loss = f32(N, nd, device=z.device) if reduction == 2 else f32((), device=z.device)
        L.call("unet_loss_finalize", vp(part), rows, N, K, ce_w, dice_w, class_w, ce_smooth, dice_smooth,
               int(ignore_bg), reduction, vp(loss), vp(coef), stream())
        ctx.save_for_backward(zc, tc, coef)
        ctx.cfg = (reduction, int(ignore_bg))
        return loss

    @staticmethod
    @once_differentiable
    def backward(ctx, gout):
        zc, tc, coef = ctx.saved_tensors
        reduction, ignore_bg = ctx.cfg
        N, K, H, W = zc.shape
        go = gout.float().contiguous()
        dz = torch.empty_like(zc)
        L.call("unet_loss_grad", N, K, H * W, vp(zc), vp(tc), vp(coef), vp(go), int(reduction == 2), ignore_bg,
               vp(dz), stream())
        return dz, None, None, None, None, None, None, None, None


class _FusedMultiLoss(torch.autograd.Function):
    """Σ_s w_s · base(z_s, t) over S same-shape logit sets in one reduce / finalize / grad launch each."""

    @staticmethod
    def forward(ctx, t, weights, cfg, *zs):
        ce_w, dice_w, class_w, ce_smooth, dice_smooth, ignore_bg = cfg
        S = len(zs)
        N, K, H, W = zs[0].shape
        zc = [z.detach() if (z.dtype == torch.float32 and z.is_contiguous()) else z.detach().float().contiguous()
              for z in zs]
        tc = t if (t.dtype == torch.int64 and t.is_contiguous()) else t.long().contiguous()
        HW = H * W
        rows = L.load().unet_loss_rows(HW)
        dev = zs[0].device
        part = f32(S, N, rows, 4 + 3 * K, device=dev)
        zp = (L.c_vp * S)(*[z.data_ptr() for z in zc])
        L.call("unet_loss_reduce_multi", S, N, K, HW, zp, vp(tc), vp(part), stream())
        coef = f32(S, N, 2 + 2 * K, device=dev)
        loss = f32((), device=dev)
        wts = (L.c_float * S)(*weights)
        L.call("unet_loss_finalize_multi", vp(part), rows, S, wts, N, K, ce_w, dice_w, class_w, ce_smooth, dice_smooth,
               int(ignore_bg), 0, vp(loss), vp(coef), stream())
        ctx.save_for_backward(tc, coef, *zc)
        ctx.ignore_bg = int(ignore_bg)
        return loss

    @staticmethod
    @once_differentiable
    def backward(ctx, gout):
        tc, coef, *zc = ctx.saved_tensors
        S = len(zc)
        N, K, H, W = zc[0].shape
        go = gout.float().contiguous()
        dz = [torch.empty_like(z) for z in zc]
        zp = (L.c_vp * S)(*[z.data_ptr() for z in zc])
        dp = (L.c_vp * S)(*[d.data_ptr() for d in dz])
        L.call("unet_loss_grad_multi", S, N, K, H * W, zp, vp(tc), vp(coef), vp(go), 0, ctx.ignore_bg, dp, stream())
        return (None, None, None, *dz)


def _fused(z, t, ce_w, dice_w, class_w, ce_smooth=1e-6, dice_smooth=1.0, ignore_bg=True, reduction="mean"):
    require_device(z, "predictions")
    if z.dim() != 4 or t.shape != (z.shape[0], z.shape[2], z.shape[3]):
        raise RuntimeError(f"expected predictions (N, C, H, W) and targets (N, H, W); got {tuple(z.shape)} and "
                           f"{tuple(t.shape)}")
    return _FusedLoss.apply(z, t, float(ce_w), float(dice_w), float(class_w), float(ce_smooth), float(dice_smooth),
                            bool(ignore_bg), _RED[reduction])


class DiceLoss(nn.Module):
    """1 - (2|P∩G| + s)/(|P| + |G| + s) on softmax probabilities — reference loss.py:18-85."""

    def __init__(self, smooth: float = 1.0, reduction: str = "mean", ignore_background: bool = True):
        super().__init__()
        self.smooth = smooth
        self.reduction = reduction
        self.ignore_background = ignore_background

    def forward(self, predictions: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        return _fused(predictions, targets, 0.0, 1.0, 0.5, 1e-6, self.smooth, self.ignore_background, self.reduction)


class BalancedCELoss(nn.Module):
    """Per-image balanced cross entropy (tumour pixels share `class_weight`, background the rest) —
    reference loss.py:88-150."""

    def __init__(self, class_weight: float = 0.5, smooth: float = 1e-6):
        super().__init__()
        self.class_weight = class_weight
        self.smooth = smooth

    def forward(self, predictions: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        return _fused(predictions, targets, 1.0, 0.0, self.class_weight, self.smooth, 1.0, True, "mean")


class DiceBCELoss(nn.Module):
    """ce_weight * BalancedCE + dice_weight * Dice — reference loss.py:153-191 (one fused pass)."""

    def __init__(self, ce_weight: float = 1.0, dice_weight: float = 1.0, class_weight: float = 0.5):
        super().__init__()
        self.ce_weight = ce_weight
        self.dice_weight = dice_weight
        self.balanced_ce = BalancedCELoss(class_weight=class_weight)
        self.dice_loss = DiceLoss(ignore_background=True)

    def forward(self, predictions: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        return _fused(predictions, targets, self.ce_weight, self.dice_weight, self.balanced_ce.class_weight,
                      self.balanced_ce.smooth, self.dice_loss.smooth, self.dice_loss.ignore_background, "mean")


class DeepSupervisionLoss(nn.Module):
    """Σ_k w_k · base(pred_k, targets) over [main, ds1, ds2, ds3] — reference loss.py:194-229.
    With one of the fused bases (DiceBCE / Dice(mean) / BalancedCE) all the sets run through one launch of
    each loss pass; any other base criterion is applied per set as in the reference."""

    def __init__(self, base_criterion: nn.Module, weights: list = None):
        super().__init__()
        self.base_criterion = base_criterion
        self.weights = weights or [1.0, 0.4, 0.2, 0.1]

    def forward(self, predictions, targets: torch.Tensor) -> torch.Tensor:
        if isinstance(predictions, (list, tuple)):
            cfg = _fused_cfg(self.base_criterion)
            n = min(len(predictions), len(self.weights))
            if (cfg is not None and 1 <= n <= 4 and all(p.dim() == 4 and p.shape == predictions[0].shape
                                                        for p in predictions[:n])):
                # the four logit sets through one reduce / finalize / grad launch (unet_loss_*_multi)
                require_device(predictions[0], "predictions")
                if targets.shape != (predictions[0].shape[0], predictions[0].shape[2], predictions[0].shape[3]):
                    raise RuntimeError(f"expected targets (N, H, W), got {tuple(targets.shape)}")
                return _FusedMultiLoss.apply(targets, [float(w) for w in self.weights[:n]], cfg,
                                             *predictions[:n])
            total = 0.0
            for pred, w in zip(predictions, self.weights):
                total = total + w * self.base_criterion(pred, targets)
            return total
        return self.base_criterion(predictions, targets)


def _fused_cfg(crit: nn.Module):
    """(ce_w, dice_w, class_w, ce_smooth, dice_smooth, ignore_bg) of a mean-reduced fused loss, else None."""
    if type(crit) is DiceBCELoss:
        return (float(crit.ce_weight), float(crit.dice_weight), float(crit.balanced_ce.class_weight),
                float(crit.balanced_ce.smooth), float(crit.dice_loss.smooth), bool(crit.dice_loss.ignore_background))
    if type(crit) is DiceLoss and crit.reduction == "mean":
        return (0.0, 1.0, 0.5, 1e-6, float(crit.smooth), bool(crit.ignore_background))
    if type(crit) is BalancedCELoss:
        return (1.0, 0.0, float(crit.class_weight), float(crit.smooth), 1.0, True)
    return None


def create_loss_function(loss_type: str = "dice_bce", ce_weight: float = 1.0, dice_weight: float = 1.0,
                         class_weights: Optional[list] = None, balanced_class_weight: float = 0.5,
                         **kwargs) -> nn.Module:
    """Factory — reference loss.py:232-271 ('dice' | 'ce'/'crossentropy' | 'balanced_ce' | 'dice_bce')."""
    kind = loss_type.lower()
    if kind == "dice":
        return DiceLoss(ignore_background=True)
    if kind in ("ce", "crossentropy"):
        if class_weights is not None:
            return nn.CrossEntropyLoss(weight=torch.tensor(class_weights, dtype=torch.float32))
        return nn.CrossEntropyLoss()
    if kind == "balanced_ce":
        return BalancedCELoss(class_weight=balanced_class_weight)
    if kind == "dice_bce":
        return DiceBCELoss(ce_weight=ce_weight, dice_weight=dice_weight, class_weight=balanced_class_weight)
    raise ValueError(f"Unknown loss type: {loss_type}")
