"""Segmentation metrics on the device (reference: unet/utils/metrics.py).

`SegmentationMetrics` keeps the reference's API (metrics.py:16-158): `update(predictions, targets)`
accumulates a K x K int64 confusion matrix, `compute()` returns pixel accuracy, per-class and mean
IoU / Dice with the same formulas (metrics.py:86-143, classes whose score is exactly 0 are left out of
the means, :131-135).  The difference is where the counting runs: the reference moves every batch to the
host and walks the pixels in a Python loop (metrics.py:78-84); here `update` is one HIP launch
(`unet_confusion_matrix`: argmax over the logits + LDS histogram + 64-bit atomics) that accumulates into
a device tensor without synchronising, and only `compute()` / `get_confusion_matrix()` read it back.
Counts are integers, so the matrix is bit-identical to the reference's.

`compute_iou` / `compute_dice` (metrics.py:160-231) are built on the same kernel.
"""

from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch

from .._hip import lib as L
from .._hip.runtime import require_device, stream

__all__ = ["SegmentationMetrics", "compute_iou", "compute_dice", "confusion_matrix"]


def confusion_matrix(predictions: torch.Tensor, targets: torch.Tensor, num_classes: int = 2,
                     ignore_index: Optional[int] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """int64 [K, K] device tensor, confusion[t, p] (+)= pixel counts (into `out` when given).

    predictions: logits (N, C, H, W) — argmax over dim 1 — or class indices (N, H, W).  Host tensors (what
    the reference's loop takes) are copied to the current GPU first; the counting always runs in HIP.

    Targets outside [0, K) (and `ignore_index`) are not counted, as in the reference's update()
    (metrics.py:76-84).  (compute_iou / compute_dice count every pixel instead: `_class_counts`.)"""
    if not predictions.is_cuda:
        predictions = predictions.to(f"cuda:{torch.cuda.current_device()}")
    if targets.device != predictions.device:
        targets = targets.to(predictions.device)
    require_device(predictions, "predictions")
    require_device(targets, "targets")
    K = int(num_classes)
    if out is None:
        out = torch.zeros(K, K, dtype=torch.int64, device=predictions.device)
    t = targets.to(torch.int64).contiguous()
    if predictions.dim() == 4:
        z = predictions.detach().float().contiguous()
        # argmax over however many channels the logits have; a class >= K is then skipped like the
        # reference's `0 <= p < num_classes` test (metrics.py:68-84)
        N, C, H, W = z.shape
        logits, labels = z.data_ptr(), None
    else:
        p = predictions.detach().to(torch.int64).contiguous()
        N = p.shape[0]
        C, H, W = 1, 1, p.numel() // max(N, 1)
        logits, labels = None, p.data_ptr()
    if t.numel() != N * H * W:
        raise ValueError(f"targets have {t.numel()} elements, predictions describe {N * H * W} pixels")
    L.call("unet_confusion_matrix", N, C, K, H * W, logits, labels, t.data_ptr(),
           int(ignore_index) if ignore_index is not None else 0, int(ignore_index is not None), out.data_ptr(),
           stream())
    return out


class SegmentationMetrics:
    """Accumulates a confusion matrix over batches and computes segmentation metrics
    (reference: metrics.py:16-158; same constructor, methods and result keys)."""

    def __init__(self, num_classes: int = 2, class_names: Optional[List[str]] = None,
                 ignore_index: Optional[int] = None):
        self.num_classes = num_classes
        self.class_names = class_names or [f'class_{i}' for i in range(num_classes)]
        self.ignore_index = ignore_index
        self._cm: Optional[torch.Tensor] = None   # device int64 accumulator

    @property
    def confusion_matrix(self) -> np.ndarray:
        """confusion[i, j] = pixels with true class i predicted as class j (host copy)."""
        if self._cm is None:
            return np.zeros((self.num_classes, self.num_classes), dtype=np.int64)
        return self._cm.cpu().numpy()

    def reset(self) -> None:
        """Reset accumulated statistics."""
        self._cm = None

    def update(self, predictions: torch.Tensor, targets: torch.Tensor) -> None:
        """Add a batch: logits (N, C, H, W) or class indices (N, H, W); targets (N, H, W).  Host tensors
        are accepted (copied to the current GPU)."""
        if not predictions.is_cuda:
            predictions = predictions.to(f"cuda:{torch.cuda.current_device()}")
        if self._cm is None:
            self._cm = torch.zeros(self.num_classes, self.num_classes, dtype=torch.int64, device=predictions.device)
        elif self._cm.device != predictions.device:
            predictions = predictions.to(self._cm.device)
        confusion_matrix(predictions, targets, self.num_classes, self.ignore_index, out=self._cm)

    def compute(self) -> Dict[str, float]:
        """pixel_accuracy, mean_iou, mean_dice, class_iou, class_dice (metrics.py:86-143).

        All classes at once from the matrix: with tp = diag, |pred| = column sums and |true| = row sums,
        IoU = tp / (|pred| + |true| - tp) and Dice = 2 tp / (|pred| + |true|), 0 where the denominator
        is 0; the means run over the classes whose score is non-zero.  Integer counts divided in float64,
        as the reference's per-class scalar arithmetic does, so the values are identical."""
        cm = self.confusion_matrix
        names = self.class_names
        total = int(cm.sum())
        tp = np.diagonal(cm)
        both = cm.sum(0) + cm.sum(1)                 # |pred| + |true| per class
        union, dsum = both - tp, both
        iou = np.divide(tp, union, out=np.zeros(len(tp)), where=union > 0)
        dice = np.divide(2 * tp, dsum, out=np.zeros(len(tp)), where=dsum > 0)

        def nz_mean(v):
            v = v[v > 0]
            return float(np.mean(v)) if v.size else 0.0

        return {
            'pixel_accuracy': float(tp.sum() / total) if total else 0.0,
            'mean_iou': nz_mean(iou) if total else 0.0,
            'mean_dice': nz_mean(dice) if total else 0.0,
            'class_iou': dict(zip(names, map(float, iou))),
            'class_dice': dict(zip(names, map(float, dice))),
        }

    def get_confusion_matrix(self) -> np.ndarray:
        """Return the confusion matrix (host copy)."""
        return self.confusion_matrix.copy()


def _class_counts(predictions: torch.Tensor, targets: torch.Tensor, num_classes: int):
    """(|pred ∩ target|, |pred|, |target|) per class c < num_classes over EVERY pixel, as the reference's
    per-class masks count them (metrics.py:183-188, 217-221): one `unet_confusion_matrix_ext` launch
    into a (K+1) x (K+1) matrix whose last row / column holds targets / predictions outside [0, K)
    (e.g. an ignore label 255, or argmax classes >= K when the logits have C != K channels)."""
    if not predictions.is_cuda:
        predictions = predictions.to(f"cuda:{torch.cuda.current_device()}")
    if targets.device != predictions.device:
        targets = targets.to(predictions.device)
    require_device(predictions, "predictions")
    K = int(num_classes)
    t = targets.to(torch.int64).contiguous()
    if predictions.dim() == 4:
        z = predictions.detach().float().contiguous()
        N, C, H, W = z.shape
        logits, labels, P = z.data_ptr(), None, N * H * W
    else:
        p = predictions.detach().to(torch.int64).contiguous()
        N, C, P = p.shape[0], 0, p.numel()
        logits, labels = None, p.data_ptr()
    if t.numel() != P:
        raise ValueError(f"targets have {t.numel()} elements, predictions describe {P} pixels")
    cm = torch.zeros(K + 1, K + 1, dtype=torch.int64, device=predictions.device)
    L.call("unet_confusion_matrix_ext", N, C, K, P // max(N, 1), logits, labels, t.data_ptr(), cm.data_ptr(),
           stream())
    cm = cm.to(torch.float32)
    tp = torch.diagonal(cm)[:K]
    pred = cm.sum(0)[:K]     # pixels predicted as class c (any target)
    true = cm.sum(1)[:K]     # pixels labelled class c (any prediction)
    return tp, pred, true


def compute_iou(predictions: torch.Tensor, targets: torch.Tensor, num_classes: int = 2,
                smooth: float = 1e-6) -> torch.Tensor:
    """Per-class (I + s) / (U + s), U = |pred ∪ target| (metrics.py:160-193)."""
    tp, pred, true = _class_counts(predictions, targets, num_classes)
    return (tp + smooth) / ((pred + true - tp) + smooth)


def compute_dice(predictions: torch.Tensor, targets: torch.Tensor, num_classes: int = 2,
                 smooth: float = 1e-6) -> torch.Tensor:
    """Per-class (2I + s) / (|pred| + |target| + s) (metrics.py:196-231)."""
    tp, pred, true = _class_counts(predictions, targets, num_classes)
    return (2.0 * tp + smooth) / ((pred + true) + smooth)
