"""Hot-path utilities (reference: unet/utils/__init__.py): the losses and the segmentation metrics
(confusion matrix counted on the device).  The reference's host-side callbacks/plots/dataset are out
of scope."""

from .loss import DiceLoss, BalancedCELoss, DiceBCELoss, DeepSupervisionLoss, create_loss_function
from .metrics import SegmentationMetrics, compute_dice, compute_iou
from .config import load_config, create_model, create_criterion, build_from_config

__all__ = ["DiceLoss", "BalancedCELoss", "DiceBCELoss", "DeepSupervisionLoss", "create_loss_function",
           "SegmentationMetrics", "compute_iou", "compute_dice", "load_config", "create_model", "create_criterion",
           "build_from_config"]
