"""Hot-path utilities (reference: unet/utils/__init__.py).  Only the losses are part of this build;
the reference's host-side metrics/callbacks/plots are out of scope."""

from .loss import DiceLoss, BalancedCELoss, DiceBCELoss, DeepSupervisionLoss, create_loss_function

__all__ = ["DiceLoss", "BalancedCELoss", "DiceBCELoss", "DeepSupervisionLoss", "create_loss_function"]
