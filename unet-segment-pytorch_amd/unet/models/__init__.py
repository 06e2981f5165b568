"""UNet model components (reference: unet/models/__init__.py)."""

from .layers import DoubleConv, Down, Up, OutConv, AttentionGate, AttentionUp
from .unet import UNet, AttentionUNet

__all__ = ["DoubleConv", "Down", "Up", "OutConv", "AttentionGate", "AttentionUp", "UNet", "AttentionUNet"]
