"""MI355X-native drop-in for the `unet` package of seagochen/unet-segment-pytorch (hot path only).

`unet.models` and `unet.utils.loss` keep the reference's names, constructors, state_dict layout and
forward signatures; their compute runs as hand-written HIP kernels for gfx950.
"""

__version__ = "0.1.0"

from .models.unet import UNet, AttentionUNet
from .models.layers import DoubleConv, Down, Up, OutConv, AttentionGate, AttentionUp
from ._hip.runtime import set_precision, get_precision

__all__ = [
    "UNet",
    "AttentionUNet",
    "DoubleConv",
    "Down",
    "Up",
    "OutConv",
    "AttentionGate",
    "AttentionUp",
    "set_precision",
    "get_precision",
]
