"""UNet / AttentionUNet with the reference's API (unet/models/unet.py of seagochen/unet-segment-pytorch).

The whole network runs as one HIP launch plan (`unet._hip.stages.NetworkPlan`): the BN-apply/ReLU/
pad/concat/attention-multiply between modules is fused into the next convolution's tile loader, and
the max-pooled / bilinear-upsampled maps are written once each (`unet_materialize_pool` /
`unet_materialize`) and read plain.  Autograd sees one node per reference module (so DDP overlaps
its all-reduces with the rest of the backward); the parameter tree is the reference's.
"""

import torch
import torch.nn as nn

from .._hip.functions import run_network
from .layers import AttentionUp, DoubleConv, Down, OutConv, Up


class UNet(nn.Module):
    """U-Net (Ronneberger et al.) — reference unet.py:16-106.

    Args: n_channels (1 grayscale / 3 RGB), n_classes, bilinear (else ConvTranspose2d up),
    base_features (64).  forward(x[N, C, H, W]) -> logits[N, n_classes, H, W].
    Extra attribute `hip_precision` ('fp32' default / 'bf16') selects the kernels' operand type.
    """

    def __init__(self, n_channels: int = 1, n_classes: int = 2, bilinear: bool = True, base_features: int = 64):
        super().__init__()
        self.n_channels = n_channels
        self.n_classes = n_classes
        self.bilinear = bilinear
        f = base_features
        factor = 2 if bilinear else 1
        self.inc = DoubleConv(n_channels, f)
        self.down1 = Down(f, 2 * f)
        self.down2 = Down(2 * f, 4 * f)
        self.down3 = Down(4 * f, 8 * f)
        self.down4 = Down(8 * f, 16 * f // factor)
        self.up1 = Up(16 * f, 8 * f // factor, bilinear)
        self.up2 = Up(8 * f, 4 * f // factor, bilinear)
        self.up3 = Up(4 * f, 2 * f // factor, bilinear)
        self.up4 = Up(2 * f, f, bilinear)
        self.outc = OutConv(f, n_classes)
        self.hip_precision = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return run_network(self, x, attention=False)[0]

    def get_num_params(self, trainable_only: bool = True) -> int:
        return sum(p.numel() for p in self.parameters() if p.requires_grad or not trainable_only)


class AttentionUNet(nn.Module):
    """Attention U-Net (Oktay et al.) — reference unet.py:109-217.

    With deep_supervision=True and in training mode, forward returns
    [logits, ds1, ds2, ds3] (auxiliary heads on d2, d3, d4, bilinearly resized to the input size);
    otherwise the logits tensor.
    """

    def __init__(self, n_channels: int = 1, n_classes: int = 2, bilinear: bool = True, base_features: int = 64,
                 deep_supervision: bool = False):
        super().__init__()
        self.n_channels = n_channels
        self.n_classes = n_classes
        self.bilinear = bilinear
        self.deep_supervision = deep_supervision
        f = base_features
        factor = 2 if bilinear else 1
        self.inc = DoubleConv(n_channels, f)
        self.down1 = Down(f, 2 * f)
        self.down2 = Down(2 * f, 4 * f)
        self.down3 = Down(4 * f, 8 * f)
        self.down4 = Down(8 * f, 16 * f // factor)
        self.up1 = AttentionUp(16 * f, 8 * f // factor, bilinear)
        self.up2 = AttentionUp(8 * f, 4 * f // factor, bilinear)
        self.up3 = AttentionUp(4 * f, 2 * f // factor, bilinear)
        self.up4 = AttentionUp(2 * f, f, bilinear)
        self.outc = OutConv(f, n_classes)
        if deep_supervision:
            self.ds_out3 = OutConv(8 * f // factor, n_classes)
            self.ds_out2 = OutConv(4 * f // factor, n_classes)
            self.ds_out1 = OutConv(2 * f // factor, n_classes)
        self.hip_precision = None

    def forward(self, x: torch.Tensor):
        outs = run_network(self, x, attention=True)
        if self.deep_supervision and self.training:
            return list(outs)
        return outs[0]

    def get_num_params(self, trainable_only: bool = True) -> int:
        return sum(p.numel() for p in self.parameters() if p.requires_grad or not trainable_only)
