"""U-Net building blocks with the reference's constructor signatures and parameter layout.

Drop-in for unet/models/layers.py of seagochen/unet-segment-pytorch: the same class names,
constructor arguments, submodule names and nn.Sequential indices (so state_dict keys and
checkpoints are interchangeable), and the same forward signatures.  The parameters live in
ordinary nn.Conv2d / nn.BatchNorm2d containers (fp32 OIHW); `forward` runs the HIP launch plan in
`unet._hip` instead of ATen.  There is no CPU path: inputs must be on the ROCm GPU.
"""

import torch
import torch.nn as nn

from .._hip.functions import run_module


def _conv_bn_relu(cin: int, cout: int):
    return [nn.Conv2d(cin, cout, kernel_size=3, padding=1, bias=False), nn.BatchNorm2d(cout), nn.ReLU(inplace=True)]


class DoubleConv(nn.Module):
    """(conv3x3 -> BN -> ReLU) x 2 — reference layers.py:16-41.  `mid_channels` defaults to
    `out_channels`."""

    def __init__(self, in_channels: int, out_channels: int, mid_channels: int = None):
        super().__init__()
        mid = out_channels if mid_channels is None else mid_channels
        self.double_conv = nn.Sequential(*_conv_bn_relu(in_channels, mid), *_conv_bn_relu(mid, out_channels))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return run_module(self, "double_conv", x)


class Down(nn.Module):
    """MaxPool2d(2) -> DoubleConv — reference layers.py:44-61."""

    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.maxpool_conv = nn.Sequential(nn.MaxPool2d(2), DoubleConv(in_channels, out_channels))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return run_module(self, "down", x)


class Up(nn.Module):
    """up(x1) -> pad to skip -> cat([skip, up]) -> DoubleConv — reference layers.py:64-106.
    bilinear: Upsample(x2, align_corners=True) and DoubleConv(in, out, in//2);
    else ConvTranspose2d(in, in//2, 2, 2) and DoubleConv(in, out)."""

    def __init__(self, in_channels: int, out_channels: int, bilinear: bool = True):
        super().__init__()
        if bilinear:
            self.up = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True)
            self.conv = DoubleConv(in_channels, out_channels, in_channels // 2)
        else:
            self.up = nn.ConvTranspose2d(in_channels, in_channels // 2, kernel_size=2, stride=2)
            self.conv = DoubleConv(in_channels, out_channels)

    def forward(self, x1: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
        return run_module(self, "up", x1, x2)


class OutConv(nn.Module):
    """1x1 conv with bias — reference layers.py:109-123."""

    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size=1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return run_module(self, "out_conv", x)


class AttentionGate(nn.Module):
    """Additive attention gate (Oktay et al.) — reference layers.py:126-192.
    g_up = bilinear(g, size=x) ; s = sigmoid(BN(psi(relu(BN(W_g g_up) + BN(W_x x))))) ; return x * s."""

    def __init__(self, gate_channels: int, skip_channels: int, inter_channels: int = None):
        super().__init__()
        inter = skip_channels // 2 if inter_channels is None else inter_channels
        self.W_g = nn.Sequential(nn.Conv2d(gate_channels, inter, kernel_size=1, bias=False), nn.BatchNorm2d(inter))
        self.W_x = nn.Sequential(nn.Conv2d(skip_channels, inter, kernel_size=1, bias=False), nn.BatchNorm2d(inter))
        self.psi = nn.Sequential(nn.Conv2d(inter, 1, kernel_size=1, bias=False), nn.BatchNorm2d(1), nn.Sigmoid())
        self.relu = nn.ReLU(inplace=True)

    def forward(self, g: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
        return run_module(self, "attention_gate", g, x)


class AttentionUp(nn.Module):
    """Gate the skip with the pre-upsample decoder map, then Up — reference layers.py:195-255."""

    def __init__(self, in_channels: int, out_channels: int, bilinear: bool = True):
        super().__init__()
        if bilinear:
            self.up = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True)
            gate_channels = skip_channels = in_channels // 2
            self.conv = DoubleConv(in_channels, out_channels, in_channels // 2)
        else:
            self.up = nn.ConvTranspose2d(in_channels, in_channels // 2, kernel_size=2, stride=2)
            gate_channels, skip_channels = in_channels, in_channels // 2
            self.conv = DoubleConv(in_channels, out_channels)
        self.attention = AttentionGate(gate_channels=gate_channels, skip_channels=skip_channels)

    def forward(self, x1: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
        return run_module(self, "attention_up", x1, x2)
