"""Device-side slice preprocessing (the GPU input pipeline).

The reference prepares every training slice on the CPU in a DataLoader worker
(`LungTumorDataset.__getitem__`, unet/data/dataset.py:133-171, and the albumentations-free fallback
`apply_basic_transforms`, unet/data/augmentations.py:119-171): PIL decode, a float round trip
(u8 / 255 * 255 -> uint8), `Image.resize(BILINEAR)` of the image and `NEAREST` of the mask, a random
horizontal flip, /255 and (x - mean) / std, mask > 127 -> int64.  At ~1,000 img/s per node, 4 CPU
workers per GPU cannot keep up.  Here only the PNG decode stays on the host: a batch of decoded 8-bit
slices is uploaded once and every other step runs as integer/byte HIP kernels (csrc/infer.hip) with
Pillow's own resampling tables (unet.utils.pil_tables), bit-exact with the CPU path.

    tf = GpuSliceTransform(img_size=512)
    images, masks = tf(u8_slices, u8_masks, flips=draw_flips(len(u8_slices)))
"""

from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from .._hip import lib as L
from .._hip.runtime import require_device, stream, vp
from .pil_tables import bilinear_tables, nearest_table


def draw_flips(n: int, rng=np.random) -> np.ndarray:
    """The reference's per-sample flip decision, `np.random.rand() > 0.5` (augmentations.py:161), drawn in
    sample order from the same global numpy stream."""
    return np.array([rng.rand() > 0.5 for _ in range(n)], dtype=bool)


class _Tables:
    def __init__(self, device):
        self.device = device
        self._cache = {}

    def bilinear(self, in_size: int, out_size: int):
        key = ("b", in_size, out_size)
        if key not in self._cache:
            b, k = bilinear_tables(in_size, out_size)
            self._cache[key] = (torch.from_numpy(b.copy()).to(self.device), torch.from_numpy(k.copy()).to(self.device),
                                k.shape[1])
        return self._cache[key]

    def nearest(self, in_size: int, out_size: int) -> torch.Tensor:
        key = ("n", in_size, out_size)
        if key not in self._cache:
            self._cache[key] = torch.from_numpy(nearest_table(in_size, out_size).copy()).to(self.device)
        return self._cache[key]


def resize_bilinear_u8(x: torch.Tensor, out_h: int, out_w: int, tables: _Tables, roundtrip: bool) -> Tuple[torch.Tensor, bool]:
    """PIL Image.resize((out_w, out_h), BILINEAR) of a (N, h, w) uint8 device batch (horizontal pass, then
    vertical, each only when that size changes, as Pillow does).  `roundtrip` applies the dataset's
    u8 -> float -> u8 truncation to the source pixels of the first pass; returns (result, still_pending)."""
    N, h, w = x.shape
    cur, rt = x, roundtrip
    if w != out_w:
        b, k, ks = tables.bilinear(w, out_w)
        out = torch.empty(N, h, out_w, dtype=torch.uint8, device=x.device)
        L.call("unet_resample_u8", 1, N, h, w, out_w, vp(cur), int(rt), vp(b), vp(k), ks, vp(out), stream())
        cur, rt = out, False
    if h != out_h:
        b, k, ks = tables.bilinear(h, out_h)
        out = torch.empty(N, out_h, out_w, dtype=torch.uint8, device=x.device)
        L.call("unet_resample_u8", 0, N, h, out_w, out_h, vp(cur), int(rt), vp(b), vp(k), ks, vp(out), stream())
        cur, rt = out, False
    return cur, rt


class GpuSliceTransform:
    """`apply_basic_transforms(image, mask, img_size, mean, std, is_train)` (augmentations.py:119-171) for a
    batch of decoded slices, on the GPU.  images / masks: uint8 (N, h, w) (host or device; the 8-bit
    'L' decode of the PNGs, as dataset.py:146-147 reads them); flips: bool (N,) or None (no flip: the
    validation path)."""

    def __init__(self, img_size: int = 256, mean: float = 0.5, std: float = 0.5, device="cuda"):
        self.img_size = int(img_size)
        self.mean, self.std = float(mean), float(std)
        self.device = torch.device(device)
        self.tables = _Tables(self.device)

    def __call__(self, images: torch.Tensor, masks: Optional[torch.Tensor] = None,
                 flips: Optional[Sequence[bool]] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        x = torch.as_tensor(images)
        if x.dim() == 2:
            x = x[None]
        if x.dtype != torch.uint8 or x.dim() != 3:
            raise RuntimeError(f"expected uint8 images (N, H, W), got {x.dtype} {tuple(x.shape)}")
        x = x.to(self.device, non_blocking=True).contiguous()
        require_device(x, "images")
        N, h, w = x.shape
        S = self.img_size
        r, pending = resize_bilinear_u8(x, S, S, self.tables, roundtrip=True)
        fl = None
        if flips is not None:
            fl = torch.as_tensor(np.asarray(flips, dtype=np.uint8)).to(self.device, non_blocking=True)
            if fl.numel() != N:
                raise RuntimeError(f"{fl.numel()} flip flags for {N} images")
        img = torch.empty(N, 1, S, S, dtype=torch.float32, device=self.device)
        mk, mask_out, yt, xt, mh, mw = None, None, None, None, 0, 0
        if masks is not None:
            mk = torch.as_tensor(masks)
            if mk.dim() == 2:
                mk = mk[None]
            if mk.dtype != torch.uint8 or mk.shape[0] != N:
                raise RuntimeError(f"expected uint8 masks (N, H, W), got {mk.dtype} {tuple(mk.shape)}")
            mk = mk.to(self.device, non_blocking=True).contiguous()
            mh, mw = mk.shape[1], mk.shape[2]
            yt, xt = self.tables.nearest(mh, S), self.tables.nearest(mw, S)
            mask_out = torch.empty(N, S, S, dtype=torch.int64, device=self.device)
        L.call("unet_slice_finish", N, S, S, vp(r), int(pending), mh, mw, vp(mk), vp(yt), vp(xt), vp(fl), self.mean,
               self.std, vp(img), vp(mask_out), stream())
        return img, mask_out
