"""CPU oracle for the data path around the network (TEST INFRASTRUCTURE ONLY; the product never imports
this module).  Plain numpy + Pillow restatements of:

* the training slice path: dataset.py:146-149 (8-bit 'L' slice -> float32 / 255; mask > 127 -> int64) and
  the albumentations-free `apply_basic_transforms` (augmentations.py:119-171): the float round trip
  (image * 255).astype(uint8), PIL resize BILINEAR / NEAREST, optional left-right flip, (x - mean) / std;
* predict.py's `preprocess_image` (:100-135, from an already decoded 8-bit slice) and `postprocess_mask`
  (:138-165: softmax, p1 > threshold -> 255, PIL NEAREST resize);
* `resample_with_tables`: the integer passes of Pillow's 8-bit resampler driven by
  unet.utils.pil_tables — pins those tables against Pillow itself.
Pillow is the reference's own third-party dependency (requirements.txt); it is importable here and on
the GPU box, so these restatements are checked against it directly in the tests."""

from __future__ import annotations

import numpy as np
import torch
from PIL import Image

PRECISION_BITS = 22


def training_slice(img_u8: np.ndarray, mask_u8: np.ndarray, img_size: int, flip: bool, mean=0.5, std=0.5):
    """dataset.py:146-149 + augmentations.py:145-171 with the flip decision given."""
    image = np.asarray(img_u8, dtype=np.float32) / 255.0                      # dataset.py:146
    mask = (np.asarray(mask_u8, dtype=np.uint8) > 127).astype(np.int64)       # dataset.py:148-149
    img_pil = Image.fromarray((image * 255).astype(np.uint8))                 # augmentations.py:150
    mask_pil = Image.fromarray(mask.astype(np.uint8))                         # :151
    img_pil = img_pil.resize((img_size, img_size), Image.BILINEAR)            # :154
    mask_pil = mask_pil.resize((img_size, img_size), Image.NEAREST)           # :155
    image = np.array(img_pil, dtype=np.float32) / 255.0                       # :158
    mask = np.array(mask_pil, dtype=np.int64)                                 # :159
    if flip:                                                                  # :161-163
        image = np.fliplr(image).copy()
        mask = np.fliplr(mask).copy()
    image = (image - mean) / std                                              # :166
    return torch.from_numpy(image).unsqueeze(0).float(), torch.from_numpy(mask).long()


def predict_preprocess(img_u8: np.ndarray, img_size: int, mean=0.5, std=0.5) -> torch.Tensor:
    """predict.py:119-131 from the decoded 8-bit slice."""
    image_resized = Image.fromarray(np.asarray(img_u8, dtype=np.uint8)).resize((img_size, img_size), Image.BILINEAR)
    image_array = np.array(image_resized, dtype=np.float32) / 255.0
    image_normalized = (image_array - mean) / std
    return torch.from_numpy(image_normalized).unsqueeze(0).unsqueeze(0).float()


def predict_postprocess(prediction: torch.Tensor, original_size, threshold: float = 0.5) -> np.ndarray:
    """predict.py:155-165 for one image (prediction (1, C, H, W); original_size = (W, H))."""
    probs = torch.softmax(prediction, dim=1)
    tumor_prob = probs[0, 1].cpu().numpy()
    mask = (tumor_prob > threshold).astype(np.uint8) * 255
    return np.array(Image.fromarray(mask).resize(tuple(original_size), Image.NEAREST))


def resample_with_tables(img: np.ndarray, out_h: int, out_w: int, tables) -> np.ndarray:
    """Pillow's two integer passes (horizontal, then vertical; each only if that size changes) with
    tables(in, out) -> (bounds, coeffs)."""
    img = np.asarray(img, dtype=np.uint8)

    def hpass(a, b, k):
        out = np.zeros((a.shape[0], len(b)), np.uint8)
        for x, (x0, n) in enumerate(b):
            ss = (1 << (PRECISION_BITS - 1)) + (a[:, x0:x0 + n].astype(np.int64) * k[x, :n]).sum(1)
            out[:, x] = np.clip(ss >> PRECISION_BITS, 0, 255)
        return out

    h, w = img.shape
    if w != out_w:
        img = hpass(img, *tables(w, out_w))
    if h != out_h:
        img = hpass(img.T.copy(), *tables(h, out_h)).T.copy()
    return img
