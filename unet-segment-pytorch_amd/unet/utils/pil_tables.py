"""Pillow's resampling tables (host side of the device input pipeline / inference post-processing).

The reference resizes with PIL (`Image.resize(BILINEAR)` for slices, `NEAREST` for masks,
unet/data/augmentations.py:153-154, scripts/predict.py:124,162).  Pillow 8-bit resampling is integer
arithmetic on coefficient tables that it computes in double precision; the device kernels
(csrc/infer.hip) run the integer part, and these functions build the same tables Pillow builds:

* `bilinear_tables(in, out)`: Resample.c `precompute_coeffs` with the bilinear filter (support 1,
  widened by the downscale factor) and `normalize_coeffs_8bpc` (coefficients in 22-bit fixed point,
  rounded half away from zero) -> (bounds[out][2] = (first source index, count), coeffs[out][ksize]);
* `nearest_table(in, out)`: Geometry.c `ImagingScaleAffine` — the source coordinate starts at
  0.5 * in / out and advances by in / out per output pixel (repeated double additions, truncated), which
  is not always floor((o + 0.5) * in / out).
Bit-exactness against Pillow itself is checked in tests (test_pipeline_tables_match_pillow).
"""

from __future__ import annotations

import math
from functools import lru_cache

import numpy as np

PRECISION_BITS = 32 - 8 - 2


@lru_cache(maxsize=64)
def bilinear_tables(in_size: int, out_size: int):
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    coeffs = np.zeros((out_size, ksize), np.int32)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        w = []
        ww = 0.0
        for x in range(xmax):
            v = (x + xmin - center + 0.5) * ss
            v = -v if v < 0 else v
            f = 1.0 - v if v < 1.0 else 0.0
            w.append(f)
            ww += f
        for x in range(xmax):
            k = w[x] / ww if ww != 0.0 else w[x]
            coeffs[xx, x] = int(-0.5 + k * (1 << PRECISION_BITS)) if k < 0 else int(0.5 + k * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, coeffs


@lru_cache(maxsize=64)
def nearest_table(in_size: int, out_size: int) -> np.ndarray:
    a0 = in_size / out_size
    xo = a0 * 0.5
    t = np.empty(out_size, np.int32)
    for x in range(out_size):
        t[x] = -1 if xo < 0 else int(xo)
        xo += a0
    return np.clip(t, 0, in_size - 1).astype(np.int32)
