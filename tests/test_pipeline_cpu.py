"""CPU: the host-side tables of the device input pipeline / inference post-processing against Pillow
itself (the reference's resampler: augmentations.py:153-154, predict.py:124,162)."""

import numpy as np
import pytest
from PIL import Image

from oracle import pipeline_oracle as PO


SIZES = [(512, 512, 256, 256), (300, 400, 512, 512), (512, 512, 333, 777), (64, 48, 100, 30), (7, 9, 3, 20),
         (512, 512, 511, 513), (1000, 700, 512, 512)]


@pytest.mark.parametrize("h,w,oh,ow", SIZES)
def test_pipeline_tables_match_pillow(h, w, oh, ow):
    from unet.utils.pil_tables import bilinear_tables, nearest_table
    rng = np.random.default_rng(h * 7 + ow)
    img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    ref = np.array(Image.fromarray(img).resize((ow, oh), Image.BILINEAR))
    mine = PO.resample_with_tables(img, oh, ow, bilinear_tables)
    assert np.array_equal(ref, mine)
    refn = np.array(Image.fromarray(img).resize((ow, oh), Image.NEAREST))
    assert np.array_equal(refn, img[nearest_table(h, oh)][:, nearest_table(w, ow)])
