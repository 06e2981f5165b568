"""On-device confusion matrix / segmentation metrics (csrc/metrics.hip, unet/utils/metrics.py) against
the reference's definitions (unet/utils/metrics.py:55-231) as restated in oracle/unet_oracle.py and
the committed fixture tests/golden/metrics.pt.  Integer counts: bit-exact."""

from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"


def _o():
    from oracle import unet_oracle as O
    return O


def test_confusion_golden_fixture():
    from unet.utils.metrics import SegmentationMetrics
    g = torch.load(GOLD / "metrics.pt", weights_only=True)
    m = SegmentationMetrics(num_classes=2)
    m.update(g["z"].cuda(), g["t"].cuda())
    assert np.array_equal(m.get_confusion_matrix(), g["confusion"].numpy())
    r = m.compute()
    assert r["mean_dice"] == pytest.approx(float(g["mean_dice"]), abs=1e-12)
    assert r["mean_iou"] == pytest.approx(float(g["mean_iou"]), abs=1e-12)


@pytest.mark.parametrize("shape", [(4, 2, 512, 512), (3, 2, 37, 53), (2, 5, 64, 80)])
def test_confusion_matches_oracle(shape):
    from unet.utils.metrics import SegmentationMetrics, compute_dice, compute_iou
    O = _o()
    N, K, H, W = shape
    gen = torch.Generator().manual_seed(11)
    z = torch.randn(N, K, H, W, generator=gen)
    z[0, :, :3, :3] = 0.25                         # ties: the first maximum wins
    t = torch.randint(0, K, (N, H, W), generator=gen)
    m = SegmentationMetrics(num_classes=K)
    m.update(z.cuda(), t.cuda())
    m.update(z.argmax(1).cuda(), t.cuda())         # class-index input, accumulated
    ref = O.confusion_matrix(z.argmax(1), t, K) * 2
    assert np.array_equal(m.get_confusion_matrix(), ref.numpy())
    # per-class IoU / Dice of metrics.py:160-231 (float32 counts, smoothing 1e-6)
    p = z.argmax(1)
    ious = torch.stack([((p == c) & (t == c)).float().sum().add(1e-6) / ((p == c) | (t == c)).float().sum().add(1e-6)
                        for c in range(K)])
    dices = torch.stack([(2.0 * ((p == c).float() * (t == c).float()).sum() + 1e-6) /
                         ((p == c).float().sum() + (t == c).float().sum() + 1e-6) for c in range(K)])
    assert torch.equal(compute_iou(z.cuda(), t.cuda(), K).cpu(), ious)
    assert torch.equal(compute_dice(z.cuda(), t.cuda(), K).cpu(), dices)


def test_confusion_ignore_index_and_out_of_range():
    from unet.utils.metrics import SegmentationMetrics
    O = _o()
    gen = torch.Generator().manual_seed(12)
    z = torch.randn(2, 2, 40, 40, generator=gen)
    t = torch.randint(0, 2, (2, 40, 40), generator=gen)
    t[0, :5] = 255                                  # ignored
    t[1, :2] = 7                                    # out of range: skipped like the reference loop
    m = SegmentationMetrics(num_classes=2, ignore_index=255)
    m.update(z.cuda(), t.cuda())
    keep = (t != 255) & (t < 2)
    ref = O.confusion_matrix(z.argmax(1)[keep], t[keep], 2)
    assert np.array_equal(m.get_confusion_matrix(), ref.numpy())
    m.reset()
    assert m.compute()["mean_dice"] == 0.0


def test_metrics_accept_host_tensors():
    """update() with CPU tensors (what the reference's loop takes) counts on the GPU: same matrix as the
    device inputs, accumulated into one device matrix."""
    from unet.utils.metrics import SegmentationMetrics, compute_dice
    O = _o()
    gen = torch.Generator().manual_seed(13)
    z = torch.randn(2, 2, 33, 47, generator=gen)
    t = torch.randint(0, 2, (2, 33, 47), generator=gen)
    m = SegmentationMetrics(num_classes=2)
    m.update(z, t)
    m.update(z.cuda(), t)
    assert np.array_equal(m.get_confusion_matrix(), (O.confusion_matrix(z.argmax(1), t, 2) * 2).numpy())
    assert m.compute() == O.segmentation_scores(m.get_confusion_matrix(), m.class_names)
    assert torch.equal(compute_dice(z, t).cpu(), compute_dice(z.cuda(), t.cuda()).cpu())


@pytest.mark.parametrize("C,K", [(2, 2), (3, 2), (2, 3)])
def test_iou_dice_count_every_pixel(C, K):
    """compute_iou / compute_dice with targets outside [0, K) (an ignore label 255, a stray 7) and logits
    whose channel count C differs from num_classes: the reference's per-class masks count such pixels in
    |pred == c| (metrics.py:183-188, 217-221); the extended (K+1)^2 matrix does the same."""
    from unet.utils.metrics import compute_dice, compute_iou
    O = _o()
    gen = torch.Generator().manual_seed(14 + C * 3 + K)
    z = torch.randn(3, C, 45, 61, generator=gen)
    t = torch.randint(0, K, (3, 45, 61), generator=gen)
    t[0, :6] = 255
    t[2, :, :4] = 7
    t[1, 3, 5] = -1
    ri, rd = O.class_iou_dice(z.argmax(1), t, K)
    assert torch.equal(compute_iou(z.cuda(), t.cuda(), K).cpu(), ri)
    assert torch.equal(compute_dice(z.cuda(), t.cuda(), K).cpu(), rd)
    # class-index predictions, including labels >= K
    p = z.argmax(1)
    ri, rd = O.class_iou_dice(p, t, K)
    assert torch.equal(compute_iou(p.cuda(), t.cuda(), K).cpu(), ri)
    assert torch.equal(compute_dice(p, t, K).cpu(), rd)


@pytest.mark.parametrize("C,K", [(3, 2), (2, 3), (5, 2)])
def test_update_logits_channels_differ_from_num_classes(C, K):
    """SegmentationMetrics.update with logits whose channel count C != num_classes: the reference takes the
    argmax over all C channels and skips pixels whose class (target or prediction) is outside [0, K)
    (metrics.py:68-84); the device kernel does the same (unet_confusion_matrix with C and K)."""
    from unet.utils.metrics import SegmentationMetrics
    O = _o()
    gen = torch.Generator().manual_seed(40 + C * 7 + K)
    z = torch.randn(2, C, 37, 53, generator=gen)
    t = torch.randint(0, max(C, K) + 1, (2, 37, 53), generator=gen)
    m = SegmentationMetrics(num_classes=K)
    m.update(z.cuda(), t.cuda())
    m.update(z, t)                          # host tensors too
    p = z.argmax(1)
    keep = (t >= 0) & (t < K) & (p >= 0) & (p < K)
    ref = O.confusion_matrix(p[keep], t[keep], K) * 2
    assert np.array_equal(m.get_confusion_matrix(), ref.numpy())
