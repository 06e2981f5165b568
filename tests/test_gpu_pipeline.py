"""GPU: the data path around the network, bit-exact against the CPU oracle (numpy + Pillow restatements of
the reference; oracle/pipeline_oracle.py).

* training slices: GpuSliceTransform vs dataset.py:146-149 +
  apply_basic_transforms (augmentations.py:119-171), with and without the flip, for resize-free
  (512 -> 512), down- and up-scaling and non-square inputs; image fp32 and mask int64 identical;
* inference (row f1): preprocess_images vs predict.py:100-135; postprocess_masks vs predict.py:138-165
  (softmax / threshold / NEAREST; pixels whose p1 is within 1e-6 of the threshold are exempt, their count
  reported); the HIP-graph eval forward equals the eager eval forward bit for bit; predict_masks end to end.
"""

import numpy as np
import pytest
import torch

from oracle import pipeline_oracle as PO

pytestmark = pytest.mark.gpu


def _slices(n, h, w, seed):
    rng = np.random.default_rng(seed)
    imgs = rng.integers(0, 256, (n, h, w), dtype=np.uint8)
    masks = np.zeros((n, h, w), np.uint8)
    for i in range(n):
        cy, cx, r = rng.integers(h // 4, 3 * h // 4), rng.integers(w // 4, 3 * w // 4), rng.integers(3, max(4, h // 6))
        yy, xx = np.mgrid[:h, :w]
        masks[i][(yy - cy) ** 2 + (xx - cx) ** 2 <= r * r] = 255
        masks[i][rng.random((h, w)) < 0.01] = 128          # values either side of the > 127 cut
    return imgs, masks


@pytest.mark.parametrize("h,w,S", [(512, 512, 512), (512, 512, 256), (300, 400, 512), (333, 200, 128)])
def test_training_slices_bit_exact(h, w, S):
    from unet.utils.gpu_pipeline import GpuSliceTransform
    imgs, masks = _slices(4, h, w, h + w + S)
    flips = np.array([True, False, True, False])
    img, mask = GpuSliceTransform(img_size=S)(torch.from_numpy(imgs), torch.from_numpy(masks), flips)
    for i in range(4):
        ri, rm = PO.training_slice(imgs[i], masks[i], S, bool(flips[i]))
        assert torch.equal(img[i].cpu(), ri), (i, float((img[i].cpu() - ri).abs().max()))
        assert torch.equal(mask[i].cpu(), rm), i


def test_validation_slices_no_flip():
    from unet.utils.gpu_pipeline import GpuSliceTransform, draw_flips
    imgs, masks = _slices(3, 256, 256, 3)
    img, mask = GpuSliceTransform(img_size=512)(torch.from_numpy(imgs), torch.from_numpy(masks))
    for i in range(3):
        ri, rm = PO.training_slice(imgs[i], masks[i], 512, False)
        assert torch.equal(img[i].cpu(), ri) and torch.equal(mask[i].cpu(), rm)
    np.random.seed(11)
    a = draw_flips(8)
    np.random.seed(11)
    assert list(a) == [np.random.rand() > 0.5 for _ in range(8)]   # the reference's per-sample draw


@pytest.mark.parametrize("h,w,S", [(512, 512, 256), (300, 420, 256), (512, 512, 512)])
def test_predict_preprocess_bit_exact(h, w, S):
    from unet.utils.inference import preprocess_images
    imgs, _ = _slices(2, h, w, 17)
    out = preprocess_images(torch.from_numpy(imgs), S)
    for i in range(2):
        assert torch.equal(out[i:i + 1].cpu(), PO.predict_preprocess(imgs[i], S))


@pytest.mark.parametrize("H,W,oh,ow", [(256, 256, 512, 512), (256, 256, 300, 420), (64, 64, 64, 64), (128, 96, 333, 77)])
def test_postprocess_masks(H, W, oh, ow):
    from unet.utils.inference import postprocess_masks
    g = torch.Generator().manual_seed(H + ow)
    z = torch.randn(3, 2, H, W, generator=g) * 2
    z[0, :, :8, :8] = 0.0                                  # exact ties: p1 == 0.5, not > 0.5
    zc = z.cuda()
    got = postprocess_masks(zc, (ow, oh), 0.5).cpu().numpy()
    near = 0
    for i in range(3):
        ref = PO.predict_postprocess(zc[i:i + 1], (ow, oh), 0.5)   # the reference runs softmax on the device
        p1 = torch.softmax(z[i:i + 1], 1)[0, 1].numpy()
        from unet.utils.pil_tables import nearest_table
        p1n = p1[nearest_table(H, oh)][:, nearest_table(W, ow)]
        diff = got[i] != ref
        near += int(diff.sum())
        assert not (diff & (np.abs(p1n - 0.5) >= 1e-6)).any(), i
    print(f"\npostprocess: {near} near-threshold pixels differ")


def test_graphed_predictor_matches_eager_and_predict_masks():
    from unet.models import AttentionUNet
    from unet.utils.inference import GraphedPredictor, postprocess_masks, predict_masks, preprocess_images
    torch.manual_seed(0)
    m = AttentionUNet(1, 2, base_features=8).cuda()
    m.hip_precision = "bf16"
    # non-trivial running statistics: one train-mode step's BN updates
    m.train()
    with torch.no_grad():
        m(torch.rand(2, 1, 128, 128, device="cuda") * 2 - 1)
    m.eval()
    imgs, _ = _slices(2, 300, 300, 5)
    x = preprocess_images(torch.from_numpy(imgs), 128)
    with torch.no_grad():
        eager = m(x).clone()
    gp = GraphedPredictor(m, x.shape)
    for _ in range(2):
        out = gp(x)
        assert torch.equal(out, eager)
    masks, ratio = predict_masks(m, torch.from_numpy(imgs), 128, predictor=gp)
    ref = postprocess_masks(eager, (300, 300))
    assert torch.equal(masks, ref)
    assert torch.allclose(ratio, (ref > 127).float().mean((1, 2)))
    assert masks.shape == (2, 300, 300) and masks.dtype == torch.uint8


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_eval_single_pass_gate_in_the_network(prec):
    """model.eval() under no_grad takes the one-pass attention gate (unet_gate_psi_eval); with autograd
    enabled it keeps the two-pass training form.  Both against the fp64 oracle's eval logits: the
    one-pass form (projections never rounded to 16 bits) is no less accurate."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    from oracle import unet_oracle as O
    from unet.models import AttentionUNet
    torch.manual_seed(0)
    m = AttentionUNet(1, 2).cuda()
    m.hip_precision = prec
    m.train()
    with torch.no_grad():
        m(torch.rand(2, 1, 64, 64, device="cuda") * 2 - 1)     # non-trivial running statistics
    m.eval()
    x = torch.rand(2, 1, 64, 64, device="cuda") * 2 - 1
    with torch.no_grad():
        one = m(x).double()
    two = m(x).detach().double()                                # grad enabled: two-pass gate
    p = {k: v.detach().double().cuda() for k, v in m.state_dict().items()}
    ref = O.attention_unet_forward(p, x.double(), training=False)
    e1 = float((one - ref).norm() / ref.norm())
    e2 = float((two - ref).norm() / ref.norm())
    print(f"\n{prec} eval logits rel-L2 vs fp64: one-pass gate {e1:.3e}, two-pass {e2:.3e}")
    assert e1 <= 1.1 * e2 + 1e-3 and e1 <= 2e-2, (e1, e2)
    assert not torch.equal(one, two)        # the one-pass kernel did run
