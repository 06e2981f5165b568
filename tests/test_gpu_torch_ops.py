"""The TORCH_LIBRARY(unet_hip) operators (csrc/torch_ops.cpp, unet._hip.torch_ops) against the package's own ctypes
path on the same inputs: the fused loss (forward value and gradient) and the confusion matrix, bit-identical (the
same kernels on the same stream; reference loss.py:18-191, metrics.py:55-84)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from unet._hip import torch_ops
    return torch_ops.load()


def _batch(N, K, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    z = (torch.randn(N, K, H, W, generator=g) * 3).cuda()
    t = torch.randint(0, K, (N, H, W), generator=g).cuda()
    return z, t


# (module, the _fused arguments it passes: ce_w, dice_w, class_w, ce_smooth, dice_smooth, ignore_bg, reduction)
def _cases():
    from unet.utils.loss import BalancedCELoss, DiceBCELoss, DiceLoss
    return [
        (DiceBCELoss(), (1.0, 1.0, 0.5, 1e-6, 1.0, True, 0)),
        (DiceBCELoss(ce_weight=0.3, dice_weight=2.0, class_weight=0.8), (0.3, 2.0, 0.8, 1e-6, 1.0, True, 0)),
        (DiceLoss(), (0.0, 1.0, 0.5, 1e-6, 1.0, True, 0)),
        (DiceLoss(reduction="sum", ignore_background=False), (0.0, 1.0, 0.5, 1e-6, 1.0, False, 1)),
        (DiceLoss(reduction="none"), (0.0, 1.0, 0.5, 1e-6, 1.0, True, 2)),
        (BalancedCELoss(class_weight=0.3), (1.0, 0.0, 0.3, 1e-6, 1.0, True, 0)),
    ]


@pytest.mark.parametrize("shape", [(2, 2, 64, 96), (3, 4, 33, 47)])
def test_loss_ops_match_modules(shape):
    ops = _ops()
    z0, t = _batch(*shape, seed=sum(shape))
    for i, (mod, args) in enumerate(_cases()):
        z = z0.clone().requires_grad_(True)
        loss = mod(z, t)
        gout = torch.rand(loss.shape, generator=torch.Generator().manual_seed(i)).cuda() + 0.5
        loss.backward(gout)
        l2, coef = ops.dice_bce_fwd(z0, t, *args)
        dz = ops.dice_bce_bwd(z0, t, coef, gout, args[6], args[5])
        assert torch.equal(l2, loss.detach()), (mod, l2, loss)
        assert torch.equal(dz, z.grad), (mod, float((dz - z.grad).abs().max()))


@pytest.mark.parametrize("ignore", [-1, 1])
def test_confusion_matrix_op_matches_metrics(ignore):
    from unet.utils.metrics import confusion_matrix
    ops = _ops()
    z, t = _batch(2, 3, 40, 72, seed=7)
    t[0, :5] = 7                     # outside [0, K): skipped by both
    cm_ref = confusion_matrix(z, t, 3, None if ignore < 0 else ignore)
    cm = ops.confusion_matrix(z, t, 3, ignore)
    assert cm.dtype == torch.int64 and torch.equal(cm, cm_ref), (cm, cm_ref)
    assert int(cm.sum()) == int(((t >= 0) & (t < 3) & (t != ignore)).sum())
