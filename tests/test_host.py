"""CPU: host-side logic of the drop-in — API surface, parameter tree, seeded init, C-ABI exports,
and the fail-loudly contract (no CPU fallback)."""

import re

import numpy as np
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parent.parent


def test_api_surface():
    import unet
    from unet.models import AttentionGate, AttentionUNet, AttentionUp, DoubleConv, Down, OutConv, Up, UNet  # noqa
    from unet.utils.loss import (BalancedCELoss, DeepSupervisionLoss, DiceBCELoss, DiceLoss,  # noqa
                                 create_loss_function)
    assert unet.__version__ == "0.1.0"
    for n in ["UNet", "AttentionUNet", "DoubleConv", "Down", "Up", "OutConv", "AttentionGate", "AttentionUp"]:
        assert n in unet.__all__


def test_state_dict_layout_matches_reference(golden_models):
    from unet.models import AttentionUNet, UNet
    for name, rec in golden_models.items():
        torch.manual_seed(0)
        c = rec["x"].shape[1]
        m = (UNet(c, 2, rec["bilinear"], rec["base"]) if rec["kind"] == "unet"
             else AttentionUNet(c, 2, rec["bilinear"], rec["base"], rec["deep_supervision"]))
        sd = m.state_dict()
        assert list(sd.keys()) == rec["keys"], name
        assert {k: list(v.shape) for k, v in sd.items()} == rec["shapes"], name
        assert sum(p.numel() for p in m.parameters()) == rec["num_params"]
        for k, s in rec["param_sums"].items():   # seeded init is bit-identical to the reference's
            assert float(sd[k].double().sum()) == pytest.approx(s, abs=1e-9), (name, k)


def test_full_size_seeded_init():
    from conftest import load_golden
    from unet.models import AttentionUNet, UNet
    ref = load_golden("seeded.pt")
    torch.manual_seed(0)
    m = AttentionUNet(1, 2)
    assert float(m.inc.double_conv[0].weight.detach().sum()) == ref["first_conv_sum"]
    assert m.get_num_params() == ref["num_params"] == 17612458
    assert UNet(1, 2).get_num_params() == ref["num_params_unet"] == 17261890
    assert list(m.state_dict().keys()) == ref["keys_attention_unet"]


def test_reference_checkpoint_loads(golden_models):
    from unet.models import AttentionUNet
    rec = golden_models["attention_unet_b8"]
    m = AttentionUNet(1, 2, True, 8)
    m.load_state_dict(rec["init"])          # strict: every key and shape matches


def test_create_loss_function():
    from unet.utils.loss import BalancedCELoss, DiceBCELoss, DiceLoss, create_loss_function
    assert isinstance(create_loss_function("dice_bce"), DiceBCELoss)
    assert isinstance(create_loss_function("DICE"), DiceLoss)
    assert isinstance(create_loss_function("balanced_ce", balanced_class_weight=0.3), BalancedCELoss)
    assert isinstance(create_loss_function("ce"), torch.nn.CrossEntropyLoss)
    with pytest.raises(ValueError):
        create_loss_function("focal")


def _header_symbols():
    text = (ROOT / "include" / "unet_hip.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(unet_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    import ctypes
    from unet._hip import lib as L
    path = L.library_path()
    assert path.exists(), "libunet_hip.so not built (run __graft_entry__.build())"
    so = ctypes.CDLL(str(path))
    syms = _header_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(so, s), s
    assert set(syms) == set(L.exported_symbols()), "lib.py signatures out of sync with the header"
    assert L.load().unet_version() == L.ABI_VERSION
    hdr = (ROOT / "include" / "unet_hip.h").read_text()
    assert f"#define UNET_ABI_VERSION {L.ABI_VERSION}" in hdr


def test_no_cpu_fallback():
    from unet.models import DoubleConv, UNet
    from unet.utils.loss import DiceBCELoss
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        DoubleConv(1, 4)(torch.randn(1, 1, 8, 8))
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        UNet(1, 2, base_features=4)(torch.randn(1, 1, 32, 32))
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        DiceBCELoss()(torch.randn(1, 2, 8, 8), torch.zeros(1, 8, 8, dtype=torch.long))


def test_product_never_imports_oracle():
    pkg = ROOT / "unet-segment-pytorch_amd"
    for f in pkg.rglob("*.py"):
        assert "oracle" not in f.read_text().replace("oracle/ is test", ""), f


@pytest.mark.parametrize("K", [2, 3, 5])
def test_metrics_compute_matches_reference_formulas(K):
    """SegmentationMetrics.compute() (vectorised over classes) against the oracle's per-class restatement
    of metrics.py:86-143 on random confusion matrices, incl. absent classes (zero row + column), a class
    never predicted, and the empty matrix: identical floats."""
    import torch
    from oracle import unet_oracle as O
    from unet.utils.metrics import SegmentationMetrics
    rng = np.random.default_rng(K)
    mats = [rng.integers(0, 10 ** rng.integers(1, 7), (K, K)) for _ in range(20)]
    z = rng.integers(0, 1000, (K, K))
    z[1, :] = 0
    z[:, 1] = 0
    mats.append(z)
    z = rng.integers(0, 1000, (K, K))
    z[:, 0] = 0
    mats.append(z)
    mats.append(np.zeros((K, K), np.int64))
    for cm in mats:
        m = SegmentationMetrics(num_classes=K)
        m._cm = torch.from_numpy(cm.astype(np.int64))
        assert m.compute() == O.segmentation_scores(cm.astype(np.int64), m.class_names)


def test_graphed_train_step_rejects_other_optimizers():
    """GraphedTrainStep undoes its warm-up by restoring Adam's fresh state: any other optimizer, or a
    non-capturable Adam, is refused before anything touches the device."""
    from unet.models import UNet
    from unet.utils.graphed import GraphedTrainStep
    from unet.utils.loss import DiceBCELoss
    m = UNet(1, 2, base_features=4)
    with pytest.raises(RuntimeError, match="Adam"):
        GraphedTrainStep(m, DiceBCELoss(), torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9), (1, 1, 8, 8), (1, 8, 8))
    with pytest.raises(RuntimeError, match="capturable"):
        GraphedTrainStep(m, DiceBCELoss(), torch.optim.AdamW(m.parameters(), lr=1e-3), (1, 1, 8, 8), (1, 8, 8))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_relu_after_16bit_rounding_identity(dt):
    """conv5 / wgrad5 apply the BN-activation's ReLU after the 16-bit rounding, as a signed 16-bit integer max
    against 0 on the packed result (v_pk_max_i16): for a multiplier g >= 0 (the attention gate's sigmoid, or the
    0 / 1 zero-padding mask), max_i16(round16(t * g), 0) has the bits of round16(max(t, 0) * g), the round-3
    order, except that a negative zero becomes +0 (which no sum can tell apart)."""
    g = torch.Generator().manual_seed(5)
    t = torch.randn(200000, generator=g) * torch.exp(torch.randn(200000, generator=g) * 4)
    m = torch.rand(200000, generator=g)
    m[::7] = 0.0
    m[::11] = 1.0
    ref = (torch.clamp(t, min=0.0) * m).to(dt)
    new_bits = torch.clamp((t * m).to(dt).view(torch.int16), min=0)
    ref_bits = ref.view(torch.int16)
    # -0.0 (0x8000) in the reference is +0 in the new order
    ref_bits = torch.where(ref_bits == -32768, torch.zeros_like(ref_bits), ref_bits)
    assert torch.equal(new_bits, ref_bits)


def test_torch_ops_library_registers_and_refuses_cpu():
    """The TORCH_LIBRARY(unet_hip) operators (csrc/torch_ops.cpp) load on the host, report the header's ABI version,
    carry the documented schemas, and refuse CPU tensors (no CPU kernels are registered; no fallback)."""
    from unet._hip import lib as L
    from unet._hip import torch_ops
    ops = torch_ops.load()
    assert ops.abi_version() == L.ABI_VERSION
    assert "-> (Tensor loss, Tensor coef)" in str(ops.dice_bce_fwd.default._schema)
    assert "int ignore_index=-1" in str(ops.confusion_matrix.default._schema)
    z, t = torch.randn(1, 2, 8, 8), torch.zeros(1, 8, 8, dtype=torch.long)
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        ops.dice_bce_fwd(z, t, 1.0, 1.0, 0.5, 1e-6, 1.0, True, 0)
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        ops.confusion_matrix(z, t, 2)
