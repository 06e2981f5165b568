"""unet.utils.config: the model / loss block of scripts/train.py:306-342 driven by a YAML config with the
reference's keys (configs/lung_tumor.yaml layout), plus this backend's model.backend / model.precision keys.
CPU only: construction, no forward."""

import pytest
import torch

from unet.models import AttentionUNet, UNet
from unet.utils import build_from_config, create_criterion, create_model
from unet.utils.loss import DeepSupervisionLoss, DiceBCELoss, DiceLoss

YAML = """
model:
  type: attention_unet
  n_channels: 1
  n_classes: 2
  bilinear: true
  base_features: 64
  deep_supervision: false
  precision: bf16
loss:
  type: dice_bce
  balanced_class_weight: 0.5
  ce_weight: 1.0
  dice_weight: 1.0
train:
  lr: 0.00005
"""


def test_yaml_builds_reference_model_and_loss(tmp_path):
    p = tmp_path / "cfg.yaml"
    p.write_text(YAML)
    model, crit = build_from_config(str(p))
    assert isinstance(model, AttentionUNet) and model.hip_precision == "bf16"
    assert isinstance(crit, DiceBCELoss)
    torch.manual_seed(0)
    ref = AttentionUNet(1, 2, bilinear=True, base_features=64)
    assert list(model.state_dict()) == list(ref.state_dict())


def test_unet_deep_supervision_and_defaults():
    cfg = {"model": {"type": "unet", "n_channels": 3, "n_classes": 2, "base_features": 16},
           "loss": {"type": "dice"}}
    m = create_model(cfg)
    assert isinstance(m, UNet) and not isinstance(m, AttentionUNet) and m.hip_precision == "fp32"
    assert isinstance(create_criterion(cfg), DiceLoss)
    cfg = {"model": {"type": "attention", "n_channels": 1, "n_classes": 2, "base_features": 8,
                     "deep_supervision": True}, "loss": {"type": "dice_bce", "ds_weights": [1.0, 0.5, 0.25, 0.1]}}
    m, c = build_from_config(cfg)
    assert m.deep_supervision
    assert isinstance(c, DeepSupervisionLoss) and c.weights == [1.0, 0.5, 0.25, 0.1]


@pytest.mark.parametrize("key,val", [("backend", "cuda"), ("precision", "int8")])
def test_bad_backend_or_precision_raises(key, val):
    cfg = {"model": {"type": "unet", "n_channels": 1, "n_classes": 2, key: val}, "loss": {"type": "dice"}}
    with pytest.raises(ValueError):
        create_model(cfg)
