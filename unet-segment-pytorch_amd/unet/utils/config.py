"""YAML-config front end for the training hot path: the model / loss construction block of the reference's
scripts/train.py (:306-342, reading configs/lung_tumor.yaml's `model:` and `loss:` sections) as library
functions, plus the two keys this backend adds.

Keys read (reference meaning unchanged):
  model.type (unet | attention_unet | attention), model.n_channels, model.n_classes, model.bilinear,
  model.base_features, model.deep_supervision;
  loss.type, loss.ce_weight, loss.dice_weight, loss.class_weights, loss.balanced_class_weight,
  loss.ds_weights (deep supervision only).
Keys added:
  model.backend   — "hip" (the only backend of this package; anything else is an error, not a silent
                    fallback to another implementation);
  model.precision — "fp32" (default: the reference's fp32 arithmetic), "bf16" or "fp16" (16-bit operands,
                    fp32 accumulation; fp16 is meant to be used with torch.amp.GradScaler, as for C5).
Only yaml.safe_load is used to read a file."""

from typing import Any, Dict, Tuple, Union

import torch.nn as nn

_PRECISIONS = ("fp32", "bf16", "fp16")


def load_config(path: str) -> Dict[str, Any]:
    """scripts/train.py load_config: a YAML file -> dict (safe loader only)"""
    import yaml
    with open(path) as f:
        return yaml.safe_load(f)


def _section(config: Dict[str, Any], name: str) -> Dict[str, Any]:
    sec = config.get(name)
    if not isinstance(sec, dict):
        raise KeyError(f"config has no '{name}:' section")
    return sec


def create_model(config: Dict[str, Any]) -> nn.Module:
    """scripts/train.py:306-323: UNet or AttentionUNet from `model:`; sets the HIP operand precision"""
    from unet.models import AttentionUNet, UNet
    mc = _section(config, "model")
    backend = str(mc.get("backend", "hip")).lower()
    if backend != "hip":
        raise ValueError(f"model.backend '{backend}' is not provided by this package (only 'hip')")
    prec = str(mc.get("precision", "fp32")).lower()
    if prec not in _PRECISIONS:
        raise ValueError(f"model.precision must be one of {_PRECISIONS}, got '{prec}'")
    kw = dict(n_channels=mc["n_channels"], n_classes=mc["n_classes"], bilinear=mc.get("bilinear", True),
              base_features=mc.get("base_features", 64))
    kind = str(mc.get("type", "unet")).lower()
    if kind in ("attention_unet", "attention"):
        model = AttentionUNet(**kw, deep_supervision=mc.get("deep_supervision", False))
    else:
        model = UNet(**kw)
    model.hip_precision = prec
    return model


def create_criterion(config: Dict[str, Any]) -> nn.Module:
    """scripts/train.py:325-342: create_loss_function from `loss:`, wrapped in DeepSupervisionLoss when
    model.deep_supervision is set (default weights [1.0, 0.4, 0.2, 0.1])"""
    from unet.utils.loss import DeepSupervisionLoss, create_loss_function
    lc = _section(config, "loss")
    base = create_loss_function(loss_type=lc["type"], ce_weight=lc.get("ce_weight", 1.0),
                                dice_weight=lc.get("dice_weight", 1.0), class_weights=lc.get("class_weights"),
                                balanced_class_weight=lc.get("balanced_class_weight", 0.5))
    if config.get("model", {}).get("deep_supervision", False):
        return DeepSupervisionLoss(base, weights=lc.get("ds_weights", [1.0, 0.4, 0.2, 0.1]))
    return base


def build_from_config(config: Union[str, Dict[str, Any]]) -> Tuple[nn.Module, nn.Module]:
    """(model, criterion) from a config dict or a YAML path; the caller moves the model to the device and
    builds the optimizer from `train:` as scripts/train.py:345-349 does"""
    if isinstance(config, str):
        config = load_config(config)
    return create_model(config), create_criterion(config)
