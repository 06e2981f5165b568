"""Shared helpers for the GPU parity tests (HIP path vs golden fixtures / oracle)."""

from __future__ import annotations

import torch


def rel_err(a: torch.Tensor, b: torch.Tensor) -> float:
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def max_abs(a: torch.Tensor, b: torch.Tensor) -> float:
    return float((a.detach().double().cpu() - b.detach().double().cpu()).abs().max())


def build_model(rec: dict, device="cuda"):
    from unet.models import AttentionUNet, UNet
    kind = rec["kind"]
    c = rec["x"].shape[1]
    torch.manual_seed(0)   # the fixtures were recorded from models built right after manual_seed(0)
    if kind == "unet":
        m = UNet(n_channels=c, n_classes=2, bilinear=rec["bilinear"], base_features=rec["base"])
    else:
        m = AttentionUNet(n_channels=c, n_classes=2, bilinear=rec["bilinear"], base_features=rec["base"],
                          deep_supervision=rec["deep_supervision"])
    if "init" in rec:
        m.load_state_dict(rec["init"])
    return m.to(device)


def grad_report(model, ref_grads: dict):
    """max relative error (per tensor, normalised by the tensor's max |ref|) over all param grads"""
    worst = (0.0, "")
    named = dict(model.named_parameters())
    for k, g in ref_grads.items():
        p = named[k]
        assert p.grad is not None, f"no grad for {k}"
        scale = float(g.abs().max()) + 1e-12
        e = max_abs(p.grad, g) / scale
        if e > worst[0]:
            worst = (e, k)
    return worst
