"""CPU: pin the oracle (oracle/unet_oracle.py) against the golden vectors recorded from the reference.

The oracle is the checker of every GPU parity test, so it must reproduce the reference's outputs,
loss, gradients and BN running-stat updates on the recorded inputs (same ATen ops on the same CPU,
so the agreement is at the ulp level)."""

import pytest
import torch

from oracle import unet_oracle as O


def _params(rec):
    p = {}
    for k, v in rec["init"].items():
        t = v.clone()
        if t.is_floating_point() and not (k.endswith("running_mean") or k.endswith("running_var")):
            t.requires_grad_(True)
        p[k] = t
    return p


def _seeded_params(rec):
    """Models stored without weights: rebuild them with this package's constructors after
    torch.manual_seed(0) (the fixture records the per-tensor sums to prove the init is identical)."""
    from unet.models import AttentionUNet, UNet
    torch.manual_seed(0)
    c = rec["x"].shape[1]
    if rec["kind"] == "unet":
        m = UNet(c, 2, rec["bilinear"], rec["base"])
    else:
        m = AttentionUNet(c, 2, rec["bilinear"], rec["base"], rec["deep_supervision"])
    for k, s in rec["param_sums"].items():
        assert abs(float(m.state_dict()[k].double().sum()) - s) <= 1e-9 * (1 + abs(s)), k
    return O.params_from_module(m)


@pytest.mark.parametrize("name", ["attention_unet_b8", "unet_b8", "attention_unet_b4_ds", "attention_unet_b4_odd",
                                  "unet_b4_transposed", "attention_unet_b4_3ch_transposed"])
def test_oracle_model_matches_reference(golden_models, name):
    rec = golden_models[name]
    p = _params(rec) if "init" in rec else _seeded_params(rec)
    fwd = O.unet_forward if rec["kind"] == "unet" else O.attention_unet_forward
    kw = {} if rec["kind"] == "unet" else {"deep_supervision": rec["deep_supervision"]}
    out = fwd(p, rec["x"], bilinear=rec["bilinear"], training=True, **kw)
    if rec["deep_supervision"]:
        loss = O.deep_supervision_loss(out, rec["t"], O.dice_bce_loss)
    else:
        loss = O.dice_bce_loss(out, rec["t"])
    loss.backward()
    outs = out if isinstance(out, list) else [out]
    for o, r in zip(outs, rec["outputs"]):
        assert torch.allclose(o.detach(), r, atol=1e-6, rtol=1e-5)
    assert abs(float(loss) - float(rec["loss"])) <= 1e-6
    for k, g in rec["grads"].items():
        assert torch.allclose(p[k].grad, g, atol=1e-6, rtol=1e-4), k
    for k, b in rec["buffers_after"].items():
        assert torch.allclose(p[k].float(), b.float(), atol=1e-6, rtol=1e-5), k
    # eval mode with the updated running stats
    with torch.no_grad():
        ev = fwd({k: v.detach() for k, v in p.items()}, rec["x"], bilinear=rec["bilinear"], training=False)
    assert torch.allclose(ev, rec["eval_logits"], atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("name", ["dice_bce", "dice", "balanced_ce", "dice_bce_w", "dice_bce_c3"])
def test_oracle_losses_match_reference(golden_losses, name):
    ref = golden_losses["cases"][name]
    z = (ref["z"] if "z" in ref else golden_losses["z"]).clone().requires_grad_(True)
    t = ref["t"] if "t" in ref else golden_losses["t"]
    fn = {"dice_bce": O.dice_bce_loss, "dice": O.dice_loss, "balanced_ce": O.balanced_ce_loss,
          "dice_bce_w": lambda a, b: O.dice_bce_loss(a, b, 0.7, 1.3, 0.3), "dice_bce_c3": O.dice_bce_loss}[name]
    loss = fn(z, t)
    loss.backward()
    assert abs(float(loss) - float(ref["loss"])) <= 1e-6
    assert torch.allclose(z.grad, ref["grad"], atol=1e-8, rtol=1e-5)


def test_oracle_metrics_match_reference():
    from conftest import load_golden
    rec = load_golden("metrics.pt")
    pred = rec["z"].softmax(1).argmax(1)
    cm = O.confusion_matrix(pred, rec["t"])
    assert torch.equal(cm, rec["confusion"].to(cm.dtype))
