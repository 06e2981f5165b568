"""GPU diagnostic: prints HIP-vs-golden errors for every fixture and times a full-size step.
Not a test (no asserts); run:  python tests/gpu_diag.py [--full]"""

import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "unet-segment-pytorch_amd"))

from conftest import load_golden  # noqa: E402
from hip_helpers import build_model, grad_report, max_abs, rel_err  # noqa: E402
from test_gpu_parity import MODULE_CASES, _module_for  # noqa: E402


def modules():
    gm = load_golden("modules.pt")
    for name in MODULE_CASES:
        rec = gm[name]
        try:
            m = _module_for(name, rec)
            m.hip_precision = "fp32"
            ins = [i.cuda().requires_grad_(True) for i in rec["inputs"]]
            y = m(*ins)
            (y * rec["gout"].cuda()).sum().backward()
            torch.cuda.synchronize()
            gi = [max_abs(i.grad, r) for i, r in zip(ins, rec["grad_inputs"])]
            e, k = grad_report(m, rec["grads"])
            print(f"[module {name}] out {max_abs(y, rec['out']):.2e} (max {float(rec['out'].abs().max()):.2f}) "
                  f"din {['%.2e' % v for v in gi]} dparam {e:.2e} ({k})", flush=True)
        except Exception as ex:  # noqa: BLE001
            print(f"[module {name}] ERROR {type(ex).__name__}: {ex}", flush=True)


def models():
    from unet.utils.loss import DeepSupervisionLoss, DiceBCELoss
    gm = load_golden("models.pt")
    for name in ["attention_unet_b8", "unet_b8", "attention_unet_b4_ds", "attention_unet_b4_odd"]:
        rec = gm[name]
        for prec in ("fp32", "bf16"):
            try:
                m = build_model(rec)
                m.hip_precision = prec
                m.train()
                out = m(rec["x"].cuda())
                crit = DiceBCELoss()
                if rec["deep_supervision"]:
                    crit = DeepSupervisionLoss(crit)
                loss = crit(out, rec["t"].cuda())
                loss.backward()
                torch.cuda.synchronize()
                outs = out if isinstance(out, list) else [out]
                oe = [max_abs(o, r) for o, r in zip(outs, rec["outputs"])]
                re_ = [rel_err(o, r) for o, r in zip(outs, rec["outputs"])]
                e, k = grad_report(m, rec["grads"])
                print(f"[model {name} {prec}] logits maxabs {['%.2e' % v for v in oe]} rel {['%.1e' % v for v in re_]} "
                      f"loss {float(loss):.6f} vs {float(rec['loss']):.6f} dparam {e:.2e} ({k})", flush=True)
            except Exception as ex:  # noqa: BLE001
                import traceback
                traceback.print_exc()
                print(f"[model {name} {prec}] ERROR {type(ex).__name__}: {ex}", flush=True)


def full(prec="bf16", bs=4, iters=5, attention=True):
    from unet.models import AttentionUNet, UNet
    from unet.utils.loss import DiceBCELoss
    torch.manual_seed(0)
    m = (AttentionUNet(1, 2) if attention else UNet(1, 2)).cuda().train()
    m.hip_precision = prec
    x = torch.rand(bs, 1, 512, 512, device="cuda") * 2 - 1
    t = (torch.rand(bs, 512, 512, device="cuda") < 0.01).long()
    crit = DiceBCELoss()
    for i in range(2):
        loss = crit(m(x), t)
        loss.backward()
    torch.cuda.synchronize()
    t0 = time.time()
    for i in range(iters):
        loss = crit(m(x), t)
        loss.backward()
    torch.cuda.synchronize()
    dt = (time.time() - t0) / iters
    print(f"[full {'attn' if attention else 'unet'} {prec} bs{bs}] {dt*1e3:.1f} ms/step  {bs/dt:.1f} img/s  loss {float(loss):.4f}",
          flush=True)


def autocast_ref():
    """Inherent bf16 error: the oracle (ATen) under torch.autocast(bf16) on the GPU vs the fp32 golden."""
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    from oracle import unet_oracle as O
    gm = load_golden("models.pt")
    for name in ["attention_unet_b8", "unet_b8"]:
        rec = gm[name]
        p = {k: (v.cuda().requires_grad_(True) if v.is_floating_point() and "running" not in k else v.cuda())
             for k, v in rec["init"].items()}
        fwd = O.unet_forward if rec["kind"] == "unet" else O.attention_unet_forward
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = fwd(p, rec["x"].cuda(), training=True)
        loss = O.dice_bce_loss(out.float(), rec["t"].cuda())
        loss.backward()
        worst = max((float((p[k].grad.cpu() - g).abs().max()) / (float(g.abs().max()) + 1e-12), k)
                    for k, g in rec["grads"].items())
        print(f"[autocast-bf16 {name}] logits rel {rel_err(out.float(), rec['outputs'][0]):.1e} maxabs "
              f"{max_abs(out.float(), rec['outputs'][0]):.2e} loss {float(loss):.6f} dparam {worst[0]:.2e} ({worst[1]})",
              flush=True)


if __name__ == "__main__":
    print(torch.cuda.get_device_name(0), flush=True)
    modules()
    models()
    autocast_ref()
    if "--full" in sys.argv:
        full("bf16")
        full("fp32", iters=2)
