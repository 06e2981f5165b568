"""Bounds-checked sweep of the HIP path (UNET_GUARD=1 debug mode, csrc/guard_alloc.cpp): every device
allocation carries 4 KiB guard bands and every library call is followed by a device sync and a check of all
bands, so an out-of-bounds write raises GuardViolation naming the call.  Runs the network forward + loss +
backward (and the eval forward) over the shapes and modes the GPU suite uses, including the ones of
tests/test_gpu_parity.py::test_fp16_grad_scaler_steps (AttentionUNet 3-ch, base 16, 2 x 128^2, fp16, a 2^40
loss scale that saturates the fp16 gradients).

Usage: UNET_GUARD=1 python tools/guard_sweep.py [quick]   (must start in a fresh process: the guard
allocator replaces torch's before the first CUDA allocation)"""

import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "unet-segment-pytorch_amd"))

if os.environ.get("UNET_GUARD", "") in ("", "0"):
    raise SystemExit("set UNET_GUARD=1")

import torch  # noqa: E402

from unet._hip import lib as L  # noqa: E402  (installs the guard allocator)


def self_test():
    """The guard must catch a 4-byte overrun of the library's own fill kernel."""
    t = torch.empty(1000, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    L.call("unet_fill_f32", t.data_ptr(), 1000, 1.0, s)
    try:
        L.call("unet_fill_f32", t.data_ptr(), 1001, 1.0, s)
    except L.GuardViolation as e:
        print(f"self-test: overrun caught ({e})", flush=True)
        return
    raise SystemExit("self-test FAILED: a 4-byte overrun was not caught")


def run(kind, prec, cin, base, n, h, w, bilinear=True, ds=False, scale=None, eval_too=True):
    from unet.models import AttentionUNet, UNet
    from unet.utils.loss import DeepSupervisionLoss, DiceBCELoss
    torch.manual_seed(0)
    if kind == "unet":
        m = UNet(cin, 2, bilinear=bilinear, base_features=base)
    else:
        m = AttentionUNet(cin, 2, bilinear=bilinear, base_features=base, deep_supervision=ds)
    m = m.cuda().train()
    m.hip_precision = prec
    g = torch.Generator().manual_seed(1)
    x = (torch.rand(n, cin, h, w, generator=g) * 2 - 1).cuda()
    t = (torch.rand(n, h, w, generator=g) < 0.1).long().cuda()
    crit = DiceBCELoss()
    if ds:
        crit = DeepSupervisionLoss(crit)
    loss = crit(m(x), t)
    (loss * scale if scale else loss).backward()
    if eval_too:
        m.eval()
        with torch.no_grad():
            m(x)
    L.guard_check("end of case")
    finite = all(bool(torch.isfinite(p.grad).all()) for p in m.parameters() if p.grad is not None)
    return float(loss.detach()), finite


CASES = [
    # test_fp16_grad_scaler_steps: overflowing scale, then sane scales
    ("attention", "fp16", 3, 16, 2, 128, 128, True, False, 2.0 ** 40),
    ("attention", "fp16", 3, 16, 2, 128, 128, True, False, 1024.0),
    ("attention", "fp32", 3, 16, 2, 128, 128, True, False, None),
    # golden-fixture shapes (base 8 / 4, odd sizes, transposed up, deep supervision)
    ("attention", "fp32", 1, 8, 2, 64, 64, True, False, None),
    ("attention", "fp32", 1, 4, 2, 64, 64, True, True, None),
    ("attention", "fp32", 1, 4, 2, 66, 66, True, False, None),
    ("unet", "fp32", 1, 4, 2, 64, 64, False, False, None),
    ("attention", "fp32", 3, 4, 2, 64, 64, False, False, None),
    # 16-bit modes on odd / small maps
    ("attention", "bf16", 1, 16, 2, 98, 98, True, False, None),
    ("attention", "fp16", 1, 16, 2, 98, 98, True, False, None),
    ("unet", "bf16", 1, 8, 2, 128, 128, False, False, None),
    ("attention", "bf16", 3, 16, 1, 96, 80, True, True, None),
    # base 64 at the small end of the bench kernels' shapes (conv5 / wgrad5 / pw / gate dispatch)
    ("attention", "bf16", 1, 64, 2, 128, 128, True, False, None),
    ("attention", "fp16", 3, 64, 1, 128, 128, True, False, 2.0 ** 40),
    ("unet", "bf16", 1, 64, 1, 128, 128, False, False, None),
]


def main():
    quick = len(sys.argv) > 1 and sys.argv[1] == "quick"
    self_test()
    for c in (CASES[:3] if quick else CASES):
        t0 = time.time()
        loss, finite = run(*c)
        print(f"clean: {c} loss {loss:.5f} finite grads {finite} ({time.time() - t0:.1f} s, "
              f"{L._guard.unet_guard_allocations()} allocations so far)", flush=True)
    print("GUARD_SWEEP_OK", flush=True)


if __name__ == "__main__":
    main()
