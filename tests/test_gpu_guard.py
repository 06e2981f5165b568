"""Bounds-checked debug mode (UNET_GUARD=1, csrc/guard_alloc.cpp + unet/_hip/lib.py): guard bands around
every device allocation, checked after every library call.  Runs tools/guard_sweep.py in a fresh process (the
guard allocator must replace torch's before the first CUDA allocation): its self-test (a deliberate 4-byte
overrun of the fill kernel must be caught) and the network forward + loss + backward + eval forward at the
shapes of test_fp16_grad_scaler_steps (incl. the overflowing 2^40 loss scale) with no guard byte touched."""

import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent


def test_guard_sweep_quick():
    env = dict(os.environ, UNET_GUARD="1")
    r = subprocess.run([sys.executable, "-u", str(ROOT / "tools" / "guard_sweep.py"), "quick"], env=env,
                       capture_output=True, text=True, timeout=300)
    print(r.stdout[-4000:], r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "self-test: overrun caught" in r.stdout
    assert "GUARD_SWEEP_OK" in r.stdout
