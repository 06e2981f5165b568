import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "unet-segment-pytorch_amd"
for p in (str(PKG), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running")


# Run last: the long trajectory tests (200-epoch chaotic overfit protocol).  Under `-x`, a failure there must
# not keep the deterministic golden-fixture parity tests from running.
_LAST = ("test_gpu_overfit.py",)


def pytest_collection_modifyitems(session, config, items):
    items.sort(key=lambda it: any(it.nodeid.split("::")[0].endswith(f) for f in _LAST))


def load_golden(name: str):
    import torch
    return torch.load(GOLDEN / name, weights_only=True)


@pytest.fixture(scope="session")
def golden_models():
    return load_golden("models.pt")


@pytest.fixture(scope="session")
def golden_modules():
    return load_golden("modules.pt")


@pytest.fixture(scope="session")
def golden_losses():
    return load_golden("losses.pt")


@pytest.fixture(autouse=True)
def _guard_check_after_test():
    """UNET_GUARD=1 runs (bounds-checking debug mode, csrc/guard_alloc.cpp): after each test, check the guard bands
    of every live device allocation once more — this also covers the torch ops that ran after the test's last
    HIP-library call (the library checks around its own calls)."""
    yield
    if os.environ.get("UNET_GUARD", "") not in ("", "0"):
        from unet._hip import lib as L
        L.guard_check("end of test (torch ops after the last library call)")
