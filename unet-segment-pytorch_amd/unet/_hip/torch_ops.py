"""The TORCH_LIBRARY(unet_hip) operators (csrc/torch_ops.cpp): the fused loss and the confusion matrix of
libunet_hip.so as `torch.ops.unet_hip.*`, for callers that want dispatcher operators (TorchScript, torch.library
tooling) rather than the package's modules.  Same kernels, same results as unet.utils.loss / unet.utils.metrics
(tests/test_gpu_torch_ops.py); no CPU kernels are registered, so a CPU tensor raises."""

from pathlib import Path

import torch

from . import lib as L

_PATH = Path(__file__).resolve().parent / "libunet_torch_ops.so"
_loaded = False


def library_path() -> Path:
    return _PATH


def load():
    """Load (once) the operator library and return the `torch.ops.unet_hip` namespace.  Raises if missing."""
    global _loaded
    if not _loaded:
        if not _PATH.exists():
            raise L.HipLibraryError(f"{_PATH} not built; run `make -C unet-segment-pytorch_amd/csrc` "
                                    "(or __graft_entry__.build()).")
        L.load()                       # the ctypes library first: the operators resolve to this same copy
        torch.ops.load_library(str(_PATH))
        if torch.ops.unet_hip.abi_version() != L.ABI_VERSION:
            raise L.HipLibraryError(f"{_PATH} was built against another ABI; rebuild it")
        _loaded = True
    return torch.ops.unet_hip
