"""ctypes binding of the C-ABI in include/unet_hip.h (libunet_hip.so, built for gfx950).

This is the ONLY way the package reaches the device: there is no CPU fallback.  If the library is
missing or no ROCm GPU is visible, every compute entry point raises.
"""

from __future__ import annotations

import ctypes
import sys
import os
from pathlib import Path

import torch  # noqa: F401  (import first: libamdhip64.so.7 must resolve to the runtime torch loaded)

_LIB_PATH = Path(os.environ.get("UNET_HIP_LIB", Path(__file__).resolve().parent / "libunet_hip.so"))

F32, BF16, F16 = 0, 1, 2
SRC_PLAIN, SRC_ACT, SRC_POOL_ACT, SRC_UP_ACT, SRC_NCHW_F32, SRC_UP_PLAIN = range(6)
OUT_Y, OUT_F32, OUT_POOL_BWD, OUT_SHUFFLE2, OUT_F32_GATED = range(5)

c_int, c_ll, c_float, c_vp, c_size = ctypes.c_int, ctypes.c_longlong, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t


class Src(ctypes.Structure):
    _fields_ = [("kind", c_int), ("C", c_int), ("H", c_int), ("W", c_int), ("data", c_vp), ("scale", c_vp),
                ("shift", c_vp), ("relu", c_int), ("up_h", c_int), ("up_w", c_int), ("pad_t", c_int),
                ("pad_l", c_int), ("sh", c_float), ("sw", c_float), ("gate_p", c_vp), ("gate_ab", c_vp)]


class ConvDesc(ctypes.Structure):
    _fields_ = [("dtype", c_int), ("N", c_int), ("H", c_int), ("W", c_int), ("Cin", c_int), ("Cout", c_int),
                ("ksize", c_int), ("nsrc", c_int), ("src", Src * 2), ("weight", c_vp), ("out_mode", c_int),
                ("out", c_vp), ("out2", c_vp), ("split", c_int), ("accum", c_int), ("accum2", c_int),
                ("stats", c_vp), ("pool_src", Src), ("bias", c_vp), ("pool_code", c_vp),
                ("bnb_y", c_vp), ("bnb_scale", c_vp), ("bnb_shift", c_vp), ("bnb_relu", c_int), ("bnb_mean", c_vp),
                ("bnb_invstd", c_vp), ("bnb_stats", c_vp), ("act_out", c_vp), ("workspace", c_vp)]


class PackJob(ctypes.Structure):
    _fields_ = [("w", c_vp), ("packed", c_vp), ("Cout", c_int), ("Cin", c_int), ("ksize", c_int), ("transpose", c_int)]


PACK_MAX_JOBS = 64


class BnFinJob(ctypes.Structure):      # unet_bn_finalize_job
    _fields_ = [("stats", c_vp), ("rows", c_int), ("C", c_int), ("count", c_ll), ("gamma", c_vp), ("beta", c_vp),
                ("running_mean", c_vp), ("running_var", c_vp), ("num_batches_tracked", c_vp), ("momentum", c_float),
                ("eps", c_float), ("mean", c_vp), ("invstd", c_vp), ("scale", c_vp), ("shift", c_vp)]


class BnBwdFinJob(ctypes.Structure):   # unet_bn_bwd_finalize_job
    _fields_ = [("sum_g", c_vp), ("sum_gx", c_vp), ("rows", c_int), ("C", c_int), ("count", c_ll), ("gamma", c_vp),
                ("mean", c_vp), ("invstd", c_vp), ("dgamma", c_vp), ("dbeta", c_vp), ("accum", c_int), ("coef", c_vp)]


BN_MULTI_MAX = 4


class WgradDesc(ctypes.Structure):
    _fields_ = [("dtype", c_int), ("N", c_int), ("H", c_int), ("W", c_int), ("Cin", c_int), ("Cout", c_int),
                ("ksize", c_int), ("nsrc", c_int), ("src", Src * 2), ("dy", c_vp), ("dw", c_vp), ("accum", c_int),
                ("workspace", c_vp)]


# name -> (restype, argtypes); mirrors include/unet_hip.h
_SIGS = {
    "unet_last_error": (ctypes.c_char_p, []),
    "unet_version": (c_int, []),
    "unet_conv_mtiles": (c_int, [c_int, c_int, c_int]),
    "unet_conv_stats_rows": (c_int, [ctypes.POINTER(ConvDesc)]),
    "unet_conv_variant": (c_int, [ctypes.POINTER(ConvDesc), ctypes.c_char_p, c_int]),
    "unet_wgrad_variant": (c_int, [ctypes.POINTER(WgradDesc), ctypes.c_char_p, c_int]),
    "unet_conv_act_out_ok": (c_int, [ctypes.POINTER(ConvDesc)]),
    "unet_conv_workspace": (c_size, [ctypes.POINTER(ConvDesc)]),
    "unet_pack_weight": (c_int, [c_int, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp]),
    "unet_packed_weight_elems": (c_int, [c_int, c_int, c_int, c_int, c_int]),
    "unet_pack_weights": (c_int, [c_int, c_int, ctypes.POINTER(PackJob), c_vp]),
    "unet_conv": (c_int, [ctypes.POINTER(ConvDesc), c_vp]),
    "unet_wgrad_workspace": (c_size, [ctypes.POINTER(WgradDesc)]),
    "unet_conv_wgrad": (c_int, [ctypes.POINTER(WgradDesc), c_vp]),
    "unet_bn_finalize": (c_int, [c_vp, c_int, c_int, c_ll, c_vp, c_vp, c_vp, c_vp, c_vp, c_float, c_float, c_vp, c_vp,
                                 c_vp, c_vp, c_vp]),
    "unet_bn_eval_affine": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_float, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "unet_bn_bwd_reduce_rows": (c_int, [c_ll, c_int]),
    "unet_bn_bwd_reduce": (c_int, [c_int, c_int, c_ll, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp]),
    "unet_bn_bwd_finalize": (c_int, [c_vp, c_vp, c_int, c_int, c_ll, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp]),
    "unet_bn_bwd_apply": (c_int, [c_int, c_int, c_ll, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp]),
    "unet_bn_bwd_reduce_pool": (c_int, [c_int, c_ll, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp,
                                        c_vp, c_int, c_vp, c_vp, c_vp, c_vp]),
    "unet_bn_bwd_apply_pool": (c_int, [c_int, c_ll, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp,
                                       c_vp, c_int, c_vp, c_vp, c_vp]),
    "unet_colsum": (c_int, [c_vp, c_int, c_int, c_vp, c_int, c_vp]),
    "unet_bn_finalize_multi": (c_int, [c_int, ctypes.POINTER(BnFinJob), c_vp]),
    "unet_bn_bwd_finalize_multi": (c_int, [c_int, ctypes.POINTER(BnBwdFinJob), c_vp]),
    "unet_gate_psi_rows": (c_int, [c_ll]),
    "unet_gate_psi": (c_int, [c_int, c_ll, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "unet_gate_psi_eval": (c_int, [c_int, c_ll, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp,
                                   c_vp, c_vp, c_vp, c_vp]),
    "unet_gate_bwd1": (c_int, [c_int, c_ll, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
                               c_vp, c_vp, c_vp]),
    "unet_gate_bwd2_rows": (c_int, [c_ll, c_int]),
    "unet_gate_bwd2": (c_int, [c_int, c_ll, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                               c_vp, c_vp, c_vp]),
    "unet_gate_bwd3": (c_int, [c_int, c_ll, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                               c_vp, c_vp]),
    "unet_upsample_bwd": (c_int, [c_ll, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_float,
                                  c_vp, c_vp, c_int, c_vp]),
    "unet_resize_nchw": (c_int, [c_ll, c_int, c_int, c_int, c_int, c_float, c_float, c_vp, c_vp, c_vp]),
    "unet_resize_nchw_bwd": (c_int, [c_ll, c_int, c_int, c_int, c_int, c_float, c_float, c_vp, c_vp, c_int, c_vp]),
    "unet_convt_bwd_rows": (c_int, [c_ll]),
    "unet_convt_bwd_prep": (c_int, [c_int, c_ll, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp,
                                    c_vp]),
    "unet_outconv_rows": (c_int, [c_ll]),
    "unet_outconv_fwd": (c_int, [c_int, c_ll, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp,
                                 c_vp]),
    "unet_outconv_bwd": (c_int, [c_int, c_ll, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp,
                                 c_int, c_vp, c_vp]),
    "unet_outconv_bwd_bn": (c_int, [c_int, c_ll, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp,
                                    c_vp, c_vp, c_vp, c_vp]),
    "unet_bn_bwd_apply_oc": (c_int, [c_int, c_ll, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp,
                                     c_vp, c_vp]),
    "unet_outconv_bwd_finalize": (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_int, c_vp]),
    "unet_nchw_to_nhwc": (c_int, [c_int, c_ll, c_int, c_int, c_int, c_vp, c_vp, c_vp]),
    "unet_nhwc_to_nchw": (c_int, [c_int, c_ll, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp]),
    "unet_gated_to_nchw": (c_int, [c_int, c_ll, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp]),
    "unet_fill_f32": (c_int, [c_vp, c_ll, c_float, c_vp]),
    "unet_materialize": (c_int, [c_int, ctypes.POINTER(Src), c_ll, c_int, c_int, c_vp, c_vp]),
    "unet_materialize_pool": (c_int, [c_int, ctypes.POINTER(Src), c_ll, c_int, c_int, c_vp, c_vp, c_vp]),
    "unet_confusion_matrix": (c_int, [c_ll, c_int, c_int, c_ll, c_vp, c_vp, c_vp, c_ll, c_int, c_vp, c_vp]),
    "unet_confusion_matrix_ext": (c_int, [c_ll, c_int, c_int, c_ll, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "unet_loss_rows": (c_int, [c_ll]),
    "unet_loss_reduce": (c_int, [c_ll, c_int, c_ll, c_vp, c_vp, c_vp, c_vp]),
    "unet_loss_finalize": (c_int, [c_vp, c_int, c_ll, c_int, c_float, c_float, c_float, c_float, c_float, c_int, c_int,
                                   c_vp, c_vp, c_vp]),
    "unet_loss_grad": (c_int, [c_ll, c_int, c_ll, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp]),
    "unet_resample_u8": (c_int, [c_int, c_ll, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_vp]),
    "unet_slice_finish": (c_int, [c_ll, c_int, c_int, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_float,
                                  c_float, c_vp, c_vp, c_vp]),
    "unet_postprocess_mask": (c_int, [c_ll, c_int, c_int, c_int, c_vp, c_int, c_float, c_int, c_int, c_vp, c_vp, c_vp,
                                      c_vp]),
    "unet_loss_reduce_multi": (c_int, [c_int, c_ll, c_int, c_ll, ctypes.POINTER(c_vp), c_vp, c_vp, c_vp]),
    "unet_loss_finalize_multi": (c_int, [c_vp, c_int, c_int, ctypes.POINTER(c_float), c_ll, c_int, c_float, c_float,
                                         c_float, c_float, c_float, c_int, c_int, c_vp, c_vp, c_vp]),
    "unet_loss_grad_multi": (c_int, [c_int, c_ll, c_int, c_ll, ctypes.POINTER(c_vp), c_vp, c_vp, c_vp, c_int, c_int,
                                     ctypes.POINTER(c_vp), c_vp]),
}

_lib = None
ABI_VERSION = 110   # include/unet_hip.h UNET_ABI_VERSION

# UNET_GUARD=1: bounds-checking debug mode (csrc/guard_alloc.cpp).  Every device allocation of the process
# gets guard bands and every library call is bracketed by a device sync + a check of all bands, so an
# out-of-bounds write is named at the call that made it (or "before" it: a torch op in between).  Must be
# set before the first CUDA allocation of the process; slow (no caching allocator); debug runs only.
_GUARD = os.environ.get("UNET_GUARD", "") not in ("", "0")
_guard = None
# queries that launch nothing
_NO_LAUNCH = {"unet_last_error", "unet_version", "unet_conv_mtiles", "unet_conv_stats_rows", "unet_conv_variant",
              "unet_wgrad_variant", "unet_conv_act_out_ok", "unet_conv_workspace", "unet_packed_weight_elems", "unet_wgrad_workspace",
              "unet_bn_bwd_reduce_rows", "unet_gate_psi_rows", "unet_gate_bwd2_rows", "unet_convt_bwd_rows",
              "unet_outconv_rows", "unet_loss_rows"}


class HipLibraryError(RuntimeError):
    pass


class GuardViolation(RuntimeError):
    pass


def _install_guard():
    global _guard
    if _guard is None:
        path = _LIB_PATH.parent / "libunet_guard.so"
        alloc = torch.cuda.memory.CUDAPluggableAllocator(str(path), "unet_guard_malloc", "unet_guard_free")
        torch.cuda.memory.change_current_allocator(alloc)
        g = ctypes.CDLL(str(path))
        g.unet_guard_check.restype = c_int
        g.unet_guard_check.argtypes = [ctypes.c_char_p, c_int]
        g.unet_guard_allocations.restype = ctypes.c_long
        _guard = g
    return _guard


def guard_check(where: str):
    """UNET_GUARD mode: raise GuardViolation if any allocation's guard band was written."""
    buf = ctypes.create_string_buffer(400)
    if _guard is not None and _guard.unet_guard_check(buf, 400):
        raise GuardViolation(f"{where}: {buf.value.decode()}")


class _GuardedLib:
    def __init__(self, lib):
        self._lib = lib

    def __getattr__(self, name):
        fn = getattr(self._lib, name)
        if name in _NO_LAUNCH:
            return fn

        def wrapped(*args):
            guard_check(f"before {name} (a torch op since the previous library call)")
            rc = fn(*args)
            guard_check(name)
            _GuardedLib.calls += 1
            if _GuardedLib.calls % 500 == 0:   # a heartbeat: a guarded run is slow (a sync + a band scan per call)
                print(f"[guard] {_GuardedLib.calls} library calls checked, last {name}", file=sys.__stderr__, flush=True)
            return rc
        return wrapped

    calls = 0


if _GUARD:
    _install_guard()


def library_path() -> Path:
    return _LIB_PATH


def load(require_gpu: bool = False):
    """Load (once) and return the ctypes library.  Raises if it is missing."""
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            raise HipLibraryError(
                f"unet HIP library not found at {_LIB_PATH}; build it with "
                f"`make -C unet-segment-pytorch_amd/csrc` (or __graft_entry__.build()). There is no CPU fallback.")
        lib = ctypes.CDLL(str(_LIB_PATH))
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.unet_version() != ABI_VERSION:   # descriptor layouts below are this version's
            raise HipLibraryError(f"{_LIB_PATH} has ABI {lib.unet_version()}, this package binds {ABI_VERSION}: "
                                  "rebuild it (make -C unet-segment-pytorch_amd/csrc)")
        _lib = _GuardedLib(lib) if _GUARD else lib
    if require_gpu and not torch.cuda.is_available():
        raise HipLibraryError("unet HIP path needs a ROCm GPU (MI355X / gfx950); none is visible.")
    return _lib


def exported_symbols():
    return list(_SIGS.keys())


def check(rc: int, what: str):
    if rc != 0:
        msg = _lib.unet_last_error().decode() if _lib is not None else ""
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def attach_workspace(d, device) -> "torch.Tensor | None":
    """Give a conv descriptor the scratch of its split-K form (unet_conv_workspace bytes) on `device` — the
    device of the descriptor's tensors — and return it (the caller keeps it alive while d is launched).  Set
    it after the descriptor's other fields and BEFORE asking unet_conv_stats_rows: the row count of the split
    form differs.  Without a workspace unet_conv runs the unsplit form."""
    n = load().unet_conv_workspace(d)
    if not n:
        return None
    ws = torch.empty(n, dtype=torch.uint8, device=device)
    d.workspace = ws.data_ptr()
    return ws


def call(name: str, *args):
    rc = getattr(load(), name)(*args)
    check(rc, name)
    return rc
