"""Runtime helpers for the HIP path: precision, streams, virtual activations, source descriptors."""

from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import lib as L

# ------------------------------------------------------------------------------------------------
# precision
# ------------------------------------------------------------------------------------------------


@dataclass(frozen=True)
class Precision:
    name: str
    code: int
    torch_dtype: torch.dtype


FP32 = Precision("fp32", L.F32, torch.float32)
BF16 = Precision("bf16", L.BF16, torch.bfloat16)
FP16 = Precision("fp16", L.F16, torch.float16)
_PRECISIONS = {"fp32": FP32, "float32": FP32, "bf16": BF16, "bfloat16": BF16, "fp16": FP16, "float16": FP16,
               "half": FP16}
_default = _PRECISIONS[os.environ.get("UNET_PRECISION", "fp32").lower()]


def set_precision(name: str) -> None:
    """Default operand precision of the HIP kernels ('fp32' = reference numerics, 'bf16', 'fp16')."""
    global _default
    _default = _PRECISIONS[name.lower()]


def get_precision(module: Optional[torch.nn.Module] = None) -> Precision:
    if module is not None:
        p = getattr(module, "hip_precision", None)
        if p is not None:
            return _PRECISIONS[p.lower()] if isinstance(p, str) else p
    return _default


# ------------------------------------------------------------------------------------------------
# device plumbing
# ------------------------------------------------------------------------------------------------

class KernelProbe:
    """Brackets selected kernel launches with HIP events on the launch stream (used by bench.py for
    the live roofline of one kernel symbol).  Disabled unless `enable()` was called."""

    def __init__(self):
        self.target = None
        self.records = []   # (start_event, end_event, algorithmic_flops)
        self.log = None     # when a list: every probed launch appends (kernel name, output mode)

    def enable(self, target):
        """target: a kernel-name prefix, or a tuple of prefixes (a kernel family)"""
        self.target = target
        self.records = []

    def disable(self):
        self.target = None

    def reset(self):
        self.records = []

    def launch(self, name_fn, flops: float, fn, mode: Optional[int] = None):
        if self.log is not None:
            self.log.append((name_fn(), mode))
        if self.target is None or not name_fn().startswith(self.target):
            return fn()
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        r = fn()
        e.record()
        self.records.append((s, e, flops))
        return r

    def summary(self):
        torch.cuda.synchronize()
        t = sum(s.elapsed_time(e) for s, e, _ in self.records) * 1e-3
        f = sum(fl for _, _, fl in self.records)
        n = len(self.records)
        return {"launches": n, "seconds": t, "flops": f, "avg_us": (t / n * 1e6) if n else None,
                "tflops": (f / t / 1e12) if t > 0 else None}


probe = KernelProbe()


def conv_kernel_name(d) -> str:
    """Instantiation unet_conv dispatches this descriptor to (csrc/conv.hip dispatch_conv)."""
    buf = ctypes.create_string_buffer(128)
    L.load().unet_conv_variant(d, buf, 128)
    return buf.value.decode()


def wgrad_kernel_name(wd) -> str:
    """Weight-gradient kernel unet_conv_wgrad dispatches this descriptor to (csrc/wgrad.hip)."""
    buf = ctypes.create_string_buffer(128)
    L.load().unet_wgrad_variant(wd, buf, 128)
    return buf.value.decode()


def require_device(t: torch.Tensor, what: str = "input") -> None:
    if not t.is_cuda:
        raise RuntimeError(
            f"unet HIP path: {what} is on {t.device}; this implementation runs only on a ROCm GPU "
            f"(MI355X). Move the model and inputs to 'cuda'. The CPU restatement in oracle/ is test "
            f"infrastructure, not a fallback.")
    L.load(require_gpu=True)


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def vp(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def f32(*shape, device) -> torch.Tensor:
    return torch.empty(*shape, dtype=torch.float32, device=device)


def up_scale(in_size: int, out_size: int) -> float:
    """fp32 align_corners scale exactly as ATen's area_pixel_compute_scale."""
    if out_size <= 1:
        return 0.0
    return float(np.float32(in_size - 1) / np.float32(out_size - 1))


def pack_weight(w: torch.Tensor, prec: Precision, transpose: bool) -> torch.Tensor:
    cout, cin, k = w.shape[0], w.shape[1], w.shape[2]
    n = L.load().unet_packed_weight_elems(prec.code, cout, cin, k, int(transpose))
    out = torch.empty(n, dtype=prec.torch_dtype, device=w.device)
    wc = w.detach()
    if wc.dtype != torch.float32 or not wc.is_contiguous():
        wc = wc.float().contiguous()
    L.call("unet_pack_weight", prec.code, vp(wc), vp(out), cout, cin, k, int(transpose), stream())
    return out


def pack_many(items, prec: Precision):
    """Pack several OIHW weights (list of (weight, transpose)) with one launch per 64; returns the
    packed tensors in order."""
    lib = L.load()
    outs, jobs, keep = [], [], []
    for w, transpose in items:
        cout, cin, k = w.shape[0], w.shape[1], w.shape[2]
        n = lib.unet_packed_weight_elems(prec.code, cout, cin, k, int(transpose))
        out = torch.empty(n, dtype=prec.torch_dtype, device=w.device)
        wc = w.detach()
        if wc.dtype != torch.float32 or not wc.is_contiguous():
            wc = wc.float().contiguous()
        keep.append(wc)
        j = L.PackJob()
        j.w, j.packed, j.Cout, j.Cin, j.ksize, j.transpose = wc.data_ptr(), out.data_ptr(), cout, cin, k, int(transpose)
        jobs.append(j)
        outs.append(out)
    for i in range(0, len(jobs), L.PACK_MAX_JOBS):
        chunk = jobs[i:i + L.PACK_MAX_JOBS]
        arr = (L.PackJob * len(chunk))(*chunk)
        L.call("unet_pack_weights", prec.code, len(chunk), arr, stream())
    return outs


def fill_zero(t: torch.Tensor) -> None:
    L.call("unet_fill_f32", vp(t), t.numel(), 0.0, stream())


# ------------------------------------------------------------------------------------------------
# virtual activations
# ------------------------------------------------------------------------------------------------


class Act:
    """A stored NHWC tensor plus the per-channel affine (+ReLU) that makes it the reference's
    activation (relu(bn(y)) of a DoubleConv half, or the identity for a materialised input).
    `grad` is the NHWC gradient w.r.t. that activation, accumulated by its consumers: fp32, or bf16
    for a single-consumer activation in bf16 mode (`grad_single`)."""

    __slots__ = ("data", "N", "H", "W", "C", "ab", "relu", "mean", "invstd", "grad", "_grad_init", "keep",
                 "bn_owned", "pool_grad", "batch_stats", "oc_fused", "fin_job")

    def __init__(self, data: torch.Tensor, ab: Optional[torch.Tensor], relu: bool,
                 mean: Optional[torch.Tensor] = None, invstd: Optional[torch.Tensor] = None):
        self.data = data
        self.N, self.H, self.W, self.C = data.shape
        self.ab = ab          # fp32 [2, C] (scale; shift) or None
        self.relu = relu
        self.mean = mean
        self.invstd = invstd
        self.grad = None
        self._grad_init = False
        self.keep = None
        # set by ConvBN.forward: the gradient is consumed by that ConvBN's BatchNorm backward, which can
        # fold a Down block's pooled gradient (pool_grad = (g2, code, ph, pw)) in on the fly
        self.bn_owned = False
        self.pool_grad = None
        self.batch_stats = True   # False: an eval-mode BN (running statistics) produced it
        # set by OutConvStage.backward when OutConv is the only consumer: (dl, w, K, bn partial sums, rows) — the
        # gradient W^T dl is recomputed by the BN-backward apply instead of being stored
        self.oc_fused = None
        # set by ConvBN.forward(defer_fin=True): (unet_bn_finalize_job, its partial sums) until finalize_many runs it
        self.fin_job = None

    @property
    def scale(self):
        return self.ab[0]

    @property
    def shift(self):
        return self.ab[1]

    @property
    def pixels(self) -> int:
        return self.N * self.H * self.W

    # -- gradient buffer management --
    def grad_target(self):
        """(buffer, accumulate) for the next contribution to this activation's gradient."""
        if self.grad is None:
            self.grad = f32(self.N, self.H, self.W, self.C, device=self.data.device)
        acc = self._grad_init
        self._grad_init = True
        return self.grad, int(acc)

    def grad_single(self, dtype: torch.dtype) -> torch.Tensor:
        """Buffer for the one and only contribution to this activation's gradient (stored, not
        accumulated): a DoubleConv's middle activation, whose only consumer is the second conv."""
        assert self.grad is None and not self._grad_init, "activation has another gradient contribution"
        self.grad = torch.empty(self.N, self.H, self.W, self.C, dtype=dtype, device=self.data.device)
        self._grad_init = True
        return self.grad

    def grad_zeroed(self) -> torch.Tensor:
        if self.grad is None:
            self.grad = f32(self.N, self.H, self.W, self.C, device=self.data.device)
        if not self._grad_init:
            fill_zero(self.grad)
            self._grad_init = True
        return self.grad

    def has_grad(self) -> bool:
        return self._grad_init

    # -- source descriptors --
    def _base(self, kind: int) -> L.Src:
        s = L.Src()
        s.kind = kind
        s.C, s.H, s.W = self.C, self.H, self.W
        s.data = self.data.data_ptr()
        if self.ab is not None:
            s.scale = self.ab[0].data_ptr()
            s.shift = self.ab[1].data_ptr()
        s.relu = int(self.relu)
        return s

    def src(self) -> L.Src:
        return self._base(L.SRC_ACT if self.ab is not None else L.SRC_PLAIN)

    def src_pool(self) -> L.Src:
        assert self.ab is not None
        return self._base(L.SRC_POOL_ACT)

    def src_up(self, up_h: int, up_w: int, pad_t: int = 0, pad_l: int = 0) -> L.Src:
        assert self.ab is not None
        s = self._base(L.SRC_UP_ACT)
        s.up_h, s.up_w, s.pad_t, s.pad_l = up_h, up_w, pad_t, pad_l
        s.sh = up_scale(self.H, up_h)
        s.sw = up_scale(self.W, up_w)
        return s

    def src_placed(self, pad_t: int, pad_l: int) -> L.Src:
        """A plain stored map placed at (pad_t, pad_l) inside a larger conv input (F.pad of a
        ConvTranspose2d output, layers.py:98-102)."""
        assert self.ab is None
        s = self._base(L.SRC_UP_PLAIN)
        s.up_h, s.up_w, s.pad_t, s.pad_l = self.H, self.W, pad_t, pad_l
        return s

    def src_gated(self, p: torch.Tensor, psi_ab: torch.Tensor) -> L.Src:
        s = self._base(L.SRC_ACT)
        s.gate_p = p.data_ptr()
        s.gate_ab = psi_ab.data_ptr()
        return s


def identity_ab(C: int, device) -> torch.Tensor:
    ab = torch.empty(2, C, dtype=torch.float32, device=device)
    L.call("unet_fill_f32", vp(ab[0]), C, 1.0, stream())
    L.call("unet_fill_f32", vp(ab[1]), C, 0.0, stream())
    return ab


def act_from_nchw(x: torch.Tensor, prec: Precision) -> Act:
    """Materialise an NCHW fp32 module input as an NHWC operand tensor (identity activation)."""
    N, C, H, W = x.shape
    xc = x.detach()
    if xc.dtype != torch.float32 or not xc.is_contiguous():
        xc = xc.float().contiguous()
    y = torch.empty(N, H, W, C, dtype=prec.torch_dtype, device=x.device)
    L.call("unet_nchw_to_nhwc", prec.code, N, C, H, W, vp(xc), vp(y), stream())
    return Act(y, identity_ab(C, x.device), False)


def nchw_src(x: torch.Tensor) -> L.Src:
    s = L.Src()
    s.kind = L.SRC_NCHW_F32
    s.C, s.H, s.W = x.shape[1], x.shape[2], x.shape[3]
    s.data = x.data_ptr()
    return s


def act_to_nchw(a: Act, prec: Precision) -> torch.Tensor:
    out = torch.empty(a.N, a.C, a.H, a.W, dtype=torch.float32, device=a.data.device)
    sc = vp(a.ab[0]) if a.ab is not None else None
    sf = vp(a.ab[1]) if a.ab is not None else None
    L.call("unet_nhwc_to_nchw", prec.code, a.N, a.C, a.H, a.W, vp(a.data), sc, sf, int(a.relu), vp(out), stream())
    return out


def grad_nchw_to_nhwc(g: torch.Tensor) -> torch.Tensor:
    N, C, H, W = g.shape
    gc = g.float().contiguous()
    out = f32(N, H, W, C, device=g.device)
    L.call("unet_nchw_to_nhwc", L.F32, N, C, H, W, vp(gc), vp(out), stream())
    return out


def grad_nhwc_to_nchw(g: torch.Tensor) -> torch.Tensor:
    N, H, W, C = g.shape
    out = f32(N, C, H, W, device=g.device)
    L.call("unet_nhwc_to_nchw", L.F32, N, C, H, W, vp(g), None, None, 0, vp(out), stream())
    return out
