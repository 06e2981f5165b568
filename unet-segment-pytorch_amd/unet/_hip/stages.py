"""Stage executor: the reference's modules re-expressed as HIP launches on virtual activations.

Each stage mirrors one reference module (file:line in the docstrings) and owns the kernel launches
for its forward and backward.  The BN-apply + ReLU of the previous DoubleConv, the zero pad, the
channel concat and the attention multiply are not launched at all: they are folded into the
consuming conv's tile loader through `unet_src` descriptors.  Two derived maps are written once per
step instead (measured faster than a 4-corner gather inside the MFMA kernels): the 2x2 max-pooled
input of each Down block (`unet_materialize_pool`, with 1-byte argmax codes for the backward) and
the bilinear x2 upsample of each Up block's decoder input (`unet_materialize`).
"""

from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch

from . import lib as L
from .runtime import (Act, Precision, conv_kernel_name, f32, pack_many, pack_weight, probe, stream, up_scale, vp,
                      wgrad_kernel_name)


def _conv_desc(prec: Precision, N: int, H: int, W: int, cin: int, cout: int, k: int, srcs: List[L.Src],
               weight: torch.Tensor) -> L.ConvDesc:
    d = L.ConvDesc()
    d.dtype = prec.code
    d.N, d.H, d.W, d.Cin, d.Cout, d.ksize = N, H, W, cin, cout, k
    d.nsrc = len(srcs)
    for i, s in enumerate(srcs):
        d.src[i] = s
    d.weight = weight.data_ptr()
    return d


def _materialize(prec: Precision, src: L.Src, N: int, H: int, W: int) -> torch.Tensor:
    """The virtual source as a plain NHWC tensor (what the consuming conv's loader would have built)."""
    out = torch.empty(N, H, W, src.C, dtype=prec.torch_dtype, device="cuda")
    L.call("unet_materialize", prec.code, src, N, H, W, vp(out), stream())
    return out


def finalize_many(acts) -> None:
    """Launch the deferred batch-statistics finalizes of several activations (ConvBN.forward(defer_fin=True))
    as one unet_bn_finalize_multi launch: the same per-channel work and results as one unet_bn_finalize each."""
    jobs = [a.fin_job for a in acts if getattr(a, "fin_job", None) is not None]
    for i in range(0, len(jobs), L.BN_MULTI_MAX):
        chunk = jobs[i:i + L.BN_MULTI_MAX]
        arr = (L.BnFinJob * len(chunk))(*[j for j, _ in chunk])
        L.call("unet_bn_finalize_multi", len(chunk), arr, stream())
    for a in acts:
        a.fin_job = None


def _bwd_fin_job(sum_g, sum_gx, rows, C, count, gamma, mean, invstd, dgamma, dbeta, coef) -> L.BnBwdFinJob:
    j = L.BnBwdFinJob()
    j.sum_g, j.sum_gx, j.rows, j.C, j.count = vp(sum_g), vp(sum_gx), rows, C, count
    j.gamma, j.mean, j.invstd = vp(gamma), vp(mean), vp(invstd)
    j.dgamma, j.dbeta, j.accum, j.coef = vp(dgamma), vp(dbeta), 0, vp(coef)
    return j


def _plain_src(t: torch.Tensor) -> L.Src:
    s = L.Src()
    s.kind = L.SRC_PLAIN
    s.H, s.W, s.C = t.shape[1], t.shape[2], t.shape[3]
    s.data = t.data_ptr()
    return s


class Grads(dict):
    """param -> fp32 gradient tensor (assigned once per backward; accumulated if reused)."""

    def put(self, p: torch.nn.Parameter, g: torch.Tensor):
        if p in self:
            self[p] = self[p] + g
        else:
            self[p] = g


# ------------------------------------------------------------------------------------------------
class ConvBN:
    """nn.Conv2d(k, bias=False) -> nn.BatchNorm2d (-> ReLU): one half of DoubleConv
    (layers.py:32-34 / 35-37) or a gate projection W_g / W_x (layers.py:151-160, relu=False)."""

    def __init__(self, conv: torch.nn.Conv2d, bn: torch.nn.BatchNorm2d, relu: bool):
        self.conv, self.bn, self.relu = conv, bn, relu
        self.k = conv.kernel_size[0]
        self.cin, self.cout = conv.in_channels, conv.out_channels
        self.pre_wp = None   # packed forward / dgrad weights, set by NetworkPlan's batched pack
        self.pre_wt = None
        self.wsrcs = None    # weight-gradient sources when the forward stored its transformed input
        self.wact = None
        self.tracked = True  # a backward will follow this forward (act_out only pays off then)

    # ---- forward ----
    def forward(self, prec: Precision, srcs: List[L.Src], N: int, H: int, W: int, training: bool,
                keep=None, defer_fin: bool = False) -> Act:
        """defer_fin: the batch-statistics finalize is not launched here but left on the result as
        `a.fin_job` (an unet_bn_finalize_job) for the caller to launch with others (`finalize_many`)."""
        dev = self.conv.weight.device
        wp = self.pre_wp if self.pre_wp is not None else pack_weight(self.conv.weight, prec, transpose=False)
        self.pre_wp = None
        y = torch.empty(N, H, W, self.cout, dtype=prec.torch_dtype, device=dev)
        d = _conv_desc(prec, N, H, W, self.cin, self.cout, self.k, srcs, wp)
        d.out_mode = L.OUT_Y
        d.out = y.data_ptr()
        # the weight gradient's input: src[0] is a BN activation (+gate) that this forward transforms anyway;
        # where the kernel can write it once (act_out), the wgrad reads that stored map instead.  Maps up to
        # 256^2 only: on the 512^2 64-channel layers the forward is already near its HBM time (read x, write
        # y), and the extra 2-byte-per-element write cost as much there (+50 us) as the wgrad saves
        # (profiles/r03_layerprof_act_out.txt)
        self.wsrcs = self.wact = None
        if training and self.tracked and srcs[0].kind == L.SRC_ACT and H * W <= 256 * 256 and not os.environ.get("UNET_NO_ACT_OUT") \
                and L.load().unet_conv_act_out_ok(d):
            act = torch.empty(N, H, W, srcs[0].C, dtype=prec.torch_dtype, device=dev)
            d.act_out = act.data_ptr()
            self.wsrcs = [_plain_src(act)] + list(srcs[1:])
            self.wact = act              # the descriptors hold raw pointers: keep the tensor alive
        ws = L.attach_workspace(d, dev)   # (split-K scratch, before the stats-row query: the row count depends on it)
        bn = self.bn
        ab = f32(2, self.cout, device=dev)
        use_batch = training or not bn.track_running_stats
        if use_batch:
            mt = L.load().unet_conv_stats_rows(d)
            stats = f32(2, self.cout, mt, device=dev)   # [2][C][rows] (unet_conv_stats_rows)
            d.stats = stats.data_ptr()
        probe.launch(lambda: conv_kernel_name(d), 2.0 * N * H * W * self.cin * self.cout * self.k ** 2,
                     lambda: L.call("unet_conv", d, stream()), d.out_mode)
        mean = f32(self.cout, device=dev)
        invstd = f32(self.cout, device=dev)
        fin_job = None
        if use_batch:
            upd = training and bn.track_running_stats
            mom = -1.0 if bn.momentum is None else float(bn.momentum)
            if defer_fin:
                j = L.BnFinJob()
                j.stats, j.rows, j.C, j.count = vp(stats), mt, self.cout, N * H * W
                j.gamma, j.beta = vp(bn.weight), vp(bn.bias)
                j.running_mean = vp(bn.running_mean) if upd else None
                j.running_var = vp(bn.running_var) if upd else None
                j.num_batches_tracked = vp(bn.num_batches_tracked) if upd else None
                j.momentum, j.eps = mom, float(bn.eps)
                j.mean, j.invstd, j.scale, j.shift = vp(mean), vp(invstd), vp(ab[0]), vp(ab[1])
                fin_job = (j, stats)   # the job holds raw pointers: keep the partial sums alive until it runs
            else:
                L.call("unet_bn_finalize", vp(stats), mt, self.cout, N * H * W, vp(bn.weight), vp(bn.bias),
                       vp(bn.running_mean) if upd else None, vp(bn.running_var) if upd else None,
                       vp(bn.num_batches_tracked) if upd else None, mom, float(bn.eps), vp(mean), vp(invstd),
                       vp(ab[0]), vp(ab[1]), stream())
        else:
            # eval mode (running statistics): mean / invstd are the running ones, which the backward of an
            # eval-mode forward treats as constants (unet_bn_bwd_finalize with count 0)
            L.call("unet_bn_eval_affine", self.cout, vp(bn.weight), vp(bn.bias), vp(bn.running_mean),
                   vp(bn.running_var), float(bn.eps), vp(ab[0]), vp(ab[1]), vp(mean), vp(invstd), stream())
        a = Act(y, ab, self.relu, mean, invstd)
        a.batch_stats = use_batch
        a.keep = keep  # keeps the source tensors alive until backward
        a.bn_owned = True
        a.fin_job = fin_job
        return a

    # ---- backward ----
    def bn_backward(self, prec: Precision, a: Act, grads: Grads, fused=None) -> torch.Tensor:
        """BatchNorm2d(+ReLU) backward: returns dy (op dtype, NHWC) at the conv output.  `fused`: the
        (partial sums [2][rows][C], rows) the producing dgrad's epilogue already reduced (bnb_*)."""
        dev = a.data.device
        P, C = a.pixels, a.C
        pool = a.pool_grad
        if a.oc_fused is not None:
            return self._bn_backward_oc(prec, a, grads)
        assert a.has_grad() or pool is not None, "activation gradient missing"
        gcode = {torch.bfloat16: L.BF16, torch.float16: L.F16}.get(a.grad.dtype, L.F32) if a.has_grad() else L.F32
        if pool is not None:
            # a Down block's input: its MaxPool2d backward is folded into both passes (the pooled dgrad is
            # routed by the argmax codes and added after the other consumers' fp32 sum)
            assert fused is None and gcode == L.F32
            g2, code, ph, pw = pool
            da = vp(a.grad) if a.has_grad() else None
            rows = L.load().unet_bn_bwd_reduce_rows(P, C)
            part = f32(2, rows, C, device=dev)
            L.call("unet_bn_bwd_reduce_pool", prec.code, a.N, a.H, a.W, C, da, vp(g2), vp(code), ph, pw,
                   vp(a.data), vp(a.ab[0]), vp(a.ab[1]), int(a.relu), vp(a.mean), vp(a.invstd), vp(part), stream())
        elif fused is not None:
            part, rows = fused
        else:
            rows = L.load().unet_bn_bwd_reduce_rows(P, C)
            part = f32(2, rows, C, device=dev)
            L.call("unet_bn_bwd_reduce", prec.code, gcode, P, C, vp(a.grad), vp(a.data), vp(a.ab[0]),
                   vp(a.ab[1]), int(a.relu), vp(a.mean), vp(a.invstd), vp(part), stream())
        dgamma, dbeta, coef = f32(C, device=dev), f32(C, device=dev), f32(3, C, device=dev)
        L.call("unet_bn_bwd_finalize", vp(part[0]), vp(part[1]), rows, C, P if a.batch_stats else 0, vp(self.bn.weight), vp(a.mean),
               vp(a.invstd), vp(dgamma), vp(dbeta), 0, vp(coef), stream())
        grads.put(self.bn.weight, dgamma)
        grads.put(self.bn.bias, dbeta)
        dy = torch.empty(a.N, a.H, a.W, C, dtype=prec.torch_dtype, device=dev)
        if pool is not None:
            L.call("unet_bn_bwd_apply_pool", prec.code, a.N, a.H, a.W, C, da, vp(g2), vp(code), ph, pw, vp(a.data),
                   vp(a.ab[0]), vp(a.ab[1]), int(a.relu), vp(coef), vp(dy), stream())
            a.pool_grad = None
        else:
            L.call("unet_bn_bwd_apply", prec.code, gcode, P, C, vp(a.grad), vp(a.data), vp(a.ab[0]), vp(a.ab[1]),
                   int(a.relu), vp(coef), vp(dy), stream())
        return dy

    def _bn_backward_oc(self, prec: Precision, a: Act, grads: Grads) -> torch.Tensor:
        """BatchNorm2d(+ReLU) backward of OutConv's input: the sums came from unet_outconv_bwd_bn, the apply
        recomputes OutConv's input gradient from the logit gradient (unet_bn_bwd_apply_oc)."""
        dl, w, k, part, rows = a.oc_fused
        a.oc_fused = None
        dev = a.data.device
        C = a.C
        dgamma, dbeta, coef = f32(C, device=dev), f32(C, device=dev), f32(3, C, device=dev)
        L.call("unet_bn_bwd_finalize", vp(part[0]), vp(part[1]), rows, C, a.pixels if a.batch_stats else 0,
               vp(self.bn.weight), vp(a.mean), vp(a.invstd), vp(dgamma), vp(dbeta), 0, vp(coef), stream())
        grads.put(self.bn.weight, dgamma)
        grads.put(self.bn.bias, dbeta)
        dy = torch.empty(a.N, a.H, a.W, C, dtype=prec.torch_dtype, device=dev)
        L.call("unet_bn_bwd_apply_oc", prec.code, a.N, a.H, a.W, C, k, vp(a.data), vp(a.ab[0]), vp(a.ab[1]),
               int(a.relu), vp(w), vp(dl), vp(coef), vp(dy), stream())
        return dy

    def conv_backward(self, prec: Precision, dy: torch.Tensor, srcs: List[L.Src], grads: Grads,
                      dgrad: Optional[dict]):
        """wgrad into grads[conv.weight]; dgrad routed by `dgrad`:
        {'mode': 'f32', 'out': t, 'accum': 0/1, 'out2': t2, 'accum2': 0/1, 'split': s}
        {'mode': 'pool', 'out': t (initialised), 'pool_src': Src}"""
        N, H, W, cout = dy.shape
        dev = dy.device
        wd = L.WgradDesc()
        wd.dtype = prec.code
        wd.N, wd.H, wd.W, wd.Cin, wd.Cout, wd.ksize = N, H, W, self.cin, self.cout, self.k
        if self.wsrcs is not None:
            srcs = self.wsrcs          # the forward's stored copy of its (transformed) input
        wd.nsrc = len(srcs)
        for i, s in enumerate(srcs):
            wd.src[i] = s
        wd.dy = dy.data_ptr()
        dw = f32(self.cout, self.cin, self.k, self.k, device=dev)
        wd.dw = dw.data_ptr()
        wd.accum = 0
        ws_bytes = L.load().unet_wgrad_workspace(wd)
        ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=dev)
        wd.workspace = ws.data_ptr()
        probe.launch(lambda: wgrad_kernel_name(wd), 2.0 * N * H * W * self.cin * self.cout * self.k ** 2,
                     lambda: L.call("unet_conv_wgrad", wd, stream()))
        grads.put(self.conv.weight, dw)
        self.wsrcs = self.wact = None
        if dgrad is None:
            return
        wt = self.pre_wt if self.pre_wt is not None else pack_weight(self.conv.weight, prec, transpose=True)
        self.pre_wt = None
        d = _conv_desc(prec, N, H, W, self.cout, self.cin, self.k, [_plain_src(dy)], wt)
        ws = None   # split-K scratch (L.attach_workspace), attached once every other field is set
        if dgrad["mode"] == "y":
            # op-dtype gradient, stored; with "bnb" (the Act it is the gradient of) the epilogue also
            # reduces that activation's BatchNorm-backward sums, returned in dgrad["bnb_part"]
            d.out_mode = L.OUT_Y
            d.out = dgrad["out"].data_ptr()
            a = dgrad.get("bnb")
            if a is not None:
                d.bnb_y, d.bnb_scale, d.bnb_shift = vp(a.data), vp(a.ab[0]), vp(a.ab[1])
                d.bnb_relu, d.bnb_mean, d.bnb_invstd = int(a.relu), vp(a.mean), vp(a.invstd)
                ws = L.attach_workspace(d, dev)
                rows = L.load().unet_conv_stats_rows(d)
                part = f32(2, rows, self.cin, device=dev)
                d.bnb_stats = part.data_ptr()
                dgrad["bnb_part"] = (part, rows)
        elif dgrad["mode"] == "f32_gated":
            # the attention gate's W_x input gradient plus the x*s term: out (+)= s * d(x*s) + W_x^T dy
            d.out_mode = L.OUT_F32_GATED
            d.out = dgrad["out"].data_ptr()
            d.accum = int(dgrad.get("accum", 0))
            d.split = self.cin
            ps = L.Src()
            ps.kind, ps.C, ps.H, ps.W = L.SRC_PLAIN, self.cin, H, W
            ps.data, ps.gate_p, ps.gate_ab = vp(dgrad["dxs"]), vp(dgrad["gate_p"]), vp(dgrad["gate_ab"])
            d.pool_src = ps
        elif dgrad["mode"] == "pool":
            d.out_mode = L.OUT_POOL_BWD
            d.out = dgrad["out"].data_ptr()
            d.pool_src = dgrad["pool_src"]
            d.pool_code = vp(dgrad.get("code"))
        else:
            d.out_mode = L.OUT_F32
            d.out = dgrad["out"].data_ptr()
            d.accum = int(dgrad.get("accum", 0))
            d.split = int(dgrad.get("split", self.cin))
            o2 = dgrad.get("out2")
            d.out2 = o2.data_ptr() if o2 is not None else None
            d.accum2 = int(dgrad.get("accum2", 0))
        if ws is None:
            ws = L.attach_workspace(d, dev)
        probe.launch(lambda: conv_kernel_name(d), 2.0 * N * H * W * self.cin * self.cout * self.k ** 2,
                     lambda: L.call("unet_conv", d, stream()), d.out_mode)


# ------------------------------------------------------------------------------------------------
class DoubleConvStage:
    """DoubleConv: (conv3x3 -> BN -> ReLU) x 2 — layers.py:16-41."""

    def __init__(self, m):
        seq = m.double_conv
        self.c1 = ConvBN(seq[0], seq[1], True)
        self.c2 = ConvBN(seq[3], seq[4], True)

    def forward(self, prec, srcs, N, H, W, training, keep=None) -> Act:
        self.srcs = srcs
        self.a1 = self.c1.forward(prec, srcs, N, H, W, training, keep)
        self.a2 = self.c2.forward(prec, [self.a1.src()], N, H, W, training)
        return self.a2

    def backward(self, prec, grads: Grads, dgrad: Optional[dict]):
        dy2 = self.c2.bn_backward(prec, self.a2, grads)
        if prec.code != L.F32:
            # the middle activation has one consumer (the second conv): its gradient is written once,
            # in the 16-bit operand type (as under torch.autocast), which halves the dgrad store and the
            # BN-backward reads
            # BN1's backward sums are reduced by that dgrad's epilogue (no separate pass over g1 and y1)
            g1 = self.a1.grad_single(prec.torch_dtype)
            # (env UNET_NO_BNB_FUSE: A/B switch back to the separate unet_bn_bwd_reduce pass)
            route = {"mode": "y", "out": g1, "bnb": None if os.environ.get("UNET_NO_BNB_FUSE") else self.a1}
            self.c2.conv_backward(prec, dy2, [self.a1.src()], grads, route)
            fused = route.get("bnb_part")
        else:
            g1, acc = self.a1.grad_target()
            self.c2.conv_backward(prec, dy2, [self.a1.src()], grads, {"mode": "f32", "out": g1, "accum": acc})
            fused = None
        del dy2
        dy1 = self.c1.bn_backward(prec, self.a1, grads, fused)
        self.c1.conv_backward(prec, dy1, self.srcs, grads, dgrad)


# ------------------------------------------------------------------------------------------------
class GateStage:
    """AttentionGate — layers.py:126-192: W_g(g_up), W_x(x) (1x1 conv + BN), relu(sum), psi
    (1x1 conv -> BN(1) -> sigmoid), x * psi.  g_up = bilinear(g, size=x) (:183)."""

    def __init__(self, m):
        self.cg = ConvBN(m.W_g[0], m.W_g[1], False)
        self.cx = ConvBN(m.W_x[0], m.W_x[1], False)
        self.psi_conv, self.psi_bn = m.psi[0], m.psi[1]
        self.ci = self.cg.cout

    def forward(self, prec, g: Act, x: Act, training: bool, g_up: Optional[L.Src] = None,
                g_up_t: Optional[torch.Tensor] = None):
        N, H, W = x.N, x.H, x.W
        dev = x.data.device
        self.g, self.x = g, x
        # g_up_t is given only for an untracked eval-mode forward (no backward follows)
        if (not training and g_up_t is not None and prec.code != L.F32
                and self.psi_bn.track_running_stats and self.cg.bn.track_running_stats
                and self.cx.bn.track_running_stats and g.C % 32 == 0 and x.C % 32 == 0 and self.ci % 32 == 0):
            self._forward_eval(prec, g_up_t, x)
            return
        # bilinear(g -> x size) (layers.py:183): the Up stage's materialised map when it is the same one
        self.src_g = g_up if g_up is not None else g.src_up(H, W, 0, 0)
        # the two projections' BatchNorm finalizes are independent: one launch after both convs (round 5)
        self.gw = self.cg.forward(prec, [self.src_g], N, H, W, training, defer_fin=True)
        self.gw_src = [self.src_g]
        self.xw = self.cx.forward(prec, [x.src()], N, H, W, training, defer_fin=True)
        finalize_many([self.gw, self.xw])
        P = N * H * W
        self.p = f32(N, H, W, device=dev)
        rows = L.load().unet_gate_psi_rows(P)
        part = f32(2, rows, device=dev)
        self.wpsi = self.psi_conv.weight.detach().reshape(-1).float().contiguous()
        L.call("unet_gate_psi", prec.code, P, self.ci, vp(self.gw.data), vp(self.xw.data), vp(self.gw.ab),
               vp(self.xw.ab), vp(self.wpsi), vp(self.p), vp(part), stream())
        bn = self.psi_bn
        self.psi_ab = f32(2, 1, device=dev)
        use_batch = training or not bn.track_running_stats
        self.psi_batch = use_batch
        self.psi_mean, self.psi_invstd = f32(1, device=dev), f32(1, device=dev)
        if use_batch:
            upd = training and bn.track_running_stats
            mom = -1.0 if bn.momentum is None else float(bn.momentum)
            L.call("unet_bn_finalize", vp(part), rows, 1, P, vp(bn.weight), vp(bn.bias),
                   vp(bn.running_mean) if upd else None, vp(bn.running_var) if upd else None,
                   vp(bn.num_batches_tracked) if upd else None, mom, float(bn.eps), vp(self.psi_mean),
                   vp(self.psi_invstd), vp(self.psi_ab[0]), vp(self.psi_ab[1]), stream())
        else:
            L.call("unet_bn_eval_affine", 1, vp(bn.weight), vp(bn.bias), vp(bn.running_mean), vp(bn.running_var),
                   float(bn.eps), vp(self.psi_ab[0]), vp(self.psi_ab[1]), vp(self.psi_mean), vp(self.psi_invstd),
                   stream())

    def _forward_eval(self, prec, g_up_t: torch.Tensor, x: Act):
        """Eval mode, no autograd (predict.py): BN on running statistics, so psi's pre-activation is
        computed in one pass from g_up and x (unet_gate_psi_eval) without storing W_g(g) / W_x(x)."""
        dev = x.data.device
        ci = self.ci
        wg = self.cg.pre_wp if self.cg.pre_wp is not None else pack_weight(self.cg.conv.weight, prec, False)
        wx = self.cx.pre_wp if self.cx.pre_wp is not None else pack_weight(self.cx.conv.weight, prec, False)
        self.cg.pre_wp = self.cx.pre_wp = None
        gab, xab = f32(2, ci, device=dev), f32(2, ci, device=dev)
        for bn, ab in ((self.cg.bn, gab), (self.cx.bn, xab)):
            L.call("unet_bn_eval_affine", ci, vp(bn.weight), vp(bn.bias), vp(bn.running_mean), vp(bn.running_var),
                   float(bn.eps), vp(ab[0]), vp(ab[1]), None, None, stream())
        self.wpsi = self.psi_conv.weight.detach().reshape(-1).float().contiguous()
        self.p = f32(x.N, x.H, x.W, device=dev)
        L.call("unet_gate_psi_eval", prec.code, x.pixels, g_up_t.shape[-1], x.C, ci, vp(g_up_t), vp(x.data),
               vp(x.ab[0]), vp(x.ab[1]), int(x.relu), vp(wg), vp(wx), vp(gab), vp(xab), vp(self.wpsi),
               vp(self.p), stream())
        bn = self.psi_bn
        self.psi_ab = f32(2, 1, device=dev)
        L.call("unet_bn_eval_affine", 1, vp(bn.weight), vp(bn.bias), vp(bn.running_mean), vp(bn.running_var),
               float(bn.eps), vp(self.psi_ab[0]), vp(self.psi_ab[1]), None, None, stream())

    def gated_src(self) -> L.Src:
        return self.x.src_gated(self.p, self.psi_ab)

    def backward(self, prec, d_xs: torch.Tensor, grads: Grads, d_gup: torch.Tensor, d_gup_accum: int):
        """d_xs: fp32 NHWC grad of x*s.  Adds into x.grad; writes/adds W_g's input-grad into d_gup
        (fp32 NHWC at x's size, the upsampled-g space)."""
        x = self.x
        dev = x.data.device
        P, Cx, Ci = x.pixels, x.C, self.ci
        # (1) through x*s and the sigmoid; psi-BN backward sums.  Where the bf16 1x1 kernel serves the W_x
        # dgrad, the x*s term of dx is added by that dgrad's epilogue (one write of dx instead of a write
        # here plus a read-modify-write there)
        fuse = self._wx_gated_ok(prec, x)
        dx, dx_acc = (None, 0) if fuse else x.grad_target()
        dq = f32(P, device=dev)
        rows1 = L.load().unet_gate_psi_rows(P)
        part1 = f32(2, rows1, device=dev)
        L.call("unet_gate_bwd1", prec.code, P, Cx, vp(d_xs), vp(x.data), vp(x.ab[0]), vp(x.ab[1]), int(x.relu), vp(self.p),
               vp(self.psi_ab), vp(self.psi_mean), vp(self.psi_invstd), vp(dx), dx_acc, vp(dq), vp(part1), stream())
        dgp, dbp, pcoef = f32(1, device=dev), f32(1, device=dev), f32(3, device=dev)
        L.call("unet_bn_bwd_finalize", vp(part1[0]), vp(part1[1]), rows1, 1, P if self.psi_batch else 0,
               vp(self.psi_bn.weight),
               vp(self.psi_mean), vp(self.psi_invstd), vp(dgp), vp(dbp), 0, vp(pcoef), stream())
        grads.put(self.psi_bn.weight, dgp)
        grads.put(self.psi_bn.bias, dbp)
        # (2) psi conv / relu / both BN backward sums
        rows2 = L.load().unet_gate_bwd2_rows(P, Ci)
        part2 = f32(4, rows2, Ci, device=dev)
        L.call("unet_gate_bwd2", prec.code, P, Ci, vp(self.gw.data), vp(self.xw.data), vp(self.gw.ab),
               vp(self.xw.ab), vp(self.gw.mean), vp(self.gw.invstd), vp(self.xw.mean), vp(self.xw.invstd),
               vp(self.wpsi), vp(dq), vp(self.p), vp(pcoef), vp(part2), stream())
        dgg, dbg, gcoef = f32(Ci, device=dev), f32(Ci, device=dev), f32(3, Ci, device=dev)
        dgx, dbx, xcoef = f32(Ci, device=dev), f32(Ci, device=dev), f32(3, Ci, device=dev)
        dwpsi = f32(Ci, device=dev)
        # both projections' BN-backward finalizes and psi's weight gradient (a column sum) in one launch (round 5)
        jobs = [_bwd_fin_job(part2[0], part2[1], rows2, Ci, P if self.gw.batch_stats else 0, self.cg.bn.weight,
                             self.gw.mean, self.gw.invstd, dgg, dbg, gcoef),
                _bwd_fin_job(part2[0], part2[2], rows2, Ci, P if self.xw.batch_stats else 0, self.cx.bn.weight,
                             self.xw.mean, self.xw.invstd, dgx, dbx, xcoef),
                _bwd_fin_job(part2[3], None, rows2, Ci, 0, None, None, None, None, dwpsi, None)]
        L.call("unet_bn_bwd_finalize_multi", len(jobs), (L.BnBwdFinJob * len(jobs))(*jobs), stream())
        grads.put(self.cg.bn.weight, dgg)
        grads.put(self.cg.bn.bias, dbg)
        grads.put(self.cx.bn.weight, dgx)
        grads.put(self.cx.bn.bias, dbx)
        grads.put(self.psi_conv.weight, dwpsi.view(1, Ci, 1, 1))
        # (3) dgw, dxw
        dgw = torch.empty(x.N, x.H, x.W, Ci, dtype=prec.torch_dtype, device=dev)
        dxw = torch.empty_like(dgw)
        L.call("unet_gate_bwd3", prec.code, P, Ci, vp(self.gw.data), vp(self.xw.data), vp(self.gw.ab),
               vp(self.xw.ab), vp(self.wpsi), vp(dq), vp(self.p), vp(pcoef), vp(gcoef), vp(xcoef), vp(dgw), vp(dxw),
               stream())
        # (4) the two 1x1 projections
        self.cg.conv_backward(prec, dgw, self.gw_src, grads,
                              {"mode": "f32", "out": d_gup, "accum": d_gup_accum})
        dx2, acc2 = x.grad_target()
        if fuse:
            self.cx.conv_backward(prec, dxw, [x.src()], grads, {"mode": "f32_gated", "out": dx2, "accum": acc2,
                                                                "dxs": d_xs, "gate_p": self.p,
                                                                "gate_ab": self.psi_ab})
        else:
            self.cx.conv_backward(prec, dxw, [x.src()], grads, {"mode": "f32", "out": dx2, "accum": acc2})

    def _wx_gated_ok(self, prec, x: Act) -> bool:
        """Whether the W_x dgrad (Ci -> Cx 1x1) runs on the kernel that serves UNET_OUT_F32_GATED."""
        if prec.code not in (L.BF16, L.F16) or os.environ.get("UNET_NO_GATE_FUSE"):   # (env: A/B switch)
            return False
        d = L.ConvDesc()
        d.dtype, d.N, d.H, d.W, d.Cin, d.Cout, d.ksize, d.nsrc = prec.code, x.N, x.H, x.W, self.ci, x.C, 1, 1
        s = L.Src()
        s.kind, s.C, s.H, s.W = L.SRC_PLAIN, self.ci, x.H, x.W
        d.src[0] = s
        d.out_mode, d.split = L.OUT_F32_GATED, x.C
        return conv_kernel_name(d).startswith("pw_conv_kernel")


# ------------------------------------------------------------------------------------------------
def mark_tracked(stage, tracked: bool):
    """Tell every ConvBN of a stage whether a backward will follow its forward."""
    for attr in ("c1", "c2", "cg", "cx"):
        cb = getattr(stage, attr, None)
        if cb is not None:
            cb.tracked = tracked
    for attr in ("dc", "gate"):
        sub = getattr(stage, attr, None)
        if sub is not None:
            mark_tracked(sub, tracked)


def _pad_geometry(x1: Act, x2: Act):
    up_h, up_w = 2 * x1.H, 2 * x1.W
    dy, dx = x2.H - up_h, x2.W - up_w
    return up_h, up_w, dy // 2, dx // 2     # F.pad([dx//2, dx-dx//2, dy//2, dy-dy//2]) — layers.py:101


class ConvTStage:
    """nn.ConvTranspose2d(Cin, Ct, kernel_size=2, stride=2) with bias — layers.py:81,218.

    Run as a 1x1 conv with 4*Ct output channels (row (2a+b)*Ct + c of the reshaped weight is
    W[:, c, a, b]) whose SHUFFLE2 epilogue scatters channel (a, b, c) of input pixel (y, x) to output
    pixel (2y+a, 2x+b) and adds the bias.  Backward: space-to-depth of the output gradient
    (unet_convt_bwd_prep, which also sums the bias gradient), then the ordinary 1x1 wgrad / dgrad."""

    def __init__(self, m: torch.nn.ConvTranspose2d):
        if m.kernel_size != (2, 2) or m.stride != (2, 2) or m.padding != (0, 0) or m.groups != 1 or \
                m.dilation != (1, 1) or m.output_padding != (0, 0):
            raise NotImplementedError("unet HIP path: only ConvTranspose2d(k=2, s=2) is supported")
        self.m = m
        self.cin, self.ct = m.in_channels, m.out_channels

    def _w4(self) -> torch.Tensor:
        return self.m.weight.detach().float().permute(2, 3, 1, 0).reshape(4 * self.ct, self.cin, 1, 1).contiguous()

    def forward(self, prec, x1: Act) -> Act:
        dev = x1.data.device
        N, h, w = x1.N, x1.H, x1.W
        self.x1 = x1
        self.w4 = self._w4()
        wp = pack_weight(self.w4, prec, transpose=False)
        y = torch.empty(N, 2 * h, 2 * w, self.ct, dtype=prec.torch_dtype, device=dev)
        d = _conv_desc(prec, N, h, w, self.cin, 4 * self.ct, 1, [x1.src()], wp)
        d.out_mode = L.OUT_SHUFFLE2
        d.out = y.data_ptr()
        b = self.m.bias
        self.bias = b.detach().float().contiguous() if b is not None else None
        d.bias = vp(self.bias)
        probe.launch(lambda: conv_kernel_name(d), 2.0 * N * h * w * self.cin * 4 * self.ct,
                     lambda: L.call("unet_conv", d, stream()), d.out_mode)
        return Act(y, None, False)

    def backward(self, prec, d_up: torch.Tensor, pad_t: int, pad_l: int, grads: Grads, need_dx: bool = True):
        """d_up: fp32 NHWC gradient at the padded map that holds this output at (pad_t, pad_l)."""
        x1 = self.x1
        dev = x1.data.device
        N, h, w, ct = x1.N, x1.H, x1.W, self.ct
        P = N * h * w
        dys = torch.empty(N, h, w, 4 * ct, dtype=prec.torch_dtype, device=dev)
        rows = L.load().unet_convt_bwd_rows(P)
        part = f32(rows, ct, device=dev)
        L.call("unet_convt_bwd_prep", prec.code, N, h, w, ct, d_up.shape[1], d_up.shape[2], pad_t, pad_l, vp(d_up),
               vp(dys), vp(part), stream())
        if self.m.bias is not None:
            db = f32(ct, device=dev)
            L.call("unet_colsum", vp(part), rows, ct, vp(db), 0, stream())
            grads.put(self.m.bias, db)
        # weight gradient of the equivalent 1x1 conv, back to the ConvTranspose2d layout [Cin][Ct][2][2]
        wd = L.WgradDesc()
        wd.dtype = prec.code
        wd.N, wd.H, wd.W, wd.Cin, wd.Cout, wd.ksize = N, h, w, self.cin, 4 * ct, 1
        wd.nsrc = 1
        wd.src[0] = x1.src()
        wd.dy = dys.data_ptr()
        dw4 = f32(4 * ct, self.cin, device=dev)
        wd.dw = dw4.data_ptr()
        wd.accum = 0
        ws = torch.empty(max(L.load().unet_wgrad_workspace(wd), 16), dtype=torch.uint8, device=dev)
        wd.workspace = ws.data_ptr()
        probe.launch(lambda: wgrad_kernel_name(wd), 2.0 * P * self.cin * 4 * ct,
                     lambda: L.call("unet_conv_wgrad", wd, stream()))
        grads.put(self.m.weight, dw4.view(2, 2, ct, self.cin).permute(3, 2, 0, 1).contiguous())
        if not need_dx:
            return
        wt = pack_weight(self.w4, prec, transpose=True)
        d = _conv_desc(prec, N, h, w, 4 * ct, self.cin, 1, [_plain_src(dys)], wt)
        d.out_mode = L.OUT_F32
        g, acc = x1.grad_target()
        d.out = g.data_ptr()
        d.accum = acc
        d.split = self.cin
        probe.launch(lambda: conv_kernel_name(d), 2.0 * P * self.cin * 4 * ct,
                     lambda: L.call("unet_conv", d, stream()), d.out_mode)


class UpStage:
    """Up (layers.py:64-106) and AttentionUp (layers.py:195-255):
    [skip (· attention), pad(up(x1))] -> DoubleConv, with the concat/pad (and bilinear upsample)
    virtual.  bilinear=False runs the ConvTranspose2d as its own stage (ConvTStage) whose output is
    read in place by the DoubleConv's loader."""

    def __init__(self, m, attention: bool):
        if isinstance(m.up, torch.nn.Upsample):
            self.convt = None
        elif isinstance(m.up, torch.nn.ConvTranspose2d):
            self.convt = ConvTStage(m.up)
        else:
            raise NotImplementedError(f"unet HIP path: unsupported up module {type(m.up).__name__}")
        self.dc = DoubleConvStage(m.conv)
        self.gate = GateStage(m.attention) if attention else None

    def forward(self, prec, x1: Act, x2: Act, training: bool, eval_only: bool = False) -> Act:
        self.x1, self.x2 = x1, x2
        self.geo = _pad_geometry(x1, x2)
        up_h, up_w, pt, pl = self.geo
        up_t = None
        if self.convt is None:
            # bilinear x2 of relu(bn(x1)), padded into the skip's frame, written once (layers.py:78,98-102)
            up_t = _materialize(prec, x1.src_up(up_h, up_w, pt, pl), x2.N, x2.H, x2.W)
            self.up_t = up_t
        if self.gate is not None:
            same = up_t is not None and up_h == x2.H and up_w == x2.W and pt == 0 and pl == 0
            self.gate.forward(prec, x1, x2, training, g_up=_plain_src(up_t) if same else None,
                              g_up_t=up_t if same and eval_only else None)
            skip = self.gate.gated_src()
        else:
            skip = x2.src()
        if self.convt is not None:
            self.u = self.convt.forward(prec, x1)
            up = self.u.src_placed(pt, pl)
        else:
            up = _plain_src(up_t)
        return self.dc.forward(prec, [skip, up], x2.N, x2.H, x2.W, training)

    def backward(self, prec, grads: Grads):
        x1, x2 = self.x1, self.x2
        dev = x2.data.device
        up_h, up_w, pt, pl = self.geo
        cu = self.convt.ct if self.convt is not None else x1.C
        d_up = f32(x2.N, x2.H, x2.W, cu, device=dev)
        if self.gate is not None:
            d_xs = f32(x2.N, x2.H, x2.W, x2.C, device=dev)
            self.dc.backward(prec, grads, {"mode": "f32", "out": d_xs, "accum": 0, "out2": d_up, "accum2": 0,
                                           "split": x2.C})
            same = (self.convt is None and up_h == x2.H and up_w == x2.W and pt == 0 and pl == 0)
            if same:
                self.gate.backward(prec, d_xs, grads, d_up, 1)
            else:
                d_gup = f32(x2.N, x2.H, x2.W, x1.C, device=dev)
                self.gate.backward(prec, d_xs, grads, d_gup, 0)
                gx, acc = x1.grad_target()
                L.call("unet_upsample_bwd", x1.N, x1.C, x1.H, x1.W, x2.H, x2.W, 0, 0, x2.H, x2.W,
                       up_scale(x1.H, x2.H), up_scale(x1.W, x2.W), vp(d_gup), vp(gx), acc, stream())
        else:
            g2, acc2 = x2.grad_target()
            self.dc.backward(prec, grads, {"mode": "f32", "out": g2, "accum": acc2, "out2": d_up, "accum2": 0,
                                           "split": x2.C})
        if self.convt is not None:
            self.convt.backward(prec, d_up, pt, pl, grads)
            return
        gx, acc = x1.grad_target()
        L.call("unet_upsample_bwd", x1.N, x1.C, x1.H, x1.W, up_h, up_w, pt, pl, x2.H, x2.W,
               up_scale(x1.H, up_h), up_scale(x1.W, up_w), vp(d_up), vp(gx), acc, stream())


class DownStage:
    """Down: MaxPool2d(2) -> DoubleConv — layers.py:44-61 (the pool is the conv loader's job)."""

    def __init__(self, m):
        self.dc = DoubleConvStage(m.maxpool_conv[1])

    def forward(self, prec, x: Act, training: bool) -> Act:
        self.x = x
        # MaxPool2d(2)(relu(bn(y))) written once (quarter size); the conv, its wgrad read it plain
        h, w = x.H // 2, x.W // 2
        self.xp = torch.empty(x.N, h, w, x.C, dtype=prec.torch_dtype, device=x.data.device)
        self.code = None
        vec = 8 if prec.code != L.F32 else 4
        cv = x.C // vec
        if x.C % vec == 0 and cv <= 256 and cv & (cv - 1) == 0:
            # the 2x2 argmax is recorded too: the pool backward then routes by one byte per element
            self.code = torch.empty(x.N, h, w, x.C, dtype=torch.uint8, device=x.data.device)
            L.call("unet_materialize_pool", prec.code, x.src_pool(), x.N, h, w, vp(self.xp), vp(self.code), stream())
        else:
            L.call("unet_materialize", prec.code, x.src_pool(), x.N, h, w, vp(self.xp), stream())
        return self.dc.forward(prec, [_plain_src(self.xp)], x.N, h, w, training)

    def backward(self, prec, grads: Grads):
        x = self.x
        cv = x.C // 8
        if self.code is not None and x.bn_owned and x.C % 8 == 0 and cv <= 256 and cv & (cv - 1) == 0 \
                and not os.environ.get("UNET_NO_POOL_FOLD") \
                and x.pixels < 2 ** 31 and x.pool_grad is None and (x.grad is None or x.grad.dtype == torch.float32):
            # the dgrad is written at the pooled resolution (plain fp32 stores); the producer's BatchNorm
            # backward routes it through the argmax codes while it reads the other consumers' gradient
            # (unet_bn_bwd_reduce_pool / _apply_pool), so the full-resolution map is never read-modified
            h, w = self.xp.shape[1], self.xp.shape[2]
            g2 = f32(x.N, h, w, x.C, device=x.data.device)
            self.dc.backward(prec, grads, {"mode": "f32", "out": g2, "accum": 0})
            x.pool_grad = (g2, self.code, h, w)
            return
        g = x.grad_zeroed()
        self.dc.backward(prec, grads, {"mode": "pool", "out": g, "pool_src": x.src_pool(), "code": self.code})


class OutConvStage:
    """OutConv: 1x1 conv with bias -> fp32 NCHW logits — layers.py:109-123."""

    def __init__(self, m, sole_consumer: bool = False):
        self.conv = m.conv
        self.k = self.conv.out_channels
        # True for the network's OutConv: the last decoder activation feeds nothing else (unet.py:92, 203)
        self.sole_consumer = sole_consumer

    def forward(self, prec, a: Act) -> torch.Tensor:
        self.a = a
        dev = a.data.device
        out = f32(a.N, self.k, a.H, a.W, device=dev)
        self.w = self.conv.weight.detach().reshape(self.k, -1).float().contiguous()
        b = self.conv.bias.detach().float().contiguous()
        L.call("unet_outconv_fwd", prec.code, a.N, a.H, a.W, a.C, self.k, vp(a.data), vp(a.ab[0]), vp(a.ab[1]),
               int(a.relu), vp(self.w), vp(b), vp(out), stream())
        return out

    def backward(self, prec, dlogits: torch.Tensor, grads: Grads):
        a = self.a
        dev = a.data.device
        dl = dlogits.float().contiguous()
        rows = L.load().unet_outconv_rows(a.pixels)
        part = f32(rows, self.k + 1, max(a.C, self.k), device=dev)
        cv = a.C // 8
        if (self.sole_consumer and a.bn_owned and not a.has_grad() and a.pool_grad is None and self.k == 2
                and a.C % 8 == 0 and cv <= 256 and cv & (cv - 1) == 0 and a.pixels < 2 ** 31
                and not os.environ.get("UNET_NO_OC_FUSE")):
            # OutConv is the activation's only consumer: its gradient W^T dl is not stored; the BN-backward sums
            # are taken here and the BN apply recomputes it (unet_outconv_bwd_bn / unet_bn_bwd_apply_oc)
            bpart = f32(2, rows, a.C, device=dev)
            L.call("unet_outconv_bwd_bn", prec.code, a.N, a.H, a.W, a.C, self.k, vp(a.data), vp(a.ab[0]),
                   vp(a.ab[1]), int(a.relu), vp(self.w), vp(dl), vp(a.mean), vp(a.invstd), vp(part), vp(bpart),
                   stream())
            a.oc_fused = (dl, self.w, self.k, bpart, rows)
        else:
            g, acc = a.grad_target()
            L.call("unet_outconv_bwd", prec.code, a.N, a.H, a.W, a.C, self.k, vp(a.data), vp(a.ab[0]), vp(a.ab[1]),
                   int(a.relu), vp(self.w), vp(dl), vp(g), acc, vp(part), stream())
        dw, db = f32(self.k, a.C, 1, 1, device=dev), f32(self.k, device=dev)
        L.call("unet_outconv_bwd_finalize", vp(part), rows, a.C, self.k, vp(dw), vp(db), 0, stream())
        grads.put(self.conv.weight, dw)
        grads.put(self.conv.bias, db)


class DSHeadStage:
    """Deep-supervision head: OutConv on a decoder map, bilinear(align_corners) to the input size —
    unet.py:170-173, 204-209."""

    def __init__(self, m):
        self.oc = OutConvStage(m)

    def forward(self, prec, a: Act, H: int, W: int) -> torch.Tensor:
        lo = self.oc.forward(prec, a)
        self.lo_shape = lo.shape
        self.size = (H, W)
        out = f32(a.N, self.oc.k, H, W, device=lo.device)
        L.call("unet_resize_nchw", a.N * self.oc.k, a.H, a.W, H, W, up_scale(a.H, H), up_scale(a.W, W), vp(lo),
               vp(out), stream())
        return out

    def backward(self, prec, dout: torch.Tensor, grads: Grads):
        a = self.oc.a
        H, W = self.size
        dlo = f32(*self.lo_shape, device=dout.device)
        dd = dout.float().contiguous()
        L.call("unet_resize_nchw_bwd", a.N * self.oc.k, a.H, a.W, H, W, up_scale(a.H, H), up_scale(a.W, W), vp(dd),
               vp(dlo), 0, stream())
        self.oc.backward(prec, dlo, grads)


# ------------------------------------------------------------------------------------------------
class NetworkPlan:
    """UNet.forward (unet.py:67-92) / AttentionUNet.forward (unet.py:175-211) as a launch plan.

    The plan is cut at the reference's module boundaries: inc, down1..4, up1..4, outc and the deep-
    supervision heads each have a forward piece (`fwd_*`) and a backward piece (`bwd_*`).  Under
    autograd every piece is its own node (`_hip.functions`), linked by empty "token" tensors along the
    reference's data flow (skip connections included), so a stage's parameter gradients are handed to
    autograd — and to DistributedDataParallel's reducer hooks — as soon as that stage's backward is done.
    Activation gradients do not travel through autograd: consumers accumulate them into the producer's
    `Act.grad` buffer, and the token graph guarantees that a producer runs its backward only after every
    consumer has."""

    def __init__(self, model, attention: bool):
        self.model = model
        self.attention = attention
        self.inc = DoubleConvStage(model.inc)
        self.downs = [DownStage(getattr(model, f"down{i}")) for i in range(1, 5)]
        self.ups = [UpStage(getattr(model, f"up{i}"), attention) for i in range(1, 5)]
        self.outc = OutConvStage(model.outc, sole_consumer=True)
        self.ds = attention and getattr(model, "deep_supervision", False)
        if self.ds:
            self.heads = [DSHeadStage(model.ds_out1), DSHeadStage(model.ds_out2), DSHeadStage(model.ds_out3)]

    def convbns(self):
        """Every conv -> BN pair of the network (their weights are packed in one launch)."""
        out = [self.inc.c1, self.inc.c2]
        for d in self.downs:
            out += [d.dc.c1, d.dc.c2]
        for u in self.ups:
            out += [u.dc.c1, u.dc.c2]
            if u.gate is not None:
                out += [u.gate.cg, u.gate.cx]
        return out

    # ---- forward pieces ----
    def begin(self, prec: Precision, x: torch.Tensor, training: bool, need_dx: bool, tracked: bool = True):
        self.prec, self.training, self.x, self.need_dx = prec, training, x, need_dx
        self.tracked = tracked   # False: no backward will follow (the eval-only kernels may be used)
        self.with_ds = self.ds and training
        self._bwd_packed = False
        cbs = self.convbns()
        jobs = [(cb.conv.weight, False) for cb in cbs]
        # a training forward that a backward follows also packs the transposed (dgrad) weights, in the same
        # launch: the fp32 weights are read once (the second layout from cache) and the backward has no pack
        # launch of its own (round 5; prepare_backward still packs them when this did not)
        tcbs = [cb for cb in cbs if cb is not self.inc.c1 or need_dx] if (tracked and training) else []
        jobs += [(cb.conv.weight, True) for cb in tcbs]
        packed = pack_many(jobs, prec)
        for cb, wp in zip(cbs, packed[:len(cbs)]):
            cb.pre_wp = wp
            cb.tracked = tracked
        for cb, wt in zip(tcbs, packed[len(cbs):]):
            cb.pre_wt = wt
        self._bwd_packed = bool(tcbs)
        self.xs, self.dec = [], []

    def fwd_inc(self):
        N, C, H, W = self.x.shape
        self.xs = [self.inc.forward(self.prec, [_nchw(self.x)], N, H, W, self.training, keep=self.x)]

    def fwd_down(self, i: int):
        self.xs.append(self.downs[i].forward(self.prec, self.xs[-1], self.training))

    def fwd_up(self, i: int):
        y = self.xs[4] if i == 0 else self.dec[-1]
        self.dec.append(self.ups[i].forward(self.prec, y, self.xs[3 - i], self.training,   # d4, d3, d2, d1
                                            eval_only=not self.tracked))

    def fwd_outc(self) -> torch.Tensor:
        return self.outc.forward(self.prec, self.dec[-1])

    def fwd_head(self, k: int) -> torch.Tensor:
        """[ds1(d2), ds2(d3), ds3(d4)][k] resized to the input size (unet.py:204-209)."""
        return self.heads[k].forward(self.prec, (self.dec[2], self.dec[1], self.dec[0])[k], self.x.shape[2],
                                     self.x.shape[3])

    def forward(self, prec: Precision, x: torch.Tensor, training: bool, need_dx: bool):
        """The whole forward in one go (no autograd: eval / no_grad)."""
        self.begin(prec, x, training, need_dx, tracked=False)
        self.fwd_inc()
        for i in range(4):
            self.fwd_down(i)
        for i in range(4):
            self.fwd_up(i)
        outs = [self.fwd_outc()]
        if self.with_ds:
            outs += [self.fwd_head(k) for k in range(3)]     # [logits, ds1(d2), ds2(d3), ds3(d4)]
        return outs

    # ---- backward pieces (run by autograd in reverse data-flow order) ----
    def prepare_backward(self):
        """Pack every transposed (dgrad) weight in one launch, once per backward pass."""
        if self._bwd_packed:
            return
        self._bwd_packed = True
        cbs = [cb for cb in self.convbns() if cb is not self.inc.c1 or self.need_dx]
        for cb, wt in zip(cbs, pack_many([(cb.conv.weight, True) for cb in cbs], self.prec)):
            cb.pre_wt = wt

    def bwd_outc(self, g: Optional[torch.Tensor], grads: Grads):
        self.prepare_backward()
        if g is None:
            x = self.x
            g = torch.zeros(x.shape[0], self.outc.k, x.shape[2], x.shape[3], device=x.device)
        self.outc.backward(self.prec, g, grads)

    def bwd_head(self, k: int, g: Optional[torch.Tensor], grads: Grads):
        self.prepare_backward()
        if g is not None:
            self.heads[k].backward(self.prec, g, grads)

    def bwd_up(self, i: int, grads: Grads):
        self.prepare_backward()
        self.ups[i].backward(self.prec, grads)

    def bwd_down(self, i: int, grads: Grads):
        self.prepare_backward()
        self.downs[i].backward(self.prec, grads)

    def bwd_inc(self, grads: Grads) -> Optional[torch.Tensor]:
        self.prepare_backward()
        if not self.need_dx:
            self.inc.backward(self.prec, grads, None)
            return None
        x = self.x
        N, C, H, W = x.shape
        gx = f32(N, H, W, C, device=x.device)
        self.inc.backward(self.prec, grads, {"mode": "f32", "out": gx, "accum": 0})
        from .runtime import grad_nhwc_to_nchw
        return grad_nhwc_to_nchw(gx)


def _nchw(x: torch.Tensor) -> L.Src:
    from .runtime import nchw_src
    return nchw_src(x)
