"""autograd.Function wrappers: the reference's modules as HIP launch plans.

`run_network` serves UNet / AttentionUNet (whole-network plan with cross-module fusion, one autograd
node per reference module so DDP's reducer sees each stage's parameter gradients as soon as they exist);
`run_module` serves a standalone DoubleConv / Down / Up / AttentionUp / AttentionGate / OutConv call
(NCHW fp32 in and out, exactly like the reference module).  Param grads are returned through
autograd, so `loss.backward()`, DDP hooks, clip_grad_norm_ and optimizers work unchanged.
"""

from __future__ import annotations

from typing import List, Sequence

import torch
from torch.autograd.function import once_differentiable

from . import lib as L
from .runtime import (Act, act_from_nchw, act_to_nchw, f32, get_precision, grad_nchw_to_nhwc, grad_nhwc_to_nchw,
                      nchw_src, require_device, stream, up_scale, vp)
from .stages import (DoubleConvStage, DownStage, GateStage, Grads, NetworkPlan, OutConvStage, UpStage,
                     mark_tracked)


# the plan's activation-gradient buffers and packed dgrad weights are consumed by the first backward
_SECOND_BACKWARD = ("unet HIP path: this graph was already backpropagated; the HIP network does not support a "
                    "second backward through the same forward (retain_graph=True / autograd.grad then backward). "
                    "Run the forward again.")


class _PlanFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, plan, params: Sequence[torch.nn.Parameter], n_in: int, *tensors):
        inputs = tensors[:n_in]
        outs = plan.forward(list(inputs), [ctx.needs_input_grad[3 + i] for i in range(n_in)])
        ctx.plan = plan
        ctx.params = params
        ctx.n_in = n_in
        return tuple(outs)

    @staticmethod
    @once_differentiable
    def backward(ctx, *gouts):
        if ctx.plan is None:
            raise RuntimeError(_SECOND_BACKWARD)
        grads = Grads()
        dins = ctx.plan.backward(list(gouts), grads)
        pgrads = [grads.get(p) for p in ctx.params]
        ctx.plan = None
        return (None, None, None, *dins, *pgrads)


def _apply(plan, module: torch.nn.Module, inputs: List[torch.Tensor]):
    params = [p for p in module.parameters()]
    track = torch.is_grad_enabled() and (any(p.requires_grad for p in params) or any(i.requires_grad for i in inputs))
    if not track:
        plan.tracked = False
        return plan.forward(inputs, [False] * len(inputs))
    return list(_PlanFn.apply(plan, params, len(inputs), *inputs, *params))


# ------------------------------------------------------------------------------------------------
class _Stage:
    """One autograd node of the network plan: `fwd()` runs the stage's launches and returns its
    output (a real tensor, or an empty token standing for the stage's virtual activation); `bwd(gouts,
    grads)` runs its backward launches and returns the gradients of its tensor inputs."""

    __slots__ = ("fwd", "bwd", "params")

    def __init__(self, fwd, bwd, params):
        self.fwd, self.bwd, self.params = fwd, bwd, params


class _StageFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, st: _Stage, n_in: int, *tensors):
        ctx.set_materialize_grads(False)     # unused outputs (a DS head outside the loss) stay None
        ctx.st, ctx.n_in = st, n_in
        return st.fwd()

    @staticmethod
    @once_differentiable
    def backward(ctx, *gouts):
        st = ctx.st
        if st is None:
            raise RuntimeError(_SECOND_BACKWARD)
        grads = Grads()
        dins = st.bwd(list(gouts), grads)
        ctx.st = None
        return (None, None, *dins, *[grads.get(p) for p in st.params])


def _stage(fwd, bwd, module, inputs: List[torch.Tensor]):
    params = [p for p in module.parameters()] if module is not None else []
    return _StageFn.apply(_Stage(fwd, bwd, params), len(inputs), *inputs, *params)


class _NetPlan:
    def __init__(self, model, attention: bool):
        self.model = model
        self.prec = get_precision(model)
        self.training = model.training
        self.net = NetworkPlan(model, attention)

    def run(self, x: torch.Tensor, track: bool):
        """Untracked: one pass over the plan.  Tracked: one autograd node per reference module, linked by
        tokens along the data flow (x -> inc -> down1..4, skips into up1..4 -> outc / DS heads)."""
        net, m = self.net, self.model
        if not track:
            return net.forward(self.prec, x, self.training, False)
        net.begin(self.prec, x, self.training, x.requires_grad)
        dev = x.device

        def token():
            return torch.empty(0, device=dev)

        def fwd_tok(f, *a):
            def run():
                f(*a)
                return token()
            return run

        def bwd_none(f, n_in, *a):
            def run(gouts, grads):
                f(*a, grads)
                return [None] * n_in
            return run

        t = [_stage(fwd_tok(net.fwd_inc), lambda g, grads: [net.bwd_inc(grads)], m.inc, [x])]
        for i in range(4):
            t.append(_stage(fwd_tok(net.fwd_down, i), bwd_none(net.bwd_down, 1, i), getattr(m, f"down{i + 1}"),
                            [t[-1]]))
        dec = []
        y = t[4]
        for i in range(4):
            y = _stage(fwd_tok(net.fwd_up, i), bwd_none(net.bwd_up, 2, i), getattr(m, f"up{i + 1}"), [y, t[3 - i]])
            dec.append(y)
        outs = [_stage(net.fwd_outc, lambda g, grads: (net.bwd_outc(g[0], grads), [None])[1], m.outc, [dec[3]])]
        if net.with_ds:
            for k, (mod, src) in enumerate(((m.ds_out1, dec[2]), (m.ds_out2, dec[1]), (m.ds_out3, dec[0]))):
                outs.append(_stage(lambda k=k: net.fwd_head(k),
                                   lambda g, grads, k=k: (net.bwd_head(k, g[0], grads), [None])[1], mod, [src]))
        return outs


def run_network(model, x: torch.Tensor, attention: bool):
    require_device(x)
    if x.dim() != 4 or x.shape[1] != model.n_channels:
        raise RuntimeError(f"expected input of shape (N, {model.n_channels}, H, W), got {tuple(x.shape)}")
    if x.dtype != torch.float32 or not x.is_contiguous():
        x = x.float().contiguous()
    track = torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in model.parameters()))
    return _NetPlan(model, attention).run(x, track)


# ------------------------------------------------------------------------------------------------
class _ModulePlan:
    """Standalone module call: NCHW fp32 inputs -> NHWC operands -> stage -> NCHW fp32 output."""

    def __init__(self, module, kind: str):
        self.m = module
        self.kind = kind
        self.prec = get_precision(module)
        self.training = module.training
        self.tracked = True      # False: no backward follows (set by _apply)

    def _stage(self, st):
        mark_tracked(st, self.tracked)
        return st

    def forward(self, inputs, needs):
        prec, tr = self.prec, self.training
        self.needs = needs
        xs = [i if (i.dtype == torch.float32 and i.is_contiguous()) else i.float().contiguous() for i in inputs]
        self.xs = xs
        k = self.kind
        if k == "double_conv":
            x = xs[0]
            N, C, H, W = x.shape
            self.st = self._stage(DoubleConvStage(self.m))
            self.out = self.st.forward(prec, [nchw_src(x)], N, H, W, tr, keep=x)
            return [act_to_nchw(self.out, prec)]
        self.acts = [act_from_nchw(x, prec) for x in xs]
        if k == "down":
            self.st = self._stage(DownStage(self.m))
            self.out = self.st.forward(prec, self.acts[0], tr)
            return [act_to_nchw(self.out, prec)]
        if k in ("up", "attention_up"):
            self.st = self._stage(UpStage(self.m, k == "attention_up"))
            self.out = self.st.forward(prec, self.acts[0], self.acts[1], tr)
            return [act_to_nchw(self.out, prec)]
        if k == "out_conv":
            self.st = self._stage(OutConvStage(self.m))
            return [self.st.forward(prec, self.acts[0])]
        if k == "attention_gate":
            g, x = self.acts
            self.st = self._stage(GateStage(self.m))
            self.st.forward(prec, g, x, tr)
            out = f32(x.N, x.C, x.H, x.W, device=x.data.device)
            L.call("unet_gated_to_nchw", prec.code, x.N, x.C, x.H, x.W, vp(x.data), vp(x.ab[0]), vp(x.ab[1]),
                   int(x.relu), vp(self.st.p), vp(self.st.psi_ab), vp(out), stream())
            return [out]
        raise ValueError(k)

    def backward(self, gouts, grads):
        prec = self.prec
        g = gouts[0]
        k = self.kind
        if k == "double_conv":
            x = self.xs[0]
            self.out.grad = grad_nchw_to_nhwc(g)
            self.out._grad_init = True
            if self.needs[0]:
                N, C, H, W = x.shape
                gx = f32(N, H, W, C, device=x.device)
                self.st.backward(prec, grads, {"mode": "f32", "out": gx, "accum": 0})
                return [grad_nhwc_to_nchw(gx)]
            self.st.backward(prec, grads, None)
            return [None]
        if k == "out_conv":
            self.st.backward(prec, g, grads)
        elif k == "attention_gate":
            gact, xact = self.acts
            d_xs = grad_nchw_to_nhwc(g)
            d_gup = f32(xact.N, xact.H, xact.W, gact.C, device=g.device)
            self.st.backward(prec, d_xs, grads, d_gup, 0)
            gg, acc = gact.grad_target()
            L.call("unet_upsample_bwd", gact.N, gact.C, gact.H, gact.W, xact.H, xact.W, 0, 0, xact.H, xact.W,
                   up_scale(gact.H, xact.H), up_scale(gact.W, xact.W), vp(d_gup), vp(gg), acc, stream())
        else:
            self.out.grad = grad_nchw_to_nhwc(g)
            self.out._grad_init = True
            self.st.backward(prec, grads)
        res = []
        for a, need in zip(self.acts, self.needs):
            if need and a.has_grad():
                res.append(grad_nhwc_to_nchw(a.grad))
            elif need:
                res.append(torch.zeros(a.N, a.C, a.H, a.W, device=a.data.device))
            else:
                res.append(None)
        return res


def run_module(module, kind: str, *inputs: torch.Tensor) -> torch.Tensor:
    for i in inputs:
        require_device(i)
    return _apply(_ModulePlan(module, kind), module, list(inputs))[0]
