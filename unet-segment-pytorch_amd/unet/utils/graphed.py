"""A training micro-step captured into a HIP graph (opt-in; reference loop: scripts/train.py:127-143).

The eager step costs ~260 C-ABI calls plus the torch allocator and autograd bookkeeping on the host
(tools/cpu_overhead.py).  `GraphedTrainStep` captures forward -> loss -> backward -> clip_grad_norm_ ->
optimizer.step for one fixed batch shape into a hipGraph (torch.cuda.CUDAGraph drives it on ROCm) and
replays it per batch, so the host enqueues one graph launch per step and the GPU runs the identical
kernels.

Requirements, checked in __init__ (RuntimeError otherwise): a fixed input / target shape; a torch.optim.Adam
or AdamW with `capturable=True` in every parameter group (their fresh state is all zeros, which is what
undoing the warm-up restores); no loss scaler (its step reads the inf flag on the host) and no
DistributedDataParallel (its reducer is not captured here).

Hyperparameters: a replay runs the optimizer step exactly as captured.  A python-float hyperparameter
(lr, weight_decay, betas, eps, ...) is therefore frozen into the graph, and __call__ raises RuntimeError if
one has changed since capture instead of silently training with the old value.  To drive the learning rate
with a scheduler (scripts/train.py:353-370), give the optimizer a device tensor lr
(`AdamW(..., lr=torch.tensor(1e-3, device="cuda"), capturable=True)`): the fused step reads it from device
memory on every replay, and torch's LR schedulers update a tensor lr in place.

Gradients: the captured forward AND backward run with the model's parameters swapped for leaf aliases
(`p.detach().requires_grad_()`: the same storage, so the optimizer's in-place updates are what the next replay
reads; swapped in `module._parameters` for the duration of the step, as torch.func.functional_call does, but
around the backward too: the HIP stages look their parameters up again when their backward runs), and the
backward is torch.autograd.grad over those aliases; the results are assigned to `p.grad`.  That matters when the caller still holds an eager step's autograd graph (e.g. its
`loss`): a parameter's AccumulateGrad node lives as long as that graph and is bound to the stream it was
created on (the default stream); a capture whose graph reaches it makes the engine sync the capture stream
with the default stream, and torch.cuda.graph's capture_end then crashed the process (segfault, round 3 and
tests/test_gpu_graphed.py on the round-3 code; DESIGN.md §7, "GraphedTrainStep and a live eager graph").  The
aliases' own AccumulateGrad nodes are created inside the capture.  Values are identical: every parameter
gets exactly one gradient per step, which AccumulateGrad would only have stored.

Weights, BN running statistics and optimizer state live in their own tensors and are updated in place by
every replay; `loss` is a device tensor that every replay overwrites; `p.grad` are the step's gradients
(graph-owned memory, overwritten by every replay).
"""

from __future__ import annotations

import contextlib
from typing import Callable, Optional, Sequence

import torch


def _frozen_hyperparameters(optimizer: torch.optim.Optimizer):
    """Per parameter group: every non-tensor hyperparameter (a graph replay uses the value captured)."""
    return [{k: v for k, v in g.items() if k != "params" and not torch.is_tensor(v)} for g in optimizer.param_groups]


@contextlib.contextmanager
def _swapped_parameters(model: torch.nn.Module, aliases):
    """model's parameters replaced by `aliases` (name -> tensor) in their modules' _parameters, restored on exit;
    a parameter registered under several names gets its alias everywhere"""
    by_id = {id(p): aliases[n] for n, p in model.named_parameters() if n in aliases}
    saved = []
    try:
        for mod in model.modules():
            for k, p in list(mod._parameters.items()):
                if p is not None and id(p) in by_id:
                    saved.append((mod, k, p))
                    mod._parameters[k] = by_id[id(p)]
        yield
    finally:
        for mod, k, p in reversed(saved):
            mod._parameters[k] = p


class GraphedTrainStep:
    def __init__(self, model: torch.nn.Module, criterion: Callable, optimizer: torch.optim.Optimizer,
                 input_shape: Sequence[int], target_shape: Sequence[int], target_dtype=torch.int64,
                 clip_norm: Optional[float] = 1.0, warmup: int = 3, device="cuda"):
        if isinstance(model, torch.nn.parallel.DistributedDataParallel):
            raise RuntimeError("GraphedTrainStep: the captured step takes gradients on leaf aliases of the "
                               "parameters, so DDP's reducer hooks would never fire (each rank would train on "
                               "its own unsynchronised gradients); graph the single-GPU step, or use eager DDP")
        if not isinstance(optimizer, (torch.optim.Adam, torch.optim.AdamW)):
            raise RuntimeError(f"GraphedTrainStep: needs torch.optim.Adam / AdamW (capturable=True), got "
                               f"{type(optimizer).__name__}: undoing the warm-up steps restores Adam's fresh state")
        if not all(g.get("capturable", False) for g in optimizer.param_groups):
            raise RuntimeError("GraphedTrainStep: the optimizer must be built with capturable=True")
        self.model, self.criterion, self.optimizer = model, criterion, optimizer
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        self.params = [p for _, p in named]
        # leaf aliases (shared storage) the captured forward runs on: their AccumulateGrad nodes are the
        # capture's own, whatever eager graph of the model the caller keeps alive
        self.leaves = {n: p.detach().requires_grad_(True) for n, p in named}
        self.clip_norm = clip_norm
        self.x = torch.zeros(*input_shape, dtype=torch.float32, device=device)
        self.t = torch.zeros(*target_shape, dtype=target_dtype, device=device)
        # warm-up on a side stream (autograd / allocator / optimizer state settle before capture); the
        # warm-up steps' updates are undone in place afterwards, so the first replay is the first step
        snap = self._snapshot()
        s = torch.cuda.Stream(device=device)
        s.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.optimizer.zero_grad(set_to_none=True)
                self._body()
        torch.cuda.current_stream(device).wait_stream(s)
        self._restore(snap)
        self.optimizer.zero_grad(set_to_none=True)
        self.hyper = _frozen_hyperparameters(optimizer)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.loss = self._body()
        self.grads = [p.grad for p in self.params]

    def _state_tensors(self):
        return [v for st in self.optimizer.state.values() for v in st.values() if torch.is_tensor(v)]

    def _snapshot(self):
        """copies of every tensor a step updates in place: parameters, buffers (BN running statistics and
        counters) and the optimizer state that already exists"""
        ts = [p.data for p in self.model.parameters()] + list(self.model.buffers()) + self._state_tensors()
        return [(t, t.detach().clone()) for t in ts]

    def _restore(self, snap):
        """undo the warm-up: saved tensors get their values back; optimizer state created by the warm-up is
        zeroed, which is the fresh state of Adam / AdamW (step 0, zero moments)"""
        known = {id(t) for t, _ in snap}
        for t, v in snap:
            t.copy_(v)
        for t in self._state_tensors():
            if id(t) not in known:
                t.zero_()

    def _body(self) -> torch.Tensor:
        with _swapped_parameters(self.model, self.leaves):
            loss = self.criterion(self.model(self.x), self.t)
            # autograd.grad over the aliases, not backward(): see the module docstring
            grads = torch.autograd.grad(loss, list(self.leaves.values()), allow_unused=True)
        for p, g in zip(self.params, grads):
            p.grad = g
        if self.clip_norm is not None:
            torch.nn.utils.clip_grad_norm_(self.params, self.clip_norm)
        self.optimizer.step()
        return loss.detach()

    def __call__(self, x: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        """One step on (x, t); returns the step's loss (a device tensor overwritten by the next call)."""
        # the keys captured (a scheduler built later adds its own bookkeeping keys, e.g. initial_lr)
        diff = sorted({k for g, cap in zip(self.optimizer.param_groups, self.hyper) for k, v in cap.items()
                       if torch.is_tensor(g.get(k)) or g.get(k) != v})
        if diff or len(self.optimizer.param_groups) != len(self.hyper):
            raise RuntimeError(
                f"GraphedTrainStep: optimizer hyperparameter(s) {diff} changed since capture; a graph replay runs "
                "the captured values.  Pass lr as a device tensor (lr=torch.tensor(v, device='cuda')) so a "
                "scheduler updates it in place, or build a new GraphedTrainStep.")
        self.x.copy_(x, non_blocking=True)
        self.t.copy_(t, non_blocking=True)
        self.graph.replay()
        for p, g in zip(self.params, self.grads):
            p.grad = g
        return self.loss
