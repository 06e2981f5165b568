"""A training micro-step captured into a HIP graph (opt-in; reference loop: scripts/train.py:127-143).

The eager step costs ~300 C-ABI calls plus the torch allocator and autograd bookkeeping on the host
(tools/cpu_overhead.py).  `GraphedTrainStep` captures forward -> loss -> backward -> clip_grad_norm_ ->
optimizer.step for one fixed batch shape into a hipGraph (torch.cuda.CUDAGraph drives it on ROCm) and
replays it per batch, so the host enqueues one graph launch per step and the GPU runs the identical
kernels.  Requirements, as for any whole-step graph capture in PyTorch: a fixed input / target shape, a
capturable optimizer (`capturable=True`, e.g. AdamW(fused=True, capturable=True)) whose fresh state is
all zeros (Adam / AdamW: the warm-up steps before capture are undone by restoring the weights and buffers
and zeroing the optimizer state they created), no loss scaler (its step reads the inf flag on the host)
and no DistributedDataParallel (its reducer is not captured here).
Weights, BN running statistics and optimizer state live in their own tensors and are updated in place by
every replay; `loss` is a device tensor that every replay overwrites.
"""

from __future__ import annotations

from typing import Callable, Optional, Sequence

import torch


class GraphedTrainStep:
    def __init__(self, model: torch.nn.Module, criterion: Callable, optimizer: torch.optim.Optimizer,
                 input_shape: Sequence[int], target_shape: Sequence[int], target_dtype=torch.int64,
                 clip_norm: Optional[float] = 1.0, warmup: int = 3, device="cuda"):
        self.model, self.criterion, self.optimizer = model, criterion, optimizer
        self.params = [p for p in model.parameters() if p.requires_grad]
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
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.loss = self._body()

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
        loss = self.criterion(self.model(self.x), self.t)
        loss.backward()
        if self.clip_norm is not None:
            torch.nn.utils.clip_grad_norm_(self.params, self.clip_norm)
        self.optimizer.step()
        return loss.detach()

    def __call__(self, x: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        """One step on (x, t); returns the step's loss (a device tensor overwritten by the next call)."""
        self.x.copy_(x, non_blocking=True)
        self.t.copy_(t, non_blocking=True)
        self.graph.replay()
        return self.loss
