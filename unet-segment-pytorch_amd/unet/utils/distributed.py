"""Data-parallel gradient averaging overlapped with the HIP backward.

The reference trains data-parallel by batch (scripts/train.py:133-143 gradient accumulation; the
multi-GPU row of BASELINE.json wraps the model in DDP).  Under torch DDP our whole-network backward is
ONE autograd node, so every gradient becomes ready at the same instant and the ~70 MB all-reduce runs
after the last weight gradient, fully exposed.  `OverlappedGradSync` instead receives a callback from
`NetworkPlan.backward` after every stage (outc, up4 .. up1, down4 .. down1, inc): the gradients that
stage just produced are packed into a flat bucket and averaged with an async all-reduce (RCCL on ROCm,
running on its own stream) while the next stage's dgrad/wgrad kernels keep the CUs busy.  The deep
stages, which hold most of the parameters, finish first, so only the small `inc` bucket is exposed.

Semantics are DDP's: gradients are averaged over ranks; `no_sync()` skips the exchange for the
first accum-1 micro-batches and the synchronised micro-batch folds the locally accumulated `p.grad`
into its buckets (so the result equals DDP's).  Only the whole-network path (UNet / AttentionUNet
forward) calls the hooks; modules used standalone keep working under torch DDP.
"""

from __future__ import annotations

import contextlib
from typing import Dict, List, Optional

import torch
import torch.distributed as dist


class OverlappedGradSync:
    """Attach to a UNet / AttentionUNet: ``sync = OverlappedGradSync(model, bucket_cap_mb=32)``.

    Broadcasts rank 0's parameters (and buffers when ``broadcast_buffers``) at construction, as DDP
    does, so every replica starts from the same weights.
    """

    def __init__(self, model: torch.nn.Module, process_group=None, bucket_cap_mb: float = 32.0,
                 broadcast_buffers: bool = False):
        if not dist.is_initialized():
            raise RuntimeError("OverlappedGradSync needs an initialised torch.distributed process group")
        self.model = model
        self.pg = process_group
        self.world = dist.get_world_size(process_group)
        self.cap = int(bucket_cap_mb * (1 << 20))
        self.params = [p for p in model.parameters() if p.requires_grad]
        self._pid = {id(p): i for i, p in enumerate(self.params)}
        self.enabled = True
        self._reset()
        with torch.no_grad():
            for p in model.parameters():
                dist.broadcast(p.data, 0, group=process_group)
            if broadcast_buffers:
                for b in model.buffers():
                    dist.broadcast(b, 0, group=process_group)
        model._grad_sync = self

    # ---- DDP-compatible surface ----
    @contextlib.contextmanager
    def no_sync(self):
        prev, self.enabled = self.enabled, False
        try:
            yield
        finally:
            self.enabled = prev

    def __call__(self, *args, **kwargs):
        return self.model(*args, **kwargs)

    # ---- hooks called by NetworkPlan.backward ----
    def _reset(self):
        self._done = set()           # params already packed into a bucket this backward
        self._pending: List[torch.Tensor] = []
        self._pending_bytes = 0
        self._buckets = []           # (flat, [params], work)

    def stage_done(self, grads: Dict[torch.nn.Parameter, torch.Tensor], final: bool = False):
        """Pack every gradient that is now complete and not yet bucketed; launch full buckets."""
        if not self.enabled:
            return
        for p in grads:
            if id(p) in self._pid and id(p) not in self._done:
                self._done.add(id(p))
                self._pending.append(p)
                self._pending_bytes += p.numel() * 4
        if self._pending and (final or self._pending_bytes >= self.cap):
            self._launch(grads)

    def _launch(self, grads):
        ps = self._pending
        self._pending, self._pending_bytes = [], 0
        flat = torch.cat([grads[p].reshape(-1).float() for p in ps])
        off = 0
        for p in ps:
            n = p.numel()
            if p.grad is not None:          # locally accumulated micro-batches (no_sync)
                flat[off:off + n].add_(p.grad.reshape(-1))
            off += n
        # divide, then SUM: DDP's own default (and every backend has SUM; gloo has no AVG)
        flat.div_(self.world)
        work = dist.all_reduce(flat, group=self.pg, async_op=True)
        self._buckets.append((flat, ps, work))

    def finish(self, grads: Dict[torch.nn.Parameter, torch.Tensor]):
        """Wait for every bucket (stream-ordered on NCCL) and hand out views of the averaged buckets.

        Parameters whose local `p.grad` was folded into a bucket get `p.grad = None`, so autograd's
        accumulation assigns the averaged total instead of adding to it.
        """
        if not self.enabled:
            return
        self.stage_done(grads, final=True)
        for flat, ps, work in self._buckets:
            work.wait()
            off = 0
            for p in ps:
                n = p.numel()
                grads[p] = flat[off:off + n].view_as(p)
                if p.grad is not None:
                    p.grad = None
                off += n
        self._reset()


def grad_sync_of(model: torch.nn.Module) -> Optional[OverlappedGradSync]:
    return getattr(model, "_grad_sync", None)
