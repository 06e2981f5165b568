"""Data-parallel training over RCCL.

The reference trains on one device and reaches its effective batch by gradient accumulation
(scripts/train.py:133-143); this path shards the batch over the GPUs of a node instead, one process
per GPU, with PyTorch's own `DistributedDataParallel` (backend "nccl" = RCCL on ROCm, over xGMI).
Nothing here re-implements DDP: the network's backward runs as one autograd node per reference module
(`unet._hip.functions`), so DDP's reducer marks a stage's parameters ready the moment that stage's
backward has finished and all-reduces full buckets while the remaining stages' kernels run.  The
backward visits outc, up4 .. up1, down4 .. down1, inc; the deep stages hold most of the 17.6 M
parameters, so only the last (small) bucket is exposed.

Gradient accumulation keeps the reference's loop: the first accum-1 micro-batches under
`ddp.no_sync()`, loss / accum on each, one synchronised backward, then clip + optimizer step.
"""

from __future__ import annotations

from typing import Optional

import torch
from torch.nn.parallel import DistributedDataParallel


def wrap_ddp(model: torch.nn.Module, device_id: Optional[int] = None, bucket_cap_mb: float = 25.0,
             broadcast_buffers: bool = True, **kwargs) -> DistributedDataParallel:
    """`DistributedDataParallel(model)` with the settings this path is measured with:
    `gradient_as_bucket_view=True` (no second copy of the 70 MB of gradients) and DDP's defaults
    otherwise.  `broadcast_buffers=False` keeps each rank's BN running statistics local (one collective
    less per forward; the reference's running statistics only matter in eval mode)."""
    return DistributedDataParallel(model, device_ids=[device_id] if device_id is not None else None,
                                   bucket_cap_mb=bucket_cap_mb, broadcast_buffers=broadcast_buffers,
                                   gradient_as_bucket_view=True, **kwargs)
