"""Inference path on the device (reference scripts/predict.py).

* `preprocess_images`: predict.py:100-135 (`preprocess_image`) for a batch — PIL BILINEAR resize of the
  8-bit slice to img_size, /255, (x - mean) / std — as byte kernels with Pillow's tables.
* `postprocess_masks`: predict.py:138-165 (`postprocess_mask`) — softmax over the classes,
  p[cls] > threshold -> 255 / 0, PIL NEAREST resize to the original size — one kernel, no host copy of
  the probabilities.
* `GraphedPredictor`: the eval-mode forward (BN with running statistics, applied inside the next conv's
  loader; no batch statistics, no backward state) captured once into a HIP graph and replayed per batch,
  so a batch-1 prediction costs one graph launch instead of ~150 kernel launches from Python.
* `predict_masks`: predict_single (predict.py:206-240) for a batch: preprocess -> graph replay ->
  postprocess, plus the tumour ratio (mask > 127).mean().
"""

from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch

from .._hip import lib as L
from .._hip.runtime import require_device, stream, vp
from .gpu_pipeline import _Tables, resize_bilinear_u8

_TABLES = {}


def _tables(device) -> _Tables:
    key = str(device)
    if key not in _TABLES:
        _TABLES[key] = _Tables(device)
    return _TABLES[key]


def preprocess_images(images: torch.Tensor, img_size: int = 256, mean: float = 0.5, std: float = 0.5,
                      device="cuda") -> torch.Tensor:
    """uint8 (N, h, w) -> fp32 (N, 1, img_size, img_size), as preprocess_image (predict.py:100-135)."""
    x = torch.as_tensor(images)
    if x.dim() == 2:
        x = x[None]
    if x.dtype != torch.uint8 or x.dim() != 3:
        raise RuntimeError(f"expected uint8 images (N, H, W), got {x.dtype} {tuple(x.shape)}")
    x = x.to(device, non_blocking=True).contiguous()
    require_device(x, "images")
    N = x.shape[0]
    r, _ = resize_bilinear_u8(x, img_size, img_size, _tables(x.device), roundtrip=False)
    out = torch.empty(N, 1, img_size, img_size, dtype=torch.float32, device=x.device)
    L.call("unet_slice_finish", N, img_size, img_size, vp(r), 0, 0, 0, None, None, None, None, float(mean),
           float(std), vp(out), None, stream())
    return out


def postprocess_masks(logits: torch.Tensor, out_size: Optional[Tuple[int, int]] = None, threshold: float = 0.5,
                      cls: int = 1) -> torch.Tensor:
    """uint8 (N, H', W') masks of 0 / 255; out_size = (W', H') as PIL's size (predict.py:142, 162)."""
    require_device(logits, "logits")
    z = logits.detach()
    if z.dtype != torch.float32 or not z.is_contiguous():
        z = z.float().contiguous()
    N, K, H, W = z.shape
    ow, oh = (W, H) if out_size is None else (int(out_size[0]), int(out_size[1]))
    t = _tables(z.device)
    out = torch.empty(N, oh, ow, dtype=torch.uint8, device=z.device)
    L.call("unet_postprocess_mask", N, K, H, W, vp(z), int(cls), float(threshold), oh, ow, vp(t.nearest(H, oh)),
           vp(t.nearest(W, ow)), vp(out), stream())
    return out


class GraphedPredictor:
    """model.eval() forward for a fixed input shape, captured into a HIP graph (torch.cuda.CUDAGraph
    drives hipGraph on ROCm).  Parameters and BN buffers are read at replay time, so weight updates
    (e.g. a reloaded checkpoint copied into the same tensors) are picked up without re-capturing."""

    def __init__(self, model: torch.nn.Module, input_shape: Sequence[int], device="cuda", warmup: int = 2):
        self.model = model.eval()
        self.x = torch.zeros(*input_shape, dtype=torch.float32, device=device)
        s = torch.cuda.Stream(device=device)
        s.wait_stream(torch.cuda.current_stream(device))
        with torch.no_grad(), torch.cuda.stream(s):
            for _ in range(warmup):
                self.model(self.x)
        torch.cuda.current_stream(device).wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(self.graph):
            self.out = self.model(self.x)

    def __call__(self, x: torch.Tensor, copy: bool = True) -> torch.Tensor:
        """Logits of x.  copy=False returns the graph's static output buffer itself, which the next call
        overwrites (no extra 8-byte-per-logit copy); the default returns an independent tensor."""
        self.x.copy_(x, non_blocking=True)
        self.graph.replay()
        return self.out.clone() if copy else self.out


def predict_masks(model: torch.nn.Module, images: torch.Tensor, img_size: int = 256, threshold: float = 0.5,
                  predictor: Optional[GraphedPredictor] = None):
    """predict_single (predict.py:206-240) for a batch of uint8 slices of one original size: returns
    (uint8 masks at the original size, tumour ratio per image)."""
    x = torch.as_tensor(images)
    if x.dim() == 2:
        x = x[None]
    N, h, w = x.shape
    dev = next(model.parameters()).device
    inp = preprocess_images(x, img_size, device=dev)
    if predictor is not None:
        logits = predictor(inp)
    else:
        with torch.no_grad():
            logits = model.eval()(inp)
    masks = postprocess_masks(logits, (w, h), threshold)
    ratio = (masks > 127).float().mean((1, 2))
    return masks, ratio
