"""FrameEncoder with its attention pooling on the HIP path.

Mirrors src/encoders.py::FrameEncoder (:210-336) of the reference: the same
constructor (frame_dim, hidden_dim=256, output_dim=128,
temporal_pooling="attention", dropout=0.1), attributes and state_dict keys
(frame_processor.0.*, attention.*, projection.0.*, projection.3.*), the same
forward(frames, mask=None) and the same errors:

  * ValueError("Unknown pooling: ...") at construction (:246-247);
  * ValueError("Expected 3D frame tensor, got shape ...") (:275-278);
  * ValueError("Unknown pooling strategy: ...") at run time (:306-309);
  * RuntimeError("Attention layer not initialized.") from attention_pool (:330-331).

attention_pool (:313-336) -- scores = attention(frames), -inf where mask == 0,
softmax over frames, nan_to_num, weighted sum -- runs forward and backward as
the HIP kernels behind mmf_attention_pool_forward / _backward
(csrc/softmax_pool.hip).  The frame MLP and the projection are nn.Linear
layers on PyTorch-ROCm (encoders are outside the fused path), and the
'average' / 'max' pooling branches stay plain torch (:288-305).  Only
FrameEncoder lives here: the reference's other encoders are not on the path.
"""

from __future__ import annotations

import os
import sys
from typing import Any, Optional, cast

import torch
import torch.nn as nn

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import mmf_native as _nat  # noqa: E402


class _AttentionPoolFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, frames, weight, bias, mask):
        L = _nat.lib()
        dev = frames.device
        B, T, D = frames.shape
        pooled = torch.empty(B, D, dtype=torch.float32, device=dev)
        weights = torch.empty(B, T, dtype=torch.float32, device=dev)
        rc = L.mmf_attention_pool_forward(B, T, D, frames.data_ptr(), weight.data_ptr(), bias.data_ptr(),
                                          _nat.ptr(mask), pooled.data_ptr(), weights.data_ptr(),
                                          _nat.stream_ptr(dev))
        _nat.check(rc, "FrameEncoder.attention_pool forward")
        ctx.save_for_backward(frames, weight, weights)
        ctx.bias_shape = bias.shape
        return pooled

    @staticmethod
    def backward(ctx, dpooled):
        L = _nat.lib()
        frames, weight, weights = ctx.saved_tensors
        dev = frames.device
        B, T, D = frames.shape
        dpooled = _nat.f32c(dpooled)
        dx = torch.empty_like(frames)
        dw = torch.empty(D, dtype=torch.float32, device=dev)
        db = torch.empty(1, dtype=torch.float32, device=dev)
        ws = torch.empty(L.mmf_attention_pool_workspace_bytes(B, D), dtype=torch.uint8, device=dev)
        rc = L.mmf_attention_pool_backward(B, T, D, frames.data_ptr(), weight.data_ptr(), weights.data_ptr(),
                                           dpooled.data_ptr(), dx.data_ptr(), dw.data_ptr(), db.data_ptr(),
                                           ws.data_ptr(), _nat.stream_ptr(dev))
        _nat.check(rc, "FrameEncoder.attention_pool backward")
        return dx, dw.view(1, D), db.view(ctx.bias_shape), None


def attention_pool(frames: torch.Tensor, attention: nn.Linear, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Learned-score softmax pooling over the frame axis (src/encoders.py:313-336) on HIP."""
    _nat.require_device(frames, "FrameEncoder input")
    frames = _nat.f32c(frames)
    m = None
    if mask is not None:
        m = mask.to(device=frames.device, dtype=torch.float32).contiguous()
        if m.shape != frames.shape[:2]:
            raise ValueError(f"mask shape {tuple(m.shape)} does not match frames {tuple(frames.shape[:2])}")
    return _AttentionPoolFunction.apply(frames, attention.weight, attention.bias, m)


class FrameEncoder(nn.Module):
    """Frame-level features -> video-level embedding (src/encoders.py:210-310)."""

    temporal_pooling: str
    attention: Optional[nn.Linear]

    def __init__(self, frame_dim: int, hidden_dim: int = 256, output_dim: int = 128,
                 temporal_pooling: str = "attention", dropout: float = 0.1):
        super().__init__()
        cast_self = cast(Any, self)
        cast_self.temporal_pooling = temporal_pooling
        self.frame_processor = nn.Sequential(nn.Linear(frame_dim, hidden_dim), nn.ReLU(), nn.Dropout(dropout))
        cast_self.attention = None
        if temporal_pooling == "attention":
            cast_self.attention = nn.Linear(hidden_dim, 1)
        elif temporal_pooling not in ("average", "max"):
            raise ValueError(f"Unknown pooling: {temporal_pooling}")
        self.projection = nn.Sequential(nn.Linear(hidden_dim, hidden_dim), nn.ReLU(), nn.Dropout(dropout),
                                        nn.Linear(hidden_dim, output_dim))

    def forward(self, frames: torch.Tensor, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        if frames.dim() != 3:
            raise ValueError(f"Expected 3D frame tensor, got shape {frames.shape}")
        processed = self.frame_processor(frames)
        if mask is not None:
            mask = mask.to(device=processed.device, dtype=processed.dtype)
        if self.temporal_pooling == "attention":
            pooled = self.attention_pool(processed, mask)
        elif self.temporal_pooling == "average":
            if mask is None:
                pooled = processed.mean(dim=1)
            else:
                wts = mask.unsqueeze(-1)
                pooled = (processed * wts).sum(dim=1) / wts.sum(dim=1).clamp_min(1e-8)
        elif self.temporal_pooling == "max":
            if mask is None:
                pooled = processed.max(dim=1).values
            else:
                pooled = processed.masked_fill(mask.unsqueeze(-1) == 0, float("-inf")).max(dim=1).values
                pooled = torch.nan_to_num(pooled, nan=0.0, neginf=0.0)
        else:
            raise ValueError(f"Unknown pooling strategy: {self.temporal_pooling}")
        return self.projection(pooled)

    def attention_pool(self, frames: torch.Tensor, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        if self.attention is None:
            raise RuntimeError("Attention layer not initialized.")
        return attention_pool(frames, self.attention, mask)
