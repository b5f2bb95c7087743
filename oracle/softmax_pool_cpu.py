"""CPU restatement of the masked-softmax weighting ops beside the fused path (ORACLE).

TEST INFRASTRUCTURE ONLY (same rules as ``oracle/hybrid_cpu.py``): only
``tests/`` may import it, as the checker; the package never does.

Pinning: ``tests/golden/gen_golden.py`` runs the reference's own
FrameEncoder / LateFusion on seeded inputs and stores outputs and gradients;
``tests/test_oracle_golden.py`` checks these restatements against them.

  FrameEncoder.attention_pool            src/encoders.py:313-336
    scores = attention(frames)           :327
    masked_fill(mask == 0, -inf)         :329-330
    softmax over frames, nan_to_num(0)   :332-333
    pooled = sum(weights * frames)       :334
  FrameEncoder.forward                   src/encoders.py:261-310
    frame_processor (Linear-ReLU-Dropout) :241-243, :280
    projection (Linear-ReLU-Dropout-Linear) :253-258, :309
  LateFusion weighting                   src/fusion.py:228-245
    base = softmax(weight_logits)        :228-230
    w = base * mask; sums                :231-235
    where(sum > 0, w / (sum + 1e-8), 1/M) :237-240
    fused = sum(stacked * w)             :242-244
"""

from __future__ import annotations

from typing import Dict, Optional, Sequence

import torch
import torch.nn.functional as F


def attention_pool(frames: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor,
                   mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    scores = F.linear(frames, weight, bias)                       # (B, T, 1)
    if mask is not None:
        scores = scores.masked_fill(mask.unsqueeze(-1) == 0, float("-inf"))
    w = torch.nan_to_num(torch.softmax(scores, dim=1), nan=0.0, posinf=0.0, neginf=0.0)
    return (w * frames).sum(dim=1)


def frame_encoder(params: Dict[str, torch.Tensor], frames: torch.Tensor,
                  mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Eval-mode FrameEncoder with attention pooling (dropout = identity)."""
    h = F.relu(F.linear(frames, params["frame_processor.0.weight"], params["frame_processor.0.bias"]))
    pooled = attention_pool(h, params["attention.weight"], params["attention.bias"], mask)
    z = F.relu(F.linear(pooled, params["projection.0.weight"], params["projection.0.bias"]))
    return F.linear(z, params["projection.3.weight"], params["projection.3.bias"])


def late_weights(stacked: torch.Tensor, weight_logits: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """fused (B, C) from stacked per-modality logits (B, M, C)."""
    M = stacked.size(1)
    w = torch.softmax(weight_logits, dim=0).unsqueeze(0).expand(stacked.size(0), -1) * mask
    s = w.sum(dim=1, keepdim=True)
    w = torch.where(s > 0, w / (s + 1e-8), torch.full_like(w, 1.0 / M))
    return (stacked * w.unsqueeze(-1)).sum(dim=1)


def late_fusion(params: Dict[str, torch.Tensor], names: Sequence[str], feats: Dict[str, torch.Tensor],
                mask: torch.Tensor):
    """Eval-mode LateFusion: per-modality classifiers then the weighting."""
    per = {}
    for i, m in enumerate(names):
        x = feats[m] * mask[:, i:i + 1]
        z = F.relu(F.linear(x, params[f"classifiers.{m}.0.weight"], params[f"classifiers.{m}.0.bias"]))
        per[m] = F.linear(z, params[f"classifiers.{m}.3.weight"], params[f"classifiers.{m}.3.bias"])
    stacked = torch.stack([per[m] for m in names], dim=1)
    return late_weights(stacked, params["weight_logits"], mask), per
