"""Drop-in `attention` module: CrossModalAttention on MI355X HIP kernels.

Import surface of src/attention.py (tests/test_attention.py:22-27):
CrossModalAttention (the hot path), TemporalAttention and
PairwiseModalityAttention (compositions over the same HIP attention kernels)
and visualize_attention (matplotlib).

CrossModalAttention mirrors src/attention.py:16-146: same
constructor arguments, attributes (hidden_dim, num_heads, head_dim,
query_proj, key_proj, value_proj, out_proj, dropout, scale), state_dict keys
and forward(query, key, value, mask=None) -> (attended, attn_weights).

Compute path: include/mmfusion.h mmf_cma_forward / mmf_cma_backward
(libmmfusion.so, gfx950), reached as torch.ops.mmfusion.cma_fwd / cma_bwd
(mmf_ops.py custom ops: traceable by torch.compile without a graph break).
There is no CPU path: CPU tensors raise.
Differences from the reference, by design:
  * the returned attention weights are not differentiable (the reference's
    are; nothing in train/eval back-propagates through them);
  * dropout masks come from Philox4x32-10 on the device, not torch's RNG, so
    train-mode outputs are statistically (not bitwise) equal.
"""

from __future__ import annotations

import os
import sys
from typing import Any, Optional, Tuple, cast

import torch
import torch.nn as nn

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import mmf_native as _nat  # noqa: E402
import mmf_ops as _ops  # noqa: E402


@torch._dynamo.assume_constant_result
def _precision() -> int:
    """torch.get_float32_matmul_precision() as the C-ABI enum (mmf_native.matmul_precision), a
    constant of a compiled graph: like the matmuls inductor emits, a traced call keeps the
    precision that was set when it was traced."""
    return _nat.matmul_precision()


_RNG_COUNTER = [0]


def _new_rng_state() -> torch.Tensor:
    """{seed, offset} for the device Philox stream of one module.

    Derived from torch.initial_seed() and a construction counter, so it is
    reproducible under torch.manual_seed WITHOUT consuming torch's RNG: the
    nn.Linear initialisation stream stays identical to the reference's.
    """
    _RNG_COUNTER[0] += 1
    x = (torch.initial_seed() * 0x9E3779B97F4A7C15 + _RNG_COUNTER[0] * 0xBF58476D1CE4E5B9) & (2**64 - 1)
    x ^= x >> 31
    x = (x * 0x94D049BB133111EB) & (2**64 - 1)
    x ^= x >> 29
    return torch.tensor([x & (2**63 - 1), 0], dtype=torch.int64)


class CrossModalAttention(nn.Module):
    """Cross-modal attention: modality A attends to modality B (src/attention.py:16-66)."""

    hidden_dim: int
    num_heads: int
    head_dim: int
    query_proj: nn.Linear
    key_proj: nn.Linear
    value_proj: nn.Linear
    out_proj: nn.Linear
    dropout: nn.Dropout
    scale: float

    def __init__(self, query_dim: int, key_dim: int, hidden_dim: int = 256, num_heads: int = 4,
                 dropout: float = 0.1):
        super().__init__()
        head_dim = hidden_dim // num_heads
        cast_self = cast(Any, self)
        cast_self.hidden_dim = hidden_dim
        cast_self.num_heads = num_heads
        cast_self.head_dim = head_dim
        assert hidden_dim % num_heads == 0, (
            f"hidden_dim ({hidden_dim}) must be divisible by num_heads ({num_heads})")
        # same construction order as the reference => same init under a seed
        self.query_proj = nn.Linear(query_dim, hidden_dim)
        self.key_proj = nn.Linear(key_dim, hidden_dim)
        self.value_proj = nn.Linear(key_dim, hidden_dim)
        self.out_proj = nn.Linear(hidden_dim, hidden_dim)
        self.dropout = nn.Dropout(dropout)
        cast_self.scale = head_dim ** -0.5
        self.register_buffer("_rng_state", _new_rng_state(), persistent=False)

    def forward(self, query: torch.Tensor, key: torch.Tensor, value: torch.Tensor,
                mask: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """src/attention.py:68-146: (B,Dq)/(B,Lq,Dq) x (B,Dk)/(B,Lk,Dk) -> (attended, weights)."""
        B = query.size(0)
        squeeze_q = query.dim() == 2
        squeeze_k = key.dim() == 2
        q3 = query.unsqueeze(1) if squeeze_q else query
        k3 = key.unsqueeze(1) if squeeze_k else key
        v3 = value.unsqueeze(1) if value.dim() == 2 else value
        if q3.dim() != 3 or k3.dim() != 3 or v3.dim() != 3:
            raise RuntimeError("CrossModalAttention expects 2-D or 3-D query/key/value tensors")
        for t, nm in ((q3, "query"), (k3, "key"), (v3, "value")):
            _nat.require_device(t, nm)
        if k3.shape[:2] != v3.shape[:2]:
            raise RuntimeError(f"key {tuple(k3.shape)} and value {tuple(v3.shape)} shapes differ")
        if q3.size(-1) != self.query_proj.in_features or k3.size(-1) != self.key_proj.in_features \
                or v3.size(-1) != self.value_proj.in_features:
            raise RuntimeError("CrossModalAttention: feature dims do not match the projections")
        lq, lk = q3.size(1), k3.size(1)
        mask_mode = 0
        m = None
        if mask is not None:
            m = mask.to(device=q3.device, dtype=torch.float32)
            if m.dim() == 1:
                mask_mode = 1
                if m.numel() != B:
                    raise RuntimeError(f"1-D mask must have {B} entries, got {m.numel()}")
            elif m.dim() == 2 and m.shape == (B, lk):
                mask_mode = 2
            else:
                raise RuntimeError(f"mask of shape {tuple(m.shape)} does not broadcast to (B, Lk)")
            m = m.contiguous()
        idesc = [B, lq, lk, self.query_proj.in_features, self.key_proj.in_features, self.hidden_dim,
                 self.num_heads, mask_mode, int(self.training), _precision()]
        attended, attn, _saved, rng_next = torch.ops.mmfusion.cma_fwd(
            idesc, float(self.dropout.p), self._rng_state, _nat.f32c(q3), _nat.f32c(k3), _nat.f32c(v3), m,
            [self.query_proj.weight, self.query_proj.bias, self.key_proj.weight, self.key_proj.bias,
             self.value_proj.weight, self.value_proj.bias, self.out_proj.weight, self.out_proj.bias])
        self._rng_state.copy_(rng_next)     # the device Philox stream advanced by one call
        attn = attn.detach()
        if squeeze_q:
            attended = attended.squeeze(1)
        if squeeze_k:
            attn = attn[:, :, :, :1]
        return attended, attn


class TemporalAttention(CrossModalAttention):
    """Self-attention over the time steps of one sequence (src/attention.py:149-281).

    Same parameters as the reference (query/key/value/out_proj, feature_dim ->
    hidden_dim) and the same forward(sequence, mask=None) -> (attended,
    weights).  The attention itself runs on the CrossModalAttention HIP kernels
    with query = key = value = sequence and a per-key mask; the reference's
    post-mask multiply (src/attention.py:245-248) keeps its exact broadcasting,
    including the extra leading dims it produces for a 2-D mask.
    """

    feature_dim: int

    def __init__(self, feature_dim: int, hidden_dim: int = 256, num_heads: int = 4, dropout: float = 0.1):
        super().__init__(feature_dim, feature_dim, hidden_dim=hidden_dim, num_heads=num_heads, dropout=dropout)
        cast(Any, self).feature_dim = feature_dim

    def forward(self, sequence: torch.Tensor,  # type: ignore[override]
                mask: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        if sequence.dim() != 3:
            raise RuntimeError(f"TemporalAttention expects (batch, seq_len, feature_dim), got {tuple(sequence.shape)}")
        B, L = sequence.size(0), sequence.size(1)
        key_mask = None
        if mask is not None:
            m = mask.to(sequence.device)
            if m.dim() == 1:          # one mask over the time axis, shared by the batch (:239-240)
                m = m.unsqueeze(0)
            key_mask = m.expand(B, L).to(torch.float32).contiguous()
        attended, weights = super().forward(sequence, sequence, sequence, mask=key_mask)
        if mask is not None:
            m = mask.to(sequence.device)
            if m.dim() == 1:
                m = m.unsqueeze(0)
            attended = attended * m.unsqueeze(1).unsqueeze(2).unsqueeze(-1)
        return attended, weights

    def pool_sequence(self, sequence: torch.Tensor, attention_weights: torch.Tensor) -> torch.Tensor:
        """Attention-weighted pooling over time (src/attention.py:253-281): the mean
        over heads and queries of the weights, renormalised, applied to the sequence."""
        if attention_weights.dim() != 4:
            raise ValueError(f"Expected attention weights with 4 dims, got {attention_weights.shape}")
        w = attention_weights.mean(dim=(1, 2))                         # (B, L)
        w = w / (w.sum(dim=1, keepdim=True) + 1e-8)
        return torch.bmm(w.unsqueeze(1), sequence).squeeze(1)


class PairwiseModalityAttention(nn.Module):
    """Attention between every ordered pair of modalities (src/attention.py:284-424).

    Per-modality Linear -> ReLU -> Dropout projections, a CrossModalAttention
    (HIP kernels) for each present "{q}_to_{k}" pair keyed by the key
    modality's mask column, then the mean of each modality's list scaled by its
    mask.  Returns (attended_features, attention_maps) like the reference.
    """

    modality_names: list
    num_modalities: int
    hidden_dim: int

    def __init__(self, modality_dims, hidden_dim: int = 256, num_heads: int = 4, dropout: float = 0.1):
        super().__init__()
        dims = dict(modality_dims)
        cast_self = cast(Any, self)
        cast_self.modality_names = list(dims)
        cast_self.num_modalities = len(dims)
        cast_self.hidden_dim = hidden_dim
        self.projections = nn.ModuleDict({
            m: nn.Sequential(nn.Linear(d, hidden_dim), nn.ReLU(), nn.Dropout(dropout)) for m, d in dims.items()})
        self.attention_layers = nn.ModuleDict({
            f"{q}_to_{k}": CrossModalAttention(hidden_dim, hidden_dim, hidden_dim=hidden_dim, num_heads=num_heads,
                                               dropout=dropout)
            for q in dims for k in dims if q != k})

    def forward(self, modality_features, modality_mask: Optional[torch.Tensor] = None):
        if not self.modality_names:
            raise ValueError("No modalities provided for PairwiseModalityAttention.")
        first = modality_features[self.modality_names[0]]
        B, dev, dt = first.size(0), first.device, first.dtype
        if modality_mask is None:
            mask = torch.ones(B, self.num_modalities, device=dev, dtype=dt)
        else:
            mask = modality_mask.to(device=dev, dtype=dt)
        proj = {m: self.projections[m](modality_features[m].to(dev)) for m in self.modality_names}
        lists = {m: [proj[m]] for m in self.modality_names}
        maps = {}
        for q in self.modality_names:
            for k in self.modality_names:
                key = f"{q}_to_{k}"
                if q == k or key not in self.attention_layers:
                    continue
                att, w = self.attention_layers[key](proj[q], proj[k], proj[k],
                                                    mask=mask[:, self.modality_names.index(k)])
                lists[q].append(att)
                maps[key] = w
        out = {}
        for i, m in enumerate(self.modality_names):
            out[m] = torch.stack(lists[m], dim=0).mean(dim=0) * mask[:, i].unsqueeze(-1)
        return out, maps


def visualize_attention(attention_weights, modality_names, save_path=None) -> None:
    """Heat map of attention weights (src/attention.py:427-480): leading dims are
    averaged down to a (queries, keys) matrix; saved to `save_path` or shown."""
    from pathlib import Path

    import matplotlib.pyplot as plt
    import numpy as np

    t = attention_weights.detach().float().cpu() if torch.is_tensor(attention_weights) \
        else torch.as_tensor(attention_weights, dtype=torch.float32)
    while t.dim() < 2:
        t = t.unsqueeze(0)
    while t.dim() > 2:
        t = t.mean(dim=0)
    grid = t.numpy()
    nq, nk = grid.shape
    fig, ax = plt.subplots(figsize=(4 + 0.5 * nk, 4))
    im = ax.imshow(grid, cmap="viridis", aspect="auto")
    ax.set_xticks(np.arange(nk))
    ax.set_yticks(np.arange(nq))
    ax.set_xticklabels(list(modality_names)[:nk], rotation=45, ha="right")
    ax.set_yticklabels(list(modality_names)[:nq])
    ax.set_xlabel("Key Modality")
    ax.set_ylabel("Query Modality")
    ax.set_title("Cross-Modal Attention Weights")
    plt.colorbar(im, ax=ax, fraction=0.046, pad=0.04)
    plt.tight_layout()
    if save_path is not None:
        out = Path(save_path)
        out.parent.mkdir(parents=True, exist_ok=True)
        fig.savefig(out, dpi=300, bbox_inches="tight")
        plt.close(fig)
    else:
        plt.show()
