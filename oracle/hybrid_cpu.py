"""CPU restatement of the cross-modal attention fusion hot path (the ORACLE).

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker / the timed CPU baseline.  The product path (the package's
``fusion.py`` / ``attention.py``) never imports it and has no CPU fallback.

Pinning: validated against golden fixtures produced by the reference itself
(``tests/golden/gen_golden.py`` imports /root/reference/src and records its
outputs; see ``tests/test_oracle_golden.py``).

This is a from-scratch functional restatement in plain torch-CPU ops (autograd
provides the backward).  Each step cites the reference line it follows:

  CrossModalAttention.forward            src/attention.py:68-146
    q/k/v projections                    :104-106
    (B,L,h,hd) -> (B,h,L,hd)              :108-116
    scores = (q @ k^T) * hd**-0.5         :118, scale :66
    1-D mask -> (B,1,1,1); 2-D -> (B,1,1,Lk); masked_fill(mask==0,-inf)  :120-124
    softmax -> nan_to_num(0) -> dropout   :126-130
    attn @ v -> (B,Lq,H) -> out_proj      :132-140
    squeeze for 2-D query / key           :142-146
  HybridFusion.forward                   src/fusion.py:331-427
    default mask / dtype cast            :352-362
    P_m = Drop(ReLU(Lin(Drop(X*mask))))  :364-374, projections :291-298
    pairwise attention, skip deleted     :383-404
    agg = mean(stack(list)) * mask       :406-408
    compute_adaptive_weights             :429-479
    fused = sum(stack * w)               :413-418; classifier :323-328,419
  Sequence mode (not in the reference): 3-D (B,L_m,D_m) inputs,
  agg mean-pooled over L_m before the weighting; at L=1 identical to the
  reference (checked bit-for-bit by gen_golden.py).
"""

from __future__ import annotations

from typing import Dict, List, Mapping, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F


def _dropout(x: torch.Tensor, p: float, train: bool, gen, site: int = 0) -> torch.Tensor:
    """nn.Dropout(p).  `gen` is a torch.Generator (CPU RNG) or a callable
    (site, tensor) -> keep mask, used by the tests to replay the device's
    Philox masks so train-mode outputs can be compared exactly."""
    if not train or p <= 0.0:
        return x
    if callable(gen):
        keep = gen(site, x).to(x.dtype)
        return x * keep / (1.0 - p)
    # the same ATen ops as nn.Dropout's CPU path (at::dropout: bernoulli_(1 - p) noise scaled
    # by 1 / (1 - p), times the input), so the timed CPU baseline pays what the reference pays
    noise = torch.empty_like(x).bernoulli_(1.0 - p, generator=gen)
    noise.div_(1.0 - p)
    return x * noise


# dropout site ids (mirror of the device's Philox streams, csrc/mmf_internal.h)
SITE_IN, SITE_PROJ, SITE_ATTN, SITE_CLS = 0x100, 0x200, 0x300, 0x400


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return x.matmul(w.t()) + b


def cma_forward(params: Mapping[str, torch.Tensor], prefix: str, query: torch.Tensor,
                key: torch.Tensor, value: torch.Tensor, num_heads: int,
                mask: Optional[torch.Tensor] = None, p: float = 0.0, train: bool = False,
                gen=None, site: int = SITE_ATTN) -> Tuple[torch.Tensor, torch.Tensor]:
    """src/attention.py:68-146."""
    B = query.shape[0]
    sq = query.dim() == 2
    sk = key.dim() == 2
    if sq:
        query = query.unsqueeze(1)
    if sk:
        key = key.unsqueeze(1)
    if value.dim() == 2:
        value = value.unsqueeze(1)
    Lq, Lk = query.shape[1], key.shape[1]
    W = lambda n: (params[f"{prefix}{n}.weight"], params[f"{prefix}{n}.bias"])  # noqa: E731
    q = linear(query, *W("query_proj"))
    k = linear(key, *W("key_proj"))
    v = linear(value, *W("value_proj"))
    H = q.shape[-1]
    hd = H // num_heads
    q = q.reshape(B, Lq, num_heads, hd).permute(0, 2, 1, 3)
    k = k.reshape(B, Lk, num_heads, hd).permute(0, 2, 1, 3)
    v = v.reshape(B, Lk, num_heads, hd).permute(0, 2, 1, 3)
    s = q.matmul(k.transpose(-1, -2)) * (hd ** -0.5)
    if mask is not None:
        mk = mask.reshape(B, 1) if mask.dim() == 1 else mask
        s = s.masked_fill((mk == 0).reshape(B, 1, 1, -1), float("-inf"))
    a = torch.softmax(s, dim=-1)
    a = torch.nan_to_num(a, nan=0.0, posinf=0.0, neginf=0.0)
    a = _dropout(a, p, train, gen, site)
    o = a.matmul(v).permute(0, 2, 1, 3).reshape(B, Lq, H)
    o = linear(o, *W("out_proj"))
    if sq:
        o = o.squeeze(1)
    if sk:
        a = a[:, :, :, :1]
    return o, a


def adaptive_weights(params: Mapping[str, torch.Tensor], names: Sequence[str],
                     feats: Mapping[str, torch.Tensor], mask: torch.Tensor) -> torch.Tensor:
    """src/fusion.py:429-479."""
    scores = torch.cat([linear(feats[m], params[f"gating_layers.{m}.weight"],
                               params[f"gating_layers.{m}.bias"]) for m in names], dim=1)
    mask = mask.to(scores.dtype)
    w = torch.softmax(scores.masked_fill(mask <= 0, float("-inf")), dim=1)
    w = torch.nan_to_num(w, nan=0.0, posinf=0.0, neginf=0.0) * mask
    sw = w.sum(dim=1, keepdim=True)
    ms = mask.sum(dim=1, keepdim=True)
    fb = torch.where(ms > 0, mask / (ms + 1e-8), torch.full_like(mask, 1.0 / len(names)))
    return torch.where(sw > 0, w / (sw + 1e-8), fb)


def pairs_present(names: Sequence[str], params: Mapping[str, torch.Tensor]) -> List[Tuple[str, str]]:
    out = []
    for q in names:
        for k in names:
            if q != k and f"attention_modules.{q}_to_{k}.query_proj.weight" in params:
                out.append((q, k))
    return out


def _relu(z: torch.Tensor, layer: str, relu_gate) -> torch.Tensor:
    """torch.relu, or with the slope given where relu_gate[layer] selects (see hybrid_forward)."""
    if relu_gate is None or layer not in relu_gate:
        return torch.relu(z)
    sel, pos = relu_gate[layer]
    return torch.where(sel.reshape(z.shape), z * pos.reshape(z.shape).to(z.dtype), torch.relu(z))


def hybrid_forward(params: Mapping[str, torch.Tensor], names: Sequence[str],
                   feats: Mapping[str, torch.Tensor], mask: Optional[torch.Tensor],
                   num_heads: int, p: float = 0.0, train: bool = False, gen=None,
                   taps: Optional[dict] = None, relu_gate: Optional[Mapping[str, tuple]] = None):
    """HybridFusion forward (src/fusion.py:331-427) + sequence-mode pooling.

    Returns (logits, info) with info = {attention_maps, fusion_weights, pooled}.
    ``taps`` (a dict, tests only) receives each ReLU's input ``z/<layer>``, its output
    ``a/<layer>`` (gradient retained) and the layer's input ``in/<layer>`` (layers: the modality
    names and "cls").  ``relu_gate`` (tests only) maps a layer to ``(sel, pos)``, two bool
    tensors of z's shape: where ``sel``, the ReLU passes z with slope ``pos`` instead of taking
    the sign of this computation's own z.  That is the kink of ReLU: for |z| within rounding of
    0, relu'(z) may differ between two fp32 summation orders, so a test hands the oracle the
    device's decision there (and only there) and keeps the plain bound everywhere.
    """
    ref = feats[names[0]]
    B = ref.shape[0]
    if mask is None:
        mask = torch.ones(B, len(names), dtype=ref.dtype)
    mask = mask.to(ref.dtype)
    P: Dict[str, torch.Tensor] = {}
    for i, m in enumerate(names):
        x = feats[m]
        mk = mask[:, i].reshape(-1, *([1] * (x.dim() - 1)))
        xd = _dropout(x * mk, p, train, gen, SITE_IN + i)
        z = linear(xd, params[f"projections.{m}.0.weight"], params[f"projections.{m}.0.bias"])
        a = _relu(z, m, relu_gate)
        if taps is not None:
            taps[f"in/{m}"], taps[f"z/{m}"], taps[f"a/{m}"] = xd.detach(), z.detach(), a
            if a.requires_grad:
                a.retain_grad()
        P[m] = _dropout(a, p, train, gen, SITE_PROJ + i)
    lists = {m: [P[m]] for m in names}
    maps: Dict[str, torch.Tensor] = {}
    for g, (q, k) in enumerate(pairs_present(names, params)):
        ki = names.index(k)
        att, a = cma_forward(params, f"attention_modules.{q}_to_{k}.", P[q], P[k], P[k],
                             num_heads, mask=mask[:, ki], p=p, train=train, gen=gen, site=SITE_ATTN + g)
        lists[q].append(att)
        maps[f"{q}_to_{k}"] = a
    pooled = []
    for i, m in enumerate(names):
        agg = torch.stack(lists[m], 0).mean(0)
        agg = agg * mask[:, i].reshape(-1, *([1] * (agg.dim() - 1)))
        pooled.append(agg.mean(1) if agg.dim() == 3 else agg)
    pooled_t = torch.stack(pooled, 1)
    w = adaptive_weights(params, names, {m: pooled[i] for i, m in enumerate(names)}, mask)
    fused = (pooled_t * w.unsqueeze(-1)).sum(1)
    zc = linear(fused, params["classifier.0.weight"], params["classifier.0.bias"])
    ac = _relu(zc, "cls", relu_gate)
    if taps is not None:
        taps["in/cls"], taps["z/cls"], taps["a/cls"] = fused.detach(), zc.detach(), ac
        if ac.requires_grad:
            ac.retain_grad()
    h = _dropout(ac, p, train, gen, SITE_CLS)
    logits = linear(h, params["classifier.3.weight"], params["classifier.3.bias"])
    return logits, {"attention_maps": maps, "fusion_weights": w, "pooled": pooled_t}


def cross_entropy_ls(logits: torch.Tensor, labels: torch.Tensor, smoothing: float = 0.05) -> torch.Tensor:
    """nn.CrossEntropyLoss(label_smoothing=0.05) as the caller uses it (src/train.py:185-186,310)."""
    return F.cross_entropy(logits, labels, label_smoothing=smoothing)


def hybrid_train_step(params: Dict[str, torch.Tensor], names: Sequence[str],
                      feats: Mapping[str, torch.Tensor], mask: torch.Tensor,
                      labels: torch.Tensor, num_heads: int, p: float,
                      gen: Optional[torch.Generator] = None) -> torch.Tensor:
    """One CPU step of the metric's unit: forward + CE(label_smoothing) + backward.

    ``params`` must be leaf tensors with requires_grad; input grads are produced
    too when the features require grad (SURVEY §8d step definition).
    """
    logits, _ = hybrid_forward(params, names, feats, mask, num_heads, p=p, train=True, gen=gen)
    loss = cross_entropy_ls(logits, labels)
    loss.backward()
    return loss.detach()
