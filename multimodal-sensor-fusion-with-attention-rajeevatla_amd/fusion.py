"""Drop-in `fusion` module: HybridFusion on MI355X HIP kernels.

Mirrors src/fusion.py of the reference so `from fusion import HybridFusion,
build_fusion_model` (src/train.py:25) resolves here unchanged:

  * HybridFusion(modality_dims, hidden_dim=256, num_classes=11, num_heads=4,
    dropout=0.1) with the reference's attributes and state_dict keys
    (projections.{m}.0.*, attention_modules.{q}_to_{k}.{query,key,value,out}_proj.*,
    gating_layers.{m}.*, classifier.{0,3}.*), src/fusion.py:248-329;
  * forward(modality_features, modality_mask=None, return_attention=False)
    -> logits | (logits, {"attention_maps", "fusion_weights"}), src/fusion.py:331-427,
    with the reference's errors raised before any kernel launch;
  * compute_adaptive_weights(features, mask), src/fusion.py:429-479, differentiable
    (gradients reach the features and gating_layers, as in the reference);
  * modality masks are validated on the host before any launch: (B, M), or (1, M)
    broadcast over the batch as the reference's indexing allows; other shapes raise;
  * build_fusion_model(fusion_type, modality_dims, num_classes, **kw), src/fusion.py:485-515.

The whole fused step (projections, pairwise Q/K/V, QK^T softmax attn.V,
out_proj, aggregation, gating softmax, weighted sum, classifier) runs as HIP
kernels through include/mmfusion.h (mmf_hybrid_forward / mmf_hybrid_backward),
reached as the torch operators torch.ops.mmfusion.hybrid_fwd / hybrid_bwd
(mmf_ops.py: custom ops with fake kernels and an autograd formula, so
torch.compile(..., mode="reduce-overhead", fullgraph=True) -- the reference
trainer's compile, src/train.py:193-231 -- traces the module without a graph break);
inputs may be 2-D (B, D_m) (reference semantics) or 3-D (B, L_m, D_m)
(sequence mode: each modality's aggregate is mean-pooled over L_m before the
weighting; identical to the reference at L = 1).  No CPU path exists: CPU
tensors raise.  EarlyFusion is plain-PyTorch plumbing kept only so the import
surface matches; LateFusion's per-modality classifiers are nn.Linear layers
and its masked softmax weighting (src/fusion.py:228-245) runs on HIP.
"""

from __future__ import annotations

import ctypes
import os
import sys
from typing import Any, Dict, List, Optional, Tuple, cast

import torch
import torch.nn as nn

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import mmf_native as _nat  # noqa: E402
import mmf_ops as _ops  # noqa: E402
from attention import CrossModalAttention, _new_rng_state, _precision  # noqa: E402

_SHAPE = torch.Tensor.shape.__get__   # (x.shape as a C-level callable: map() over the inputs)

# Bumped whenever any module registers a Parameter (nn.Module.__setattr__ / register_parameter):
# HybridFusion's cached operator parameter list (_op_params) is only valid for the Parameter
# objects it was built from.  One integer compare per forward; training steps register nothing.
_PARAM_GEN = [0]


def _param_registered(module, name, param):
    _PARAM_GEN[0] += 1


torch.nn.modules.module.register_module_parameter_registration_hook(_param_registered)


# --------------------------------------------------------------------------
# Early fusion (plumbing, torch) and Late fusion (torch classifiers + HIP weighting).
# --------------------------------------------------------------------------
def _check_mask(mask: torch.Tensor, batch: int, num_modalities: int, what: str) -> torch.Tensor:
    """Validate a modality mask before its pointer reaches a kernel (the C-ABI reads a
    contiguous (B, M) array).

    The reference indexes ``modality_mask[:, idx]`` and broadcasts it against (B, .)
    tensors (src/fusion.py:371-373,408,462-467), so a (B, M) mask and a (1, M) mask
    (broadcast over the batch) work there and every other shape raises (IndexError
    or a broadcast RuntimeError).  Here a (1, M) mask is expanded to (B, M); any
    other shape raises RuntimeError before a launch.
    """
    if mask.dim() != 2 or mask.size(1) != num_modalities or mask.size(0) not in (batch, 1):
        raise RuntimeError(f"{what}: modality_mask must have shape ({batch}, {num_modalities}) "
                           f"(or (1, {num_modalities})), got {tuple(mask.shape)}")
    if mask.size(0) != batch:
        mask = mask.expand(batch, num_modalities)
    return mask


def _mask_or_ones(features, names, mask, what="fusion"):
    first = features[names[0]]
    if mask is None:
        return torch.ones(first.size(0), len(names), device=first.device, dtype=first.dtype)
    mask = mask.to(device=first.device, dtype=first.dtype)
    return _check_mask(mask, first.size(0), len(names), what)


class EarlyFusion(nn.Module):
    """Concatenate masked encoder outputs, then an MLP (src/fusion.py:17-123)."""

    def __init__(self, modality_dims: Dict[str, int], hidden_dim: int = 256, num_classes: int = 11,
                 dropout: float = 0.1):
        super().__init__()
        dims = dict(modality_dims)
        cast_self = cast(Any, self)
        cast_self.modality_names = list(dims)
        cast_self.modality_dims = dims
        cast_self.num_classes = num_classes
        cast_self.hidden_dim = hidden_dim
        width = sum(dims.values())
        if width == 0:
            self.fusion = nn.Identity()
        else:
            self.fusion = nn.Sequential(
                nn.Linear(width, hidden_dim), nn.ReLU(), nn.Dropout(dropout),
                nn.Linear(hidden_dim, hidden_dim), nn.ReLU(), nn.Dropout(dropout),
                nn.Linear(hidden_dim, num_classes))

    def forward(self, modality_features, modality_mask=None):
        if not self.modality_names:
            raise ValueError("No modalities configured for EarlyFusion.")
        mask = _mask_or_ones(modality_features, self.modality_names, modality_mask, "EarlyFusion")
        parts = []
        for i, name in enumerate(self.modality_names):
            if name not in modality_features:
                raise KeyError(f"Missing features for modality '{name}' in EarlyFusion forward pass.")
            x = modality_features[name]
            if x.dim() != 2:
                raise ValueError(f"Expected 2D tensor for modality '{name}', got shape {x.shape}.")
            parts.append(x.to(mask.device) * mask[:, i:i + 1])
        return self.fusion(torch.cat(parts, dim=1))


def _late_weights(stacked: torch.Tensor, weight_logits: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """LateFusion's masked softmax weighting (src/fusion.py:228-245) on HIP
    (torch.ops.mmfusion.late_weights_fwd: mmf_late_fusion_forward / _backward,
    csrc/softmax_pool.hip)."""
    _nat.require_device(stacked, "LateFusion logits")
    fused, _ = torch.ops.mmfusion.late_weights_fwd(stacked, weight_logits, mask)
    return fused


class LateFusion(nn.Module):
    """Per-modality classifiers (nn.Linear on PyTorch-ROCm), then the masked
    softmax(weight_logits) weighting on HIP (src/fusion.py:126-245)."""

    def __init__(self, modality_dims: Dict[str, int], hidden_dim: int = 256, num_classes: int = 11,
                 dropout: float = 0.1):
        super().__init__()
        dims = dict(modality_dims)
        cast_self = cast(Any, self)
        cast_self.modality_names = list(dims)
        cast_self.num_modalities = len(dims)
        cast_self.modality_dims = dims
        self.classifiers = nn.ModuleDict({
            name: nn.Sequential(nn.Linear(d, hidden_dim), nn.ReLU(), nn.Dropout(dropout),
                                nn.Linear(hidden_dim, num_classes))
            for name, d in dims.items()})
        self.weight_logits = nn.Parameter(torch.zeros(self.num_modalities))
        self.dropout = nn.Dropout(dropout)

    def forward(self, modality_features, modality_mask=None):
        if not self.modality_names:
            raise ValueError("No modalities configured for LateFusion.")
        mask = _mask_or_ones(modality_features, self.modality_names, modality_mask, "LateFusion")
        per: Dict[str, torch.Tensor] = {}
        for i, name in enumerate(self.modality_names):
            if name not in modality_features:
                raise KeyError(f"Missing features for modality '{name}' in LateFusion forward pass.")
            x = modality_features[name].to(mask.device) * mask[:, i:i + 1]
            per[name] = self.classifiers[name](self.dropout(x))
        stacked = torch.stack([per[n] for n in self.modality_names], dim=1)
        return _late_weights(_nat.f32c(stacked), self.weight_logits, mask.float().contiguous()), per


# --------------------------------------------------------------------------
# HybridFusion: the accelerated hot path
# --------------------------------------------------------------------------
class _Plan:
    """Shape/pair descriptor + parameter ordering (ctypes descriptor) for the fused
    training step (train_step.HybridTrainStep)."""

    def __init__(self, model: "HybridFusion", seq: List[int], dims: List[int], batch: int,
                 pairs: List[Tuple[int, int, str]], return_attention: bool):
        d = _nat.HybridDesc()
        d.batch = batch
        d.num_modalities = model.num_modalities
        d.hidden = model.hidden_dim
        d.num_heads = model.num_heads
        d.num_classes = model.num_classes
        for m in range(model.num_modalities):
            d.seq_len[m] = seq[m]
            d.in_dim[m] = dims[m]
        d.num_pairs = len(pairs)
        for g, (q, k, _) in enumerate(pairs):
            d.pair_q[g] = q
            d.pair_k[g] = k
        d.dropout = float(model.dropout.p)
        d.training = int(model.training)
        d.return_attention = int(return_attention)
        d.matmul_precision = _nat.matmul_precision()
        # the plan switches the step's buffers are sized under (the step sets the capacities)
        d.plan_flags = _nat.lib().mmf_hybrid_plan_flags()
        self.desc = d
        self.seq = [max(s, 1) for s in seq]
        self.pairs = pairs
        # parameter order: proj (w,b) per m; per pair q,k,v,o (w,b); gate (w,b) per m; cls1; cls2
        self.names: List[str] = []
        for m in model.modality_names:
            self.names += [f"projections.{m}.0.weight", f"projections.{m}.0.bias"]
        for _, _, key in pairs:
            for proj in ("query_proj", "key_proj", "value_proj", "out_proj"):
                self.names += [f"attention_modules.{key}.{proj}.weight",
                               f"attention_modules.{key}.{proj}.bias"]
        for m in model.modality_names:
            self.names += [f"gating_layers.{m}.weight", f"gating_layers.{m}.bias"]
        self.names += ["classifier.0.weight", "classifier.0.bias", "classifier.3.weight",
                       "classifier.3.bias"]
        self.num_param_elems = 0

    # every tensor of a flat parameter / gradient buffer starts on a 256-byte
    # boundary, so the kernels' 16-byte vector paths apply to all of them
    ALIGN = 64

    def params(self, model: "HybridFusion") -> List[torch.Tensor]:
        named = dict(model.named_parameters())
        out = [named[n] for n in self.names]
        self.offsets = []
        off = 0
        for p in out:
            self.offsets.append(off)
            off += -(-p.numel() // self.ALIGN) * self.ALIGN
        self.num_param_elems = off
        return out

    def grad_views(self, flat: torch.Tensor, params) -> List[torch.Tensor]:
        return [flat[o:o + p.numel()].view_as(p) for o, p in zip(self.offsets, params)]

    def param_struct(self, ts) -> "_nat.HybridParams":
        s = _nat.HybridParams()
        M = self.desc.num_modalities
        it = iter(ts)
        nxt = lambda: next(it).data_ptr()  # noqa: E731
        for m in range(M):
            s.proj[m] = _nat.Linear(nxt(), nxt())
        for g in range(len(self.pairs)):
            s.q[g] = _nat.Linear(nxt(), nxt())
            s.k[g] = _nat.Linear(nxt(), nxt())
            s.v[g] = _nat.Linear(nxt(), nxt())
            s.o[g] = _nat.Linear(nxt(), nxt())
        for m in range(M):
            s.gate[m] = _nat.Linear(nxt(), nxt())
        s.cls1 = _nat.Linear(nxt(), nxt())
        s.cls2 = _nat.Linear(nxt(), nxt())
        return s


class HybridFusion(nn.Module):
    """Cross-modal attention + learned, mask-aware fusion weights (src/fusion.py:248-479)."""

    modality_names: list[str]
    num_modalities: int
    hidden_dim: int
    projections: nn.ModuleDict
    attention_modules: nn.ModuleDict
    gating_layers: nn.ModuleDict
    classifier: nn.Sequential
    dropout: nn.Dropout

    def __init__(self, modality_dims: Dict[str, int], hidden_dim: int = 256, num_classes: int = 11,
                 num_heads: int = 4, dropout: float = 0.1):
        super().__init__()
        dims = dict(modality_dims)
        names = list(dims)
        cast_self = cast(Any, self)
        cast_self.modality_names = names
        cast_self.num_modalities = len(names)
        cast_self.hidden_dim = hidden_dim
        cast_self.num_heads = num_heads
        cast_self.num_classes = num_classes
        # construction order == the reference's => identical init for a given seed
        self.projections = nn.ModuleDict({
            m: nn.Sequential(nn.Linear(d, hidden_dim), nn.ReLU(), nn.Dropout(dropout))
            for m, d in dims.items()})
        self.attention_modules = nn.ModuleDict({
            f"{q}_to_{k}": CrossModalAttention(hidden_dim, hidden_dim, hidden_dim=hidden_dim,
                                               num_heads=num_heads, dropout=dropout)
            for q in names for k in names if q != k})
        self.gating_layers = nn.ModuleDict({m: nn.Linear(hidden_dim, 1) for m in names})
        self.classifier = nn.Sequential(nn.Linear(hidden_dim, hidden_dim), nn.ReLU(),
                                        nn.Dropout(dropout), nn.Linear(hidden_dim, num_classes))
        self.dropout = nn.Dropout(dropout)
        self.register_buffer("_rng_state", _new_rng_state(), persistent=False)

    # ------------------------------------------------------------------ helpers
    def present_pairs(self) -> List[Tuple[int, int, str]]:
        """Pairs in the reference's iteration order, skipping deleted modules (src/fusion.py:383-389)."""
        out = []
        for qi, q in enumerate(self.modality_names):
            for ki, k in enumerate(self.modality_names):
                if q != k and f"{q}_to_{k}" in self.attention_modules:
                    out.append((qi, ki, f"{q}_to_{k}"))
        return out

    def _plan(self, feats: List[torch.Tensor], return_attention: bool) -> _Plan:
        seq, dims = self._shapes(feats)
        return _Plan(self, seq, dims, feats[0].size(0), self.present_pairs(), return_attention)

    def _shapes(self, feats: List[torch.Tensor], in_dims: Optional[List[int]] = None) -> Tuple[List[int], List[int]]:
        seq, dims = [], []
        B = feats[0].size(0)
        for m, (name, x) in enumerate(zip(self.modality_names, feats)):
            if x.dim() == 2:
                seq.append(0)
            elif x.dim() == 3:
                seq.append(int(x.size(1)))
            else:
                raise RuntimeError(f"features for modality '{name}' must be 2-D or 3-D, got {tuple(x.shape)}")
            if x.size(0) != B:
                raise RuntimeError(f"batch size mismatch for modality '{name}': {x.size(0)} vs {B}")
            in_f = in_dims[m] if in_dims is not None else self.projections[name][0].in_features
            if x.size(-1) != in_f:
                raise RuntimeError(f"modality '{name}': expected feature dim {in_f}, got {x.size(-1)}")
            dims.append(int(x.size(-1)))
        return seq, dims

    def _param_names(self, pairs: List[Tuple[int, int, str]]) -> List[str]:
        """The operator's parameter order: proj (w, b) per modality; per present pair
        query, key, value, out (w, b); gates (w, b) per modality; classifier.0; classifier.3."""
        names: List[str] = []
        for m in self.modality_names:
            names += [f"projections.{m}.0.weight", f"projections.{m}.0.bias"]
        for _, _, key in pairs:
            for proj in ("query_proj", "key_proj", "value_proj", "out_proj"):
                names += [f"attention_modules.{key}.{proj}.weight", f"attention_modules.{key}.{proj}.bias"]
        for m in self.modality_names:
            names += [f"gating_layers.{m}.weight", f"gating_layers.{m}.bias"]
        return names + ["classifier.0.weight", "classifier.0.bias", "classifier.3.weight", "classifier.3.bias"]

    # ------------------------------------------------------------------ forward
    # torch.compile (the reference compiles the fusion model, src/train.py:193-231, without
    # fullgraph): by default the module is one opaque native step to TorchDynamo -- its forward runs
    # as in eager mode (HybridSink: gradients straight into the module's flat buffer) and Dynamo
    # does not trace it, because tracing buys no fusion here (the work is already a few HIP
    # launches) and costs a cudagraph-tree replay, AOTAutograd's runtime wrappers and one
    # AccumulateGrad per parameter per step.  traceable = True keeps the fully
    # traceable form: custom operators with fake kernels and autograd formulas, fullgraph-capable.
    traceable: bool = False

    def forward(self, modality_features: Dict[str, torch.Tensor],
                modality_mask: Optional[torch.Tensor] = None, return_attention: bool = False):
        if torch.compiler.is_compiling() and not self.traceable:
            return _opaque_forward(self, modality_features, modality_mask, return_attention)
        return self._forward(modality_features, modality_mask, return_attention)

    def _forward(self, modality_features: Dict[str, torch.Tensor],
                 modality_mask: Optional[torch.Tensor] = None, return_attention: bool = False):
        if not self.modality_names:
            raise ValueError("No modalities configured for HybridFusion.")
        ref = modality_features[self.modality_names[0]]
        batch_size, device, dtype = ref.size(0), ref.device, ref.dtype
        if modality_mask is None:
            modality_mask = torch.ones(batch_size, self.num_modalities, device=device, dtype=dtype)
        else:
            modality_mask = _check_mask(modality_mask.to(device=device, dtype=dtype), batch_size,
                                        self.num_modalities, "HybridFusion")
        feats = []
        for name in self.modality_names:
            if name not in modality_features:
                raise KeyError(f"Missing features for modality '{name}' in HybridFusion forward pass.")
            feats.append(modality_features[name].to(device))
        _nat.require_device(ref, "HybridFusion input")
        # traced (torch.compile, fake tensors): the custom operator; eager: HybridSink / HybridEager
        compiling = not _ops.eager_tensor(ref)
        hooked = False   # a hook on some parameter's AccumulateGrad node (only the extension can see it)
        if compiling:
            seq, dims = self._shapes(feats)
            for p in self.parameters():
                if p.device != device or p.dtype != torch.float32:
                    raise RuntimeError("mmfusion HybridFusion needs float32 parameters on the input's device "
                                       f"(found {p.dtype} on {p.device})")
            pairs = self.present_pairs()
            named = dict(self.named_parameters())
            params = [named[n] for n in self._param_names(pairs)]
        else:
            pairs, params, in_dims, descs = self._op_params(device)
            ext = _ops.torch_ext()
            if ext is not None:
                # eager through mmf_torch's C++ node: the shape checks and the descriptor once per input
                # signature; the parameters' gradients written straight into the module's flat gradient
                # buffer (no per-parameter autograd work), the dropout state advanced in place
                key = (tuple(map(_SHAPE, feats)), self.training, return_attention, _precision(), self.dropout.p,
                       _nat.lib().mmf_hybrid_plan_flags())
                addr = descs.get(key)
                if addr is None:
                    seq, dims = self._shapes(feats, in_dims)
                    idesc = _ops.hybrid_idesc(batch_size, self.hidden_dim, self.num_heads, self.num_classes, seq, dims,
                                              [(q, k) for q, k, _ in pairs], self.training, return_attention,
                                              _precision())
                    addr = descs[key] = ctypes.addressof(_ops.hybrid_desc(idesc, float(self.dropout.p)))
                sink = self._grad_sink(params, len(pairs))
                # (the grad sink keeps the parameters outside the graph: not with tensor hooks, frozen
                # parameters or hooks on their AccumulateGrad nodes -- DistributedDataParallel's
                # reducer -- which would never run; those take HybridEager below)
                if not torch.is_grad_enabled() or sink.ok():
                    logits, fw, *maps = ext.hybrid_sink_forward(sink, addr, self._rng_state, _nat.f32c(modality_mask),
                                                                [_nat.f32c(x) for x in feats])
                    return self._finish(logits, fw, maps, pairs, dtype, return_attention)
                hooked = sink.accumulator_hooked()
                if not hooked and _ops._sink_ok(params):
                    logits, fw, *maps = ext.hybrid_sink_forward(sink, addr, self._rng_state, _nat.f32c(modality_mask),
                                                                [_nat.f32c(x) for x in feats])
                    return self._finish(logits, fw, maps, pairs, dtype, return_attention)
            seq, dims = self._shapes(feats, in_dims)
        idesc = _ops.hybrid_idesc(batch_size, self.hidden_dim, self.num_heads, self.num_classes, seq, dims,
                                  [(q, k) for q, k, _ in pairs], self.training, return_attention, _precision())
        xs = [_nat.f32c(x) for x in feats]
        if compiling:
            # (traced by TorchDynamo: the custom operator, its fake kernel and autograd formula; the
            # operator is functional, so the advanced dropout state comes back and is copied in)
            logits, fw, _saved, rng_next, maps = torch.ops.mmfusion.hybrid_fwd(
                idesc, float(self.dropout.p), self._rng_state, _nat.f32c(modality_mask), xs, params)
            self._rng_state.copy_(rng_next)     # the device Philox stream advanced by one call
        elif torch.is_grad_enabled() and not hooked and _ops._sink_ok(params):
            # eager without the C++ extension: the Python twin of its node (mmf_ops.HybridSink);
            # params[0] anchors the graph
            logits, fw, _saved, *maps = _ops.HybridSink.apply(
                idesc, float(self.dropout.p), self._rng_state, _nat.f32c(modality_mask), self, params, params[0], *xs)
        else:
            # eager, some parameter frozen or hooked: the same implementation with every parameter an
            # autograd input (mmf_ops.HybridEager)
            logits, fw, _saved, *maps = _ops.HybridEager.apply(
                idesc, float(self.dropout.p), self._rng_state, _nat.f32c(modality_mask), len(xs), *xs, *params)
        return self._finish(logits, fw, maps, pairs, dtype, return_attention)

    @staticmethod
    def _finish(logits, fw, maps, pairs, dtype, return_attention):
        if dtype != torch.float32 and dtype.is_floating_point:
            logits = logits.to(dtype)
        if return_attention:
            attention_maps = {key: maps[g].detach() for g, (_, _, key) in enumerate(pairs)}
            return logits, {"attention_maps": attention_maps, "fusion_weights": fw.detach()}
        return logits

    def _op_params(self, device) -> Tuple[List[Tuple[int, int, str]], List[torch.Tensor], List[int], Dict[tuple, int]]:
        """(present pairs, the operator's parameter list, the modalities' input widths, the eager
        path's descriptor cache: input signature -> mmf_hybrid_desc address), cached per set of
        attention modules (a deleted pair changes it) and per parameter registration anywhere
        (_PARAM_GEN: replacing a Parameter object -- `proj[0].weight = nn.Parameter(...)`,
        load_state_dict(assign=True), weight tying, parametrizations -- registers one), and dropped
        by every .to() / .cuda() / .float() (_apply), so the float32-on-one-device check runs once
        per cache: an eager step then costs no walk over the module tree."""
        keys = (tuple(self.attention_modules.keys()), _PARAM_GEN[0])
        c = self.__dict__.get("_mmf_op_params")
        if c is None or c[0] != keys:
            # (a new parameter set: the grad sink holding the old tensors goes with it)
            self.__dict__.pop("_mmf_grad_sink", None)
            pairs = self.present_pairs()
            named = dict(self.named_parameters())
            params = [named[n] for n in self._param_names(pairs)]
            for p in params:
                if p.device != params[0].device or p.dtype != torch.float32:
                    raise RuntimeError("mmfusion HybridFusion needs float32 parameters on one device "
                                       f"(found {p.dtype} on {p.device})")
            in_dims = [self.projections[m][0].in_features for m in self.modality_names]
            c = (keys, pairs, params, in_dims, {})
            self.__dict__["_mmf_op_params"] = c
        if c[2][0].device != device:
            raise RuntimeError("mmfusion HybridFusion needs float32 parameters on the input's device "
                               f"(found {c[2][0].dtype} on {c[2][0].device})")
        return c[1], c[2], c[3], c[4]

    def _grad_sink(self, params: List[torch.Tensor], num_pairs: Optional[int] = None):
        """The flat gradient buffer the eager backward writes into (mmf_ops.make_grad_sink: the C++
        node's or mmf_ops.HybridSink's)."""
        sk = self.__dict__.get("_mmf_grad_sink")
        if sk is None or not sk.matches(params) or isinstance(sk, _ops.GradSink) != (_ops.torch_ext() is None):
            P = len(self.present_pairs()) if num_pairs is None else num_pairs
            sk = _ops.make_grad_sink(params, self.num_modalities, P)
            self.__dict__["_mmf_grad_sink"] = sk
        return sk

    def mmf_grads_consumed(self) -> bool:
        """A trainer has applied the gradients the parameters' ``.grad`` hold.  If those are the
        views of the module's flat gradient buffer (the eager grad-sink path), the next backward
        writes them afresh instead of adding, with the ``.grad`` attributes left in place: returns
        True.  Otherwise (a traced backward's outputs, someone else's tensors) returns False and
        the caller resets ``.grad`` as zero_grad(set_to_none=True) does (harness.DPTrainer)."""
        sk = self.__dict__.get("_mmf_grad_sink")
        c = self.__dict__.get("_mmf_op_params")
        if sk is None or c is None or not sk.matches(c[2]):
            return False
        if not isinstance(sk, _ops.GradSink):
            return sk.consumed()   # (mmf_torch.Sink: the same check in C++)
        if not all(p.grad is v for p, v in zip(c[2], sk.views)):
            return False
        sk.fresh = True
        return True

    def _apply(self, fn, *args, **kwargs):
        self.__dict__.pop("_mmf_op_params", None)
        self.__dict__.pop("_mmf_grad_sink", None)
        return super()._apply(fn, *args, **kwargs)

    def __getstate__(self):
        # (copy.deepcopy / pickling, src/train.py:73-76: the caches are rebuilt on first use)
        st = super().__getstate__() if hasattr(super(), "__getstate__") else self.__dict__.copy()
        st = dict(st)
        st.pop("_mmf_op_params", None)
        st.pop("_mmf_grad_sink", None)
        return st

    def compute_adaptive_weights(self, modality_features: Dict[str, torch.Tensor],
                                 modality_mask: torch.Tensor) -> torch.Tensor:
        """src/fusion.py:429-479 on the device (gating scores -> masked softmax -> renormalise).

        Differentiable like the reference's: gradients reach the features and
        gating_layers through mmf_adaptive_weights_backward."""
        if modality_mask is None:
            raise ValueError("modality_mask must be provided for adaptive weighting.")
        device = modality_mask.device
        feats = []
        for name in self.modality_names:
            if name not in modality_features:
                raise KeyError(f"Missing aggregated features for modality '{name}'.")
            feats.append(modality_features[name].to(device))
        B = feats[0].size(0) if feats[0].dim() > 0 else 0
        M, H = self.num_modalities, self.hidden_dim
        for name, f in zip(self.modality_names, feats):
            # gating_layers[m](feat) then cat(dim=1) needs (B, H) per modality (src/fusion.py:452-461)
            if f.dim() != 2 or f.size(0) != B or f.size(1) != H:
                raise RuntimeError(f"compute_adaptive_weights: features of '{name}' must have shape "
                                   f"({B}, {H}), got {tuple(f.shape)}")
        mask = _check_mask(modality_mask.to(dtype=torch.float32), B, M, "compute_adaptive_weights")
        _nat.require_device(modality_mask, "modality_mask")
        gparams = []
        for name in self.modality_names:
            layer = self.gating_layers[name]
            gparams += [layer.weight, layer.bias]
        return torch.ops.mmfusion.adaptive_weights_fwd(_nat.f32c(mask), [_nat.f32c(f) for f in feats], gparams)


@torch.compiler.disable
def _opaque_forward(model: "HybridFusion", modality_features, modality_mask, return_attention):
    """HybridFusion's forward run outside TorchDynamo (HybridFusion.traceable = False)."""
    return model._forward(modality_features, modality_mask, return_attention)


def build_fusion_model(fusion_type: str, modality_dims: Dict[str, int], num_classes: int,
                       **kwargs) -> nn.Module:
    """Factory used by src/train.py:175-182 (src/fusion.py:485-515)."""
    classes = {"early": EarlyFusion, "late": LateFusion, "hybrid": HybridFusion}
    if fusion_type not in classes:
        raise ValueError(f"Unknown fusion type: {fusion_type}")
    kw = dict(kwargs)
    if fusion_type != "hybrid":
        kw.pop("num_heads", None)
    return classes[fusion_type](modality_dims=modality_dims, num_classes=num_classes, **kw)
