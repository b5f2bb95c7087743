"""Module-path training harness: the reference's MultimodalFusionModule, data-parallel.

The reference trains encoders and the fusion model jointly in one process on the
CPU through Lightning (src/train.py:125-430, Trainer(devices=1, gradient_clip_val,
accumulate_grad_batches=4), :511-524).  This is its MI355X-native equivalent for the
configs that train encoders (C3 PAMAP2, C4 MHAD), one process per GPU:

  * ``MultimodalFusionModel`` mirrors ``MultimodalFusionModule.forward``
    (src/train.py:233-291): per-modality encoder -> optional LayerNorm ->
    ``fusion_model(encoded, mask)``; modalities absent from ``features`` are skipped
    as there (:259-262).  Built from config/base.yaml's keys by ``from_config`` with
    the reference's ``build_encoder`` dispatch (src/encoders.py:400-451; SequenceEncoder
    'lstm' on csrc/lstm.hip, FrameEncoder with its attention pooling on
    csrc/softmax_pool.hip, HybridFusion on the fused HIP path).  When every encoder
    is a SequenceEncoder with one (B, T), the LSTMs of all modalities share each
    recurrence launch (``encode_sequences``).
  * ``FlatGradBuckets`` re-points every parameter into one contiguous fp32 buffer and
    its gradient into views of another (autograd accumulates into them in place), and
    all-reduces that gradient in buckets issued from post-accumulate-grad hooks: the
    fusion model's gradients (its backward runs first) are in flight over RCCL / xGMI
    while the encoders' LSTM backward still runs.  The only data-path exchange.
  * ``DPTrainer`` is Lightning's automatic optimisation for this model:
    CrossEntropyLoss(label_smoothing) (src/train.py:185-186, 310), the loss divided by
    ``accumulate`` and back-propagated per micro-batch, the gradient exchanged once per
    optimizer step (the other micro-batches accumulate locally), global-norm clipping
    and AdamW in two HIP launches over the flat buffers (mmf_clip_adamw_step_dev,
    src/train.py:374-430), CosineAnnealingLR per epoch (:394-402).
  * ``shard_indices`` is torch's DistributedSampler partition (pad by wrapping to a
    multiple of the world size, rank r takes every world-th index), used to shard the
    PAMAP2 chunk list (manifest loader batch = 1 chunk, src/data.py:560-566).
"""

from __future__ import annotations

import math
import operator
import os
import sys
from typing import Any, Dict, List, Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)


# ----------------------------------------------------------------------------- sharding
def shard_indices(n: int, rank: int, world: int, shuffle: bool = False, seed: int = 0, epoch: int = 0) -> List[int]:
    """torch.utils.data.DistributedSampler(drop_last=False) partition of range(n).

    With shuffle, the permutation is torch.randperm(n) under manual_seed(seed + epoch)
    (DistributedSampler.__iter__); the list is padded by wrapping to a multiple of
    world, and rank r takes indices r, r + world, ...  Every rank gets
    ceil(n / world) indices, so all ranks run the same number of steps."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    if n < 1:
        return []
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        idx = torch.randperm(n, generator=g).tolist()
    else:
        idx = list(range(n))
    per = math.ceil(n / world)
    total = per * world
    pad = total - n
    if pad:
        reps = math.ceil(pad / n)
        idx += (idx * reps)[:pad]
    return idx[rank:total:world]


# ----------------------------------------------------------------------------- model
class MultimodalFusionModel(nn.Module):
    """encoders -> optional LayerNorm -> fusion (src/train.py:140-191, 233-291)."""

    def __init__(self, encoders: Dict[str, nn.Module], fusion_model: nn.Module, output_dim: int,
                 layer_norm: bool = True):
        super().__init__()
        self.encoders = nn.ModuleDict(encoders)
        self.use_layer_norm = bool(layer_norm)
        self.layer_norms = nn.ModuleDict({m: nn.LayerNorm(output_dim) for m in encoders} if layer_norm else {})
        self.fusion_model = fusion_model

    @classmethod
    def from_config(cls, config: Dict[str, Any]) -> "MultimodalFusionModel":
        """Build from config/base.yaml's keys: dataset.modalities, dataset.num_classes,
        model.{encoders, output_dim, hidden_dim, num_heads, dropout, fusion_type, layer_norm}
        (the construction order of src/train.py:150-182)."""
        from encoders import FrameEncoder, SequenceEncoder
        from fusion import build_fusion_model
        ds, mc = config["dataset"], config["model"]
        out_dim = int(mc["output_dim"])
        encs: Dict[str, nn.Module] = {}
        for m in ds["modalities"]:
            ec = dict(mc.get("encoders", {}).get(m, {}))
            in_dim = int(ec.pop("input_dim", 64))
            kind = ec.pop("type", None)
            key = m.lower()
            if kind == "frame" or (kind is None and key in ("video", "frames")):
                encs[m] = FrameEncoder(frame_dim=in_dim, output_dim=out_dim, **ec)
            elif kind == "sequence" or (kind is None and (key in ("imu", "audio", "mocap", "accelerometer")
                                                          or key.startswith("imu_"))):
                encs[m] = SequenceEncoder(input_dim=in_dim, output_dim=out_dim, **ec)
            else:
                # SimpleMLPEncoder (src/encoders.py:339-397) serves config 1's EarlyFusion CPU plumbing only
                raise NotImplementedError(f"encoder for modality '{m}' ({kind or 'mlp'}) is not on the MI355X path")
        fusion = build_fusion_model(mc.get("fusion_type", "hybrid"), {m: out_dim for m in encs},
                                    int(ds.get("num_classes", 11)), hidden_dim=int(mc["hidden_dim"]),
                                    num_heads=int(mc.get("num_heads", 4)), dropout=float(mc["dropout"]))
        return cls(encs, fusion, out_dim, bool(mc.get("layer_norm", False)))

    def _batched_sequences(self, features: Dict[str, torch.Tensor]) -> bool:
        from encoders import SequenceEncoder
        present = [m for m in self.encoders if m in features]
        if len(present) < 2:
            return False
        encs = [self.encoders[m] for m in present]
        if not all(isinstance(e, SequenceEncoder) and e.rnn is not None for e in encs):
            return False
        r0 = encs[0].rnn
        shapes = {tuple(features[m].shape[:2]) for m in present}
        return (len(shapes) == 1 and all(features[m].dim() == 3 for m in present)
                and all(e.rnn.hidden_size == r0.hidden_size and e.rnn.num_layers == r0.num_layers for e in encs))

    def encode(self, features: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        if self._batched_sequences(features):
            from encoders import encode_sequences
            present = [m for m in self.encoders if m in features]
            enc = encode_sequences({m: self.encoders[m] for m in present}, {m: features[m] for m in present})
        else:
            enc = {m: self.encoders[m](features[m]) for m in self.encoders if m in features}
        out = {}
        for m in self.encoders:          # modality order = the encoders' order (src/train.py:250)
            if m not in enc:
                continue
            x = enc[m]
            if self.use_layer_norm and m in self.layer_norms:
                x = self.layer_norms[m](x)
            out[m] = x
        return out

    def forward(self, features: Dict[str, torch.Tensor], mask: Optional[torch.Tensor] = None,
                return_attention: bool = False):
        encoded = self.encode(features)
        if return_attention:
            output = self.fusion_model(encoded, mask, return_attention=True)
        else:
            output = self.fusion_model(encoded, mask)
        if isinstance(output, tuple):     # LateFusion returns (logits, per-modality logits)
            logits, aux = output[0], (output[1] if len(output) > 1 else None)
        else:
            logits, aux = output, None
        return (logits, aux) if return_attention else logits


# ----------------------------------------------------------------------------- flat buffers + bucketed all-reduce
_GRAD = torch.Tensor.grad.__get__   # (p.grad as a C-level callable: map() over parameters)


class FlatGradBuckets:
    """All parameters of `modules` in one flat fp32 buffer and their gradients in a second
    one, exchanged in buckets.

    Gradients are autograd's own tensors, as with ``zero_grad(set_to_none=True)`` (the
    reference's Lightning default): every parameter's ``.grad`` is None before a backward,
    AccumulateGrad takes the backward's gradient tensor without a copy (the HIP operators
    return one flat gradient buffer per call, sliced into views), and gathering copies the
    gradients of a bucket into its span of the flat buffer with one multi-tensor copy
    (``torch._foreach_copy_``, a launch or two for the whole bucket) and resets them to
    None.  (Gradients kept as permanent views of the flat buffer instead cost one
    in-place add launch per parameter and backward: 65 per HybridFusion step.)  Micro-
    batches before the armed one accumulate in ``.grad`` as autograd does.

    Buckets follow `groups` (lists of parameters, e.g. [fusion params, encoder params]):
    a bucket is gathered and all-reduced (sum, async) from the post-accumulate-grad hook of
    the last of its parameters to finish accumulating -- while the rest of the backward
    still runs -- when ``arm()`` was called for this backward.  ``finish()`` gathers and
    issues what is left (parameters that received no gradient) and waits.  Tensors start
    on 256-byte boundaries (the HIP kernels' 16-byte vector paths)."""

    ALIGN = 64

    def __init__(self, groups: Sequence[Sequence[nn.Parameter]], process_group=None):
        self.pg = process_group
        self.world = torch.distributed.get_world_size(process_group) if process_group is not None else 1
        params: List[nn.Parameter] = []
        seen = set()
        self.groups: List[List[nn.Parameter]] = []
        for grp in groups:
            g = [p for p in grp if p.requires_grad and id(p) not in seen]
            seen.update(id(p) for p in g)
            if g:
                self.groups.append(g)
                params += g
        if not params:
            raise ValueError("FlatGradBuckets: no trainable parameters")
        dev = params[0].device
        for p in params:
            if p.dtype != torch.float32 or p.device != dev:
                raise ValueError("FlatGradBuckets: every parameter must be fp32 on one device")
        offs, off = [], 0
        spans = []
        for g in self.groups:
            start = off
            for p in g:
                offs.append(off)
                off += -(-p.numel() // self.ALIGN) * self.ALIGN
            spans.append((start, off))
        self.numel = off
        self.params = params
        self.flat = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(off, dtype=torch.float32, device=dev)
        # per bucket: its parameters and the views of their spans of the flat gradient
        self._gviews: List[List[torch.Tensor]] = []
        it = iter(offs)
        for g in self.groups:
            views = []
            for p in g:
                o = next(it)
                self.flat[o:o + p.numel()].copy_(p.detach().reshape(-1))
                p.data = self.flat[o:o + p.numel()].view_as(p)
                p.grad = None
                views.append(self.grad[o:o + p.numel()].view_as(p))
            self._gviews.append(views)
        self.spans = spans
        self._bucket_of = {}
        for b, g in enumerate(self.groups):
            for p in g:
                self._bucket_of[id(p)] = b
        self._fresh = [True] * len(self.groups)    # the bucket's span holds no gradient yet
        self._direct_last = None                    # (grad tensors, base) of direct_grad's last match
        self._pending = [0] * len(self.groups)
        self._works: List[Any] = [None] * len(self.groups)
        self._armed = False
        # (one process: nothing to exchange, no per-parameter Python hook in the backward)
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in params] if self.world > 1 else []

    def bucket(self, b: int) -> torch.Tensor:
        s, e = self.spans[b]
        return self.grad[s:e]

    def gather(self, b: Optional[int] = None) -> None:
        """Move the parameters' ``.grad`` tensors of bucket b (every bucket: None) into the flat
        gradient -- a copy into a fresh span, an add otherwise -- and set them to None."""
        for bb in (range(len(self.groups)) if b is None else (b,)):
            dst, src, missing = [], [], []
            for p, v in zip(self.groups[bb], self._gviews[bb]):
                if p.grad is None:
                    missing.append(v)
                else:
                    dst.append(v)
                    src.append(p.grad)
                    p.grad = None
            if self._fresh[bb]:
                if dst:
                    torch._foreach_copy_(dst, src)
                if missing:
                    torch._foreach_zero_(missing)
            elif dst:
                torch._foreach_add_(dst, src)
            self._fresh[bb] = False

    def direct_grad(self) -> Optional[torch.Tensor]:
        """One process, one bucket: the tensor the parameters' ``.grad`` already live in, when it
        has this buffer's layout -- then the optimizer reads it in place and nothing is gathered.
        The HIP operators return each module's parameter gradients as views of ONE flat buffer,
        at the same 256-byte-aligned offsets and in the same order (registration order) as this
        buffer's, so after a HybridFusion backward (eager or a compiled graph's replay) every
        ``.grad`` is a view of one base at exactly ``offset - span start``.  None when any
        gradient is missing or elsewhere (several buckets, a gradient produced by a torch op, an
        accumulated sum that autograd allocated): the caller gathers instead."""
        if self.world != 1 or len(self.groups) != 1 or not self._fresh[0]:
            return None
        params, views = self.groups[0], self._gviews[0]
        last = self._direct_last
        if last is not None and all(map(operator.is_, map(_GRAD, params), last[0])):
            return last[1]   # the same gradient tensors as the last validated step (a grad sink)
        g0 = params[0].grad
        if g0 is None or g0.dtype != torch.float32 or g0.device != self.grad.device:
            return None
        st = g0.untyped_storage()
        sptr, off0 = st.data_ptr(), g0.storage_offset()
        if st.nbytes() < 4 * (off0 + self.numel):
            return None
        # every gradient in that storage at its offset in this layout, same shape and strides (the
        # padding between them is zero: the operators allocate their flat gradient zeroed)
        for p, v in zip(params, views):
            g = p.grad
            if (g is None or g.untyped_storage().data_ptr() != sptr or g.storage_offset() - off0 != v.storage_offset()
                    or g.stride() != v.stride()):
                return None
        base = g0.as_strided((self.numel,), (1,), off0)
        self._direct_last = ([p.grad for p in params], base)
        return base

    def zero_grad(self) -> None:
        """Forget the flat gradient (the next gather copies instead of adding) and any
        ungathered ``.grad``."""
        self._fresh = [True] * len(self.groups)
        for p in self.params:
            p.grad = None

    def arm(self) -> None:
        """The next backward is the last before an optimizer step: exchange its buckets."""
        self._armed = True
        self._pending = [len(g) for g in self.groups]
        self._works = [None] * len(self.groups)

    def _on_grad(self, p: torch.Tensor) -> None:
        if not self._armed:
            return
        b = self._bucket_of[id(p)]
        self._pending[b] -= 1
        if self._pending[b] == 0 and self._works[b] is None:
            self._launch(b)

    def _launch(self, b: int) -> None:
        self.gather(b)
        if self.world > 1:
            self._works[b] = torch.distributed.all_reduce(self.bucket(b), group=self.pg, async_op=True)
        else:
            self._works[b] = True

    def finish(self) -> None:
        """Gather and issue the buckets no hook issued, then wait for every exchange.  Unarmed
        (a plain backward, no exchange): gather every bucket."""
        if not self._armed:
            self.gather()
            return
        for b in range(len(self.groups)):
            if self._works[b] is None:
                self._launch(b)
        for w in self._works:
            if w is not None and w is not True:
                w.wait()
        self._armed = False

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []


# ----------------------------------------------------------------------------- trainer
class DPTrainer:
    """Automatic optimisation of the reference's training_step for MultimodalFusionModel
    (or any module returning logits), one process per GPU.

    step(batches) runs len(batches) == accumulate micro-batches: forward, CE with label
    smoothing, backward of loss / accumulate (Lightning's scaling), the last one with
    the bucketed gradient exchange armed; then clip (global norm over the rank-averaged
    gradient) + AdamW on the flat buffers in two HIP launches.  Defaults are
    config/base.yaml's training keys."""

    def __init__(self, model: nn.Module, lr: float = 1e-3, weight_decay: float = 1e-4, betas=(0.9, 0.999),
                 eps: float = 1e-8, label_smoothing: float = 0.05, gradient_clip_norm: float = 1.0,
                 accumulate: int = 4, process_group=None, buckets: Optional[Sequence[Sequence[nn.Parameter]]] = None):
        import mmf_native as nat
        self._nat = nat
        self.model = model
        dev = next(model.parameters()).device
        nat.require_device(next(model.parameters()), "DPTrainer parameters")
        self.dev = dev
        if buckets is None:
            fusion = getattr(model, "fusion_model", None)
            if fusion is not None:
                rest = [p for n, p in model.named_parameters() if not n.startswith("fusion_model.")]
                buckets = [list(fusion.parameters()), rest]
            else:
                buckets = [list(model.parameters())]
        self.flat = FlatGradBuckets(buckets, process_group)
        self.world = self.flat.world
        if process_group is not None and self.world > 1:
            # identical initial weights on every rank (DDP's broadcast from rank 0) ...
            torch.distributed.broadcast(self.flat.flat, src=torch.distributed.get_global_rank(process_group, 0),
                                        group=process_group)
            # ... but distinct dropout streams: the rank folded into each HIP module's Philox key, once
            rank = torch.distributed.get_rank(process_group)
            for mod in model.modules():
                buf = getattr(mod, "_rng_state", None)
                if isinstance(buf, torch.Tensor) and not getattr(mod, "_mmf_rank_folded", False):
                    buf[0] ^= rank * 0x9E3779B1
                    mod._mmf_rank_folded = True
        self.accumulate = int(accumulate)
        self.smoothing = label_smoothing
        self.clip_norm = gradient_clip_norm
        self.wd, self.betas, self.eps = weight_decay, betas, eps
        n = self.flat.numel
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self.step_dev = torch.zeros(1, dtype=torch.int64, device=dev)
        self.lr_dev = torch.full((1,), float(lr), dtype=torch.float32, device=dev)
        self.grad_norm = torch.zeros(1, dtype=torch.float32, device=dev)
        self.clip_coef = torch.ones(1, dtype=torch.float32, device=dev)
        L = nat.lib()
        self.clip_ws = torch.empty(L.mmf_grad_clip_workspace_bytes(), dtype=torch.uint8, device=dev)
        self.last_loss = torch.zeros((), device=dev)
        self._direct_steps = 0   # optimizer steps that read the backward's gradient buffer in place
        # modules whose backward writes their parameters' gradients into a flat buffer of their own
        # (fusion.HybridFusion's grad sink), and the parameters no such module owns
        self._sink_owners = [m for m in model.modules() if hasattr(m, "mmf_grads_consumed")]
        owned = {id(p) for m in self._sink_owners for p in m.parameters()}
        self._unsunk = [p for p in self.flat.params if id(p) not in owned]

    def set_lr(self, lr: float) -> None:
        self.lr_dev.fill_(float(lr))

    def micro_step(self, features, labels, mask=None, sync: bool = True) -> torch.Tensor:
        """One micro-batch: forward, loss / accumulate, backward; `sync` arms the exchange."""
        self.model.train()
        logits = self.model(features, mask)
        if logits.is_cuda and logits.dim() == 2 and logits.dtype == torch.float32 and labels.dtype == torch.int64:
            import mmf_ops   # (the loss and its gradient in one HIP launch)
            loss = mmf_ops.cross_entropy(logits, labels, label_smoothing=self.smoothing)
        else:
            loss = F.cross_entropy(logits, labels, label_smoothing=self.smoothing)
        if sync:
            self.flat.arm()
        (loss / self.accumulate).backward()
        return loss.detach()

    def optimizer_step(self) -> None:
        # one process, one bucket whose gradients the backward left in one buffer of this layout
        # (every HybridFusion backward does): clip + AdamW read it in place, nothing is gathered
        direct = self.flat.direct_grad()
        if direct is not None:
            grad = direct
            self._direct_steps += 1
        else:
            self.flat.finish()
            grad = self.flat.grad
        L = self._nat.lib()
        rc = L.mmf_clip_adamw_step_dev(self.flat.numel, self.flat.flat.data_ptr(), grad.data_ptr(),
                                       self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), self.step_dev.data_ptr(),
                                       self.lr_dev.data_ptr(), float(self.clip_norm), self.grad_norm.data_ptr(),
                                       self.clip_coef.data_ptr(), self.clip_ws.data_ptr(), self.betas[0],
                                       self.betas[1], self.eps, self.wd, 1.0 / self.world,
                                       self._nat.stream_ptr(self.dev))
        self._nat.check(rc, "DPTrainer clip + AdamW")
        self.flat._armed = False
        if direct is not None and self._sink_owners:
            # the gradients lived in the modules' own flat buffers (grad sinks): leave the views
            # attached and mark them consumed -- the next backward writes afresh -- instead of
            # resetting every .grad (one attribute write per parameter and step)
            for m in self._sink_owners:
                if not m.mmf_grads_consumed():
                    for p in m.parameters():
                        p.grad = None
            for p in self._unsunk:
                p.grad = None
            self.flat._fresh = [True] * len(self.flat.groups)
        else:
            self.flat.zero_grad()

    def step(self, batches: Sequence[tuple]) -> torch.Tensor:
        """batches: `accumulate` tuples (features, labels, mask); returns the mean loss."""
        if len(batches) != self.accumulate:
            raise ValueError(f"step: expected {self.accumulate} micro-batches, got {len(batches)}")
        total = torch.zeros((), device=self.dev)
        for i, (feats, labels, mask) in enumerate(batches):
            total = total + self.micro_step(feats, labels, mask, sync=(i == len(batches) - 1))
        self.optimizer_step()
        self.last_loss = total / len(batches)
        return self.last_loss

