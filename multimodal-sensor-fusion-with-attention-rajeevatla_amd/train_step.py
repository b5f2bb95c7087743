"""Data-parallel training step over the fused HybridFusion hot path.

The reference trains one process on CPU (src/train.py:511-524, devices=1);
this is the MI355X-native equivalent of its per-step work for the fusion
model: forward -> CrossEntropyLoss(label_smoothing=0.05)
(src/train.py:185-186,310) -> backward (parameter AND input grads) ->
one RCCL all-reduce of the gradients (world > 1) -> global-norm gradient
clipping (gradient_clip_norm 1.0: config/base.yaml:74, src/train.py:416-430)
-> AdamW (src/train.py:374-414; lr / weight decay from config/base.yaml:69-70).  Nothing else crosses GPUs: samples are independent
(no op mixes samples), so the batch is sharded and the weights replicated.

Layout: every parameter of the model is re-pointed into ONE contiguous fp32
buffer and its gradient into another, so the exchange is a single all-reduce
of the flat gradient and AdamW is one kernel over flat buffers.  All buffers
are allocated up front; the per-step work is pure kernel enqueues on the
current stream (fwd / CE / bwd / clip / AdamW through include/mmfusion.h), so
the step is captured once into a hipGraph and replayed.  The learning rate and
the clip factor live in device scalars that the replayed kernels read, so an LR
scheduler (set_lr / cosine_annealing_lr) needs no re-capture, and load_batch()
copies each new batch into the static input buffers the graph reads.

Gradient accumulation (Lightning's accumulate_grad_batches, config/base.yaml:75
gradient_accumulation): with accumulate = k the step's batch is k micro-batches of B/k samples
run one after the other through forward -> CE (loss scaled by 1/k, as Lightning scales it) ->
backward, the micro-batch gradients summed on the device (mmf_grad_accumulate) before the
exchange and the optimizer -- the memory of one micro-batch, the gradient of the whole batch.
"""

from __future__ import annotations

import math

import ctypes
import os
import sys
from typing import Dict, List, Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import mmf_native as _nat  # noqa: E402
from fusion import HybridFusion  # noqa: E402


def shard_batch(feats: List[torch.Tensor], mask: torch.Tensor, labels: torch.Tensor, rank: int,
                world: int):
    """Rank `rank`'s contiguous slice of a global batch (equal shards: B % world == 0).

    Equal shards keep the DP gradient exact: each rank's CE is a mean over its
    B/world samples, so the sum of the ranks' gradients divided by world is the
    mean-CE gradient of the whole batch.
    """
    B = mask.size(0)
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    if B % world:
        raise ValueError(f"global batch {B} is not divisible by world size {world}")
    n = B // world
    sl = slice(rank * n, (rank + 1) * n)
    return [f[sl] for f in feats], mask[sl], labels[sl]


def allreduce_flat(grad: torch.Tensor, process_group=None, world: int = 1) -> None:
    """The one data-path exchange of DP training: sum the flat gradient over ranks.

    A single collective over one contiguous buffer (1.77 MiB at C2): RCCL
    (backend "nccl") on MI355X, gloo in the CPU tests.  The 1/world average is
    folded into AdamW's gradient scale (mmf_adamw_step gscale), so no extra pass.
    """
    if world > 1:
        torch.distributed.all_reduce(grad, group=process_group)


def cosine_annealing_lr(epoch: int, base_lr: float, t_max: int, eta_min: Optional[float] = None) -> float:
    """torch.optim.lr_scheduler.CosineAnnealingLR in closed form, as the reference configures it
    (T_max = max_epochs, eta_min = learning_rate / 100, stepped per epoch; src/train.py:394-402)."""
    if eta_min is None:
        eta_min = base_lr / 100
    return eta_min + (base_lr - eta_min) * (1 + math.cos(math.pi * epoch / t_max)) / 2


class HybridTrainStep:
    """One optimizer step of the fusion model on the HIP path: fwd -> CE -> bwd ->
    [all-reduce] -> clip -> AdamW.  Defaults are config/base.yaml's training keys."""

    def __init__(self, model: HybridFusion, feats: List[torch.Tensor], mask: torch.Tensor,
                 labels: torch.Tensor, lr: float = 1e-3, weight_decay: float = 1e-4,
                 betas=(0.9, 0.999), eps: float = 1e-8, label_smoothing: float = 0.05,
                 gradient_clip_norm: float = 1.0, process_group=None, input_grads: bool = True,
                 accumulate: int = 1, fuse_clip: bool = True, overlap: Optional[bool] = None):
        dev = mask.device
        _nat.require_device(mask, "training inputs")
        self.model = model.train()
        self.dev = dev
        self.wd, self.betas, self.eps = weight_decay, betas, eps
        self.smoothing = label_smoothing
        self.clip_norm = gradient_clip_norm
        self.pg = process_group
        self.world = torch.distributed.get_world_size(process_group) if process_group is not None else 1
        # dropout state: the module's own {seed, offset} buffer, which every step advances on the
        # device -- a second step object on the same model (a new batch shape, the next epoch)
        # continues the stream instead of repeating its masks.  Every rank starts from the same
        # seed (identical weights), so the rank is folded into the module's Philox key once
        # (as harness.DPTrainer does), or the dropout streams would repeat across ranks
        if self.world > 1 and not getattr(model, "_mmf_rank_folded", False):
            with torch.no_grad():
                model._rng_state[0] ^= torch.distributed.get_rank(process_group) * 0x9E3779B1
            model._mmf_rank_folded = True
        self.rng = model._rng_state
        # static input buffers (graph replays read these addresses)
        self.x = [_nat.f32c(f.to(dev)).clone() for f in feats]
        self.mask = _nat.f32c(mask).clone()
        self.labels = labels.to(dev, torch.int64).contiguous().clone()
        self.accumulate = int(accumulate)
        nb = self.mask.size(0)
        if self.accumulate < 1 or nb % self.accumulate:
            raise ValueError(f"accumulate={accumulate}: the batch of {nb} samples does not split into equal micro-batches")
        self.micro = nb // self.accumulate      # samples per micro-batch
        self.plan = model._plan([x[:self.micro] for x in self.x], False)
        d = self.plan.desc
        params = self.plan.params(model)
        n = self.plan.num_param_elems
        # flat buffers (zero padding between tensors stays zero under AdamW)
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(n, dtype=torch.float32, device=dev)
        for off, p in zip(self.plan.offsets, params):
            k = p.numel()
            self.flat[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.flat[off:off + k].view_as(p)
        self.params = params
        self.gviews = self.plan.grad_views(self.grad, params)
        self.exp_avg = torch.zeros_like(self.flat)
        self.exp_avg_sq = torch.zeros_like(self.flat)
        self.step_dev = torch.zeros(1, dtype=torch.int64, device=dev)
        self.lr_dev = torch.full((1,), float(lr), dtype=torch.float32, device=dev)
        self.grad_norm = torch.zeros(1, dtype=torch.float32, device=dev)   # pre-clip total norm
        self.clip_coef = torch.ones(1, dtype=torch.float32, device=dev)
        L = _nat.lib()
        self.clip_ws = torch.empty(L.mmf_grad_clip_workspace_bytes(), dtype=torch.uint8, device=dev)
        self.saved = torch.empty(L.mmf_hybrid_saved_bytes(ctypes.byref(d)), dtype=torch.uint8, device=dev)
        self.ws = torch.empty(L.mmf_hybrid_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device=dev)
        # the buffer contract: a step under other plan switches (MMF_*) or a layout beyond these
        # capacities is refused by the library (RuntimeError) before any launch
        d.saved_capacity, d.workspace_capacity = self.saved.numel(), self.ws.numel()
        # the one-call step's arrival counts: zero once, every call leaves them zero
        self.sync = torch.zeros(L.mmf_hybrid_train_sync_bytes(ctypes.byref(d)), dtype=torch.uint8, device=dev)
        self.logits = torch.empty(nb, d.num_classes, dtype=torch.float32, device=dev)
        self.fw = torch.empty(nb, d.num_modalities, dtype=torch.float32, device=dev)
        self.dlogits = torch.empty_like(self.logits)
        self.losses = torch.zeros(self.accumulate, dtype=torch.float32, device=dev)   # per micro-batch
        self.dx = [torch.empty_like(x) for x in self.x] if input_grads else []
        self.pstruct = self.plan.param_struct(params)
        self.gstruct = self.plan.param_struct(self.gviews)
        # micro-batches after the first write their gradient here; it is added into self.grad
        self.grad_mb = torch.zeros_like(self.grad) if self.accumulate > 1 else None
        self.gstruct_mb = (self.plan.param_struct(self.plan.grad_views(self.grad_mb, params))
                           if self.grad_mb is not None else None)
        # per micro-batch pointer tables (row offsets into the static buffers)
        self.xarr = [_nat.ptr_array([x[i * self.micro:].data_ptr() for x in self.x]) for i in range(self.accumulate)]
        self.dxarr = ([_nat.ptr_array([t[i * self.micro:].data_ptr() for t in self.dx]) for i in range(self.accumulate)]
                      if input_grads else None)
        # one process, one micro-batch: step() has the train step write the clip norm's partials itself
        # (the L = 1 plan in its weight-gradient launch) and advance the step counter, and the
        # optimizer runs the update launch only
        self.fuse_clip = bool(fuse_clip) and self.world == 1 and self.accumulate == 1 and not overlap
        self._fused_pending = False   # partials written and the counter advanced by the last fwd/bwd
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        # several ranks: the exchange in two buckets overlapped with the backward.  The plan's
        # parameter order puts the modality projections first, so the flat gradient is
        # [projections | pairs, gates, classifier]; every gradient of the second span is final
        # after part 1 of the train step (the attention backward), the projections' after part 2
        # (dZ, dX, their weight gradients).  Part 1's bucket is all-reduced while part 2 runs.
        # (overlap=True with one rank: the same bucketed path, exchanges of one rank -- how the
        # RCCL calls and their stream order are exercised on a one-GPU box)
        self.overlap = (self.world > 1) if overlap is None else (bool(overlap) and self.pg is not None)
        split = self.plan.offsets[2 * d.num_modalities] if len(self.plan.offsets) > 2 * d.num_modalities else n
        self.bucket_spans = ((split, n), (0, split))    # (issued after part 1, after part 2)
        self.graph2: Optional[torch.cuda.CUDAGraph] = None

    @property
    def loss(self) -> torch.Tensor:
        """Mean CE loss of the last step (over its micro-batches).  Reading it first checks the
        one-launch step's status (check_status: a host read of the sync buffer's error word)."""
        self.check_status()
        return self.losses.mean() if self.accumulate > 1 else self.losses

    def check_status(self) -> None:
        """Raise RuntimeError if a train step issued so far had a bounded inter-workgroup wait give
        up (the launch-lean L = 1 step, mmf_hybrid_train_status): that step's gradients were
        incomplete (its loss NaN, its update a zero gradient).  The error word is cleared and the
        device already reset the sync words, so the next step runs clean."""
        L = _nat.lib()
        rc = L.mmf_hybrid_train_status(ctypes.byref(self.plan.desc), self.sync.data_ptr(), 1,
                                       _nat.stream_ptr(self.dev))
        _nat.check(rc, "train step status")

    # ---------------------------------------------------------------- host controls
    def set_lr(self, lr: float) -> None:
        """New learning rate for the next steps (a device write; no re-capture)."""
        self.lr_dev.fill_(float(lr))

    @property
    def lr(self) -> float:
        return float(self.lr_dev.item())

    def load_batch(self, feats: List[torch.Tensor], mask: torch.Tensor, labels: torch.Tensor) -> None:
        """Copy the next batch into the static input buffers the (captured) step reads.
        Shapes must equal the construction batch's (the plan and the graph are fixed)."""
        if len(feats) != len(self.x):
            raise ValueError(f"load_batch: expected {len(self.x)} modalities, got {len(feats)}")
        for i, (dst, src) in enumerate(zip(self.x, feats)):
            if tuple(src.shape) != tuple(dst.shape):
                raise ValueError(f"load_batch: modality {i} has shape {tuple(src.shape)}, expected {tuple(dst.shape)}")
        if tuple(mask.shape) != tuple(self.mask.shape) or tuple(labels.shape) != tuple(self.labels.shape):
            raise ValueError(f"load_batch: mask / labels shapes {tuple(mask.shape)} / {tuple(labels.shape)}, "
                             f"expected {tuple(self.mask.shape)} / {tuple(self.labels.shape)}")
        for dst, src in zip(self.x, feats):
            dst.copy_(src, non_blocking=True)
        self.mask.copy_(mask, non_blocking=True)
        self.labels.copy_(labels, non_blocking=True)

    # ---------------------------------------------------------------- stages
    def forward_backward(self) -> None:
        """Per micro-batch: forward -> CE (loss / accumulate) -> backward in one library call
        (mmf_hybrid_train_step: three launches on the L = 1 plan), then the gradient added into
        the accumulated one.  Gradients only: the optimizer state (its step counter included) is
        untouched until optimizer_step()."""
        self._forward_backward(False)

    def _forward_backward(self, fused: bool, part: int = 0) -> None:
        """fused (step() with fuse_clip): the train step also writes the clip norm's partials and
        advances the optimizer's step counter, for the one-launch update of optimizer_step().
        part (the overlapped exchange): 1 = every micro-batch but the last whole, the last one's
        mmf_hybrid_train_step_part 1 (every gradient but the projections'); 2 = the last
        micro-batch's part 2; 0 = everything."""
        L = _nat.lib()
        d = self.plan.desc
        st = _nat.stream_ptr(self.dev)
        C, M, b = d.num_classes, d.num_modalities, self.micro
        last = self.accumulate - 1
        for i in range(self.accumulate):
            if part == 2 and i < last:
                continue
            pi = part if i == last else 0
            g = self.gstruct if i == 0 else self.gstruct_mb
            rc = L.mmf_hybrid_train_step_part(pi, ctypes.byref(d), ctypes.byref(self.pstruct),
                                         ctypes.cast(self.xarr[i], ctypes.c_void_p), self.mask[i * b:].data_ptr(),
                                         self.labels[i * b:].data_ptr(), self.smoothing, 1.0 / self.accumulate,
                                         self.rng.data_ptr(), self.saved.data_ptr(), self.ws.data_ptr(),
                                         self.sync.data_ptr(), self.logits[i * b:].data_ptr(),
                                         self.fw[i * b:].data_ptr(), self.losses[i:].data_ptr(),
                                         self.dlogits[i * b:].data_ptr(), ctypes.byref(g),
                                         ctypes.cast(self.dxarr[i], ctypes.c_void_p) if self.dxarr else None,
                                         self.clip_ws.data_ptr() if fused else None,
                                         self.step_dev.data_ptr() if fused else None,
                                         self.grad.data_ptr(), self.grad.numel(), st)
            _nat.check(rc, "train step (forward, cross-entropy, backward)")
            self._fused_pending = fused
            if i > 0:
                # the micro-batch's gradient added into the accumulated one: all of it, or the
                # span this part finished
                lo, hi = (0, self.grad.numel()) if pi == 0 else self.bucket_spans[pi - 1]
                if hi > lo:
                    rc = L.mmf_grad_accumulate(hi - lo, self.grad_mb[lo:].data_ptr(), self.grad[lo:].data_ptr(), st)
                    _nat.check(rc, "gradient accumulation")

    def allreduce(self) -> None:
        allreduce_flat(self.grad, self.pg, self.world)

    def optimizer_step(self) -> None:
        """Clip the (rank-averaged) gradient to gradient_clip_norm, then AdamW; both read
        their scalars on the device.  After step()'s fused forward / backward (fuse_clip: one
        process, one micro-batch) the train step already wrote the norm's partials and advanced
        the step counter: one launch; otherwise the reduction pass and the update (two)."""
        L = _nat.lib()
        st = _nat.stream_ptr(self.dev)
        gscale = 1.0 / self.world
        fn = L.mmf_clip_adamw_apply_dev if self._fused_pending else L.mmf_clip_adamw_step_dev
        self._fused_pending = False
        rc = fn(self.flat.numel(), self.flat.data_ptr(), self.grad.data_ptr(), self.exp_avg.data_ptr(),
                self.exp_avg_sq.data_ptr(), self.step_dev.data_ptr(), self.lr_dev.data_ptr(), float(self.clip_norm),
                self.grad_norm.data_ptr(), self.clip_coef.data_ptr(), self.clip_ws.data_ptr(), self.betas[0],
                self.betas[1], self.eps, self.wd, gscale, st)
        _nat.check(rc, "clip + AdamW")

    # ---------------------------------------------------------------- driver
    def replay_pays(self) -> bool:
        """Whether capturing the step into a graph makes it faster.  Not for the launch-lean L = 1
        plan in one process (mmf_hybrid_lean_l1): its step is three short launches, and the graph
        replay's boundary costs more than the dispatches it saves -- C2-L1 0.0607-0.0615 ms per
        step replayed against 0.0573-0.0574 ms launched eagerly (profiles/r05/l1_eager/).  bench.py
        asks this; capture() still captures when called."""
        L = _nat.lib()
        return not (self.world == 1 and not self.overlap and L.mmf_hybrid_lean_l1(ctypes.byref(self.plan.desc)) == 1)

    def capture(self) -> None:
        """Capture fwd+CE+bwd (and clip + AdamW when single-process) into one hipGraph; with
        several ranks, the train step's two parts into two graphs (the exchange of the first
        bucket runs between their replays, outside the graphs)."""
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):
            self.forward_backward()     # warm the path outside capture (gradients only)
        torch.cuda.current_stream(self.dev).wait_stream(s)
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        if self.overlap:
            with torch.cuda.graph(g):
                self._forward_backward(False, 1)
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2):
                self._forward_backward(False, 2)
            self.graph2 = g2
        else:
            with torch.cuda.graph(g):
                self._forward_backward(self.fuse_clip)
                if self.world == 1:
                    self.optimizer_step()
        self._fused_pending = False
        self.graph = g

    def _bucket(self, k: int) -> torch.Tensor:
        lo, hi = self.bucket_spans[k]
        return self.grad[lo:hi]

    def step(self) -> None:
        if self.overlap:
            # part 1 -> exchange of its bucket (RCCL on its own stream, after part 1) while part 2
            # runs -> exchange of the projections' bucket -> wait both -> clip + AdamW
            self.graph.replay() if self.graph is not None else self._forward_backward(False, 1)
            works = [torch.distributed.all_reduce(self._bucket(0), group=self.pg, async_op=True)]
            self.graph2.replay() if self.graph2 is not None else self._forward_backward(False, 2)
            if self.bucket_spans[1][1] > self.bucket_spans[1][0]:
                works.append(torch.distributed.all_reduce(self._bucket(1), group=self.pg, async_op=True))
            for w in works:
                w.wait()
            self.optimizer_step()
            return
        if self.graph is not None:
            self.graph.replay()
            if self.world > 1:
                # (overlap=False with several ranks: the graph holds forward + backward only; the
                # exchange and the update run after the replay, outside it)
                self.allreduce()
                self.optimizer_step()
            return
        self._forward_backward(self.fuse_clip)
        self.allreduce()
        self.optimizer_step()

    def named_grads(self) -> Dict[str, torch.Tensor]:
        return dict(zip(self.plan.names, self.gviews))

    def saved_activation(self, what: str, index: int = 0) -> torch.Tensor:
        """A view of an activation the last forward left in ``saved`` (the last micro-batch's):
        ``what = "proj"``: P_m of modality ``index`` after its ReLU and dropout, (micro, L_m, H)
        (src/fusion.py:364-374); ``what = "cls_hidden"``: the classifier's hidden layer after its
        ReLU and dropout, (micro, H) (src/fusion.py:413-419).  The backward takes ReLU'(z) as
        (value > 0) from these (mmf_hybrid_saved_region)."""
        kinds = {"proj": 0, "cls_hidden": 1}
        if what not in kinds:
            raise ValueError(f"saved_activation: what must be one of {sorted(kinds)} (got {what!r})")
        d = self.plan.desc
        off, nb = ctypes.c_uint64(), ctypes.c_uint64()
        _nat.check(_nat.lib().mmf_hybrid_saved_region(ctypes.byref(d), kinds[what], int(index), ctypes.byref(off),
                                                      ctypes.byref(nb)), "mmf_hybrid_saved_region")
        flat = self.saved[off.value:off.value + nb.value].view(torch.float32)
        if what == "cls_hidden":
            return flat.view(self.micro, d.hidden)
        return flat.view(self.micro, -1, d.hidden)
