"""Data-parallel training step over the fused HybridFusion hot path.

The reference trains one process on CPU (src/train.py:511-524, devices=1);
this is the MI355X-native equivalent of its per-step work for the fusion
model: forward -> CrossEntropyLoss(label_smoothing=0.05)
(src/train.py:185-186,310) -> backward (parameter AND input grads) ->
one RCCL all-reduce of the gradients (world > 1) -> AdamW
(src/train.py:374-414).  Nothing else crosses GPUs: samples are independent
(no op mixes samples), so the batch is sharded and the weights replicated.

Layout: every parameter of the model is re-pointed into ONE contiguous fp32
buffer and its gradient into another, so the exchange is a single all-reduce
of the flat gradient and AdamW is one kernel over flat buffers.  All buffers
are allocated up front; the per-step work is pure kernel enqueues on the
current stream (fwd / CE / bwd / AdamW through include/mmfusion.h), so the
step is captured once into a hipGraph and replayed.
"""

from __future__ import annotations

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


class HybridTrainStep:
    def __init__(self, model: HybridFusion, feats: List[torch.Tensor], mask: torch.Tensor,
                 labels: torch.Tensor, lr: float = 1e-3, weight_decay: float = 0.01,
                 betas=(0.9, 0.999), eps: float = 1e-8, label_smoothing: float = 0.05,
                 process_group=None, input_grads: bool = True):
        dev = mask.device
        _nat.require_device(mask, "training inputs")
        self.model = model.train()
        self.dev = dev
        self.lr, self.wd, self.betas, self.eps = lr, weight_decay, betas, eps
        self.smoothing = label_smoothing
        self.pg = process_group
        self.world = torch.distributed.get_world_size(process_group) if process_group is not None else 1
        # static input buffers (graph replays read these addresses)
        self.x = [_nat.f32c(f.to(dev)).clone() for f in feats]
        self.mask = _nat.f32c(mask).clone()
        self.labels = labels.to(dev, torch.int64).contiguous().clone()
        self.plan = model._plan(self.x, False)
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
        L = _nat.lib()
        self.saved = torch.empty(L.mmf_hybrid_saved_bytes(ctypes.byref(d)), dtype=torch.uint8, device=dev)
        self.ws = torch.empty(L.mmf_hybrid_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device=dev)
        self.logits = torch.empty(d.batch, d.num_classes, dtype=torch.float32, device=dev)
        self.fw = torch.empty(d.batch, d.num_modalities, dtype=torch.float32, device=dev)
        self.dlogits = torch.empty_like(self.logits)
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self.dx = [torch.empty_like(x) for x in self.x] if input_grads else []
        self.pstruct = self.plan.param_struct(params)
        self.gstruct = self.plan.param_struct(self.gviews)
        self.xarr = _nat.ptr_array([x.data_ptr() for x in self.x])
        self.dxarr = _nat.ptr_array([t.data_ptr() for t in self.dx]) if input_grads else None
        self.graph: Optional[torch.cuda.CUDAGraph] = None

    # ---------------------------------------------------------------- stages
    def forward_backward(self) -> None:
        L = _nat.lib()
        d = self.plan.desc
        st = _nat.stream_ptr(self.dev)
        rc = L.mmf_hybrid_forward(ctypes.byref(d), ctypes.byref(self.pstruct),
                                  ctypes.cast(self.xarr, ctypes.c_void_p), self.mask.data_ptr(),
                                  self.model._rng_state.data_ptr(), self.saved.data_ptr(),
                                  self.logits.data_ptr(), self.fw.data_ptr(), None, st)
        _nat.check(rc, "train forward")
        rc = L.mmf_cross_entropy_ls(d.batch, d.num_classes, self.logits.data_ptr(), self.labels.data_ptr(),
                                    self.smoothing, 1.0, self.loss.data_ptr(), self.dlogits.data_ptr(), st)
        _nat.check(rc, "train cross-entropy")
        rc = L.mmf_hybrid_backward(ctypes.byref(d), ctypes.byref(self.pstruct),
                                   ctypes.cast(self.xarr, ctypes.c_void_p), self.mask.data_ptr(),
                                   self.saved.data_ptr(), self.dlogits.data_ptr(), self.ws.data_ptr(),
                                   ctypes.byref(self.gstruct),
                                   ctypes.cast(self.dxarr, ctypes.c_void_p) if self.dxarr else None, st)
        _nat.check(rc, "train backward")

    def allreduce(self) -> None:
        allreduce_flat(self.grad, self.pg, self.world)

    def optimizer_step(self) -> None:
        rc = _nat.lib().mmf_adamw_step(self.flat.numel(), self.flat.data_ptr(), self.grad.data_ptr(),
                                       self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
                                       self.step_dev.data_ptr(), self.lr, self.betas[0], self.betas[1],
                                       self.eps, self.wd, 1.0 / self.world, _nat.stream_ptr(self.dev))
        _nat.check(rc, "AdamW")

    # ---------------------------------------------------------------- driver
    def capture(self) -> None:
        """Capture fwd+CE+bwd (and AdamW when single-process) into one hipGraph."""
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):
            self.forward_backward()     # warm the path outside capture
        torch.cuda.current_stream(self.dev).wait_stream(s)
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.forward_backward()
            if self.world == 1:
                self.optimizer_step()
        self.graph = g

    def step(self) -> None:
        if self.graph is not None:
            self.graph.replay()
            if self.world > 1:
                self.allreduce()
                self.optimizer_step()
            return
        self.forward_backward()
        self.allreduce()
        self.optimizer_step()

    def named_grads(self) -> Dict[str, torch.Tensor]:
        return dict(zip(self.plan.names, self.gviews))
