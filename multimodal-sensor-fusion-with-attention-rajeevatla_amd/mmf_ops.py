"""The C-ABI entry points as torch operators (``torch.ops.mmfusion.*``).

The reference compiles its fusion model and encoders with
``torch.compile(backend="inductor", mode="reduce-overhead")`` (src/train.py:193-231,
config/base.yaml:76-79).  Each library entry point is registered here with
``torch.library.custom_op`` (the implementation calls the ctypes binding, mmf_native),
a fake (meta) implementation giving output shapes without touching the device, and an
autograd formula (``register_autograd``) that calls the matching backward entry point.
TorchDynamo therefore traces the drop-in modules into one graph (no graph breaks),
AOTAutograd sees the forward and backward operators, and the "reduce-overhead" HIP
graphs capture the library's launches like any other kernel.  Eager calls dispatch to
the same implementations, so eager and compiled runs execute identical kernels.

The operators are functional (mutate nothing): the dropout state {seed, offset} is an
input, and the forward returns the advanced state, which the module copies back into
its buffer.  Descriptors travel as int lists (their ctypes structs are rebuilt, and
cached, inside the implementation); parameter gradients come back as one flat buffer
that the autograd formula slices into per-parameter views.

Operators (csrc entry point, reference interface):
  hybrid_fwd / hybrid_bwd          mmf_hybrid_forward / _backward    src/fusion.py:331-427
  cma_fwd / cma_bwd                mmf_cma_forward / _backward       src/attention.py:68-146
  adaptive_weights_fwd / _bwd      mmf_adaptive_weights(_backward)   src/fusion.py:429-479
  attention_pool_fwd / _bwd        mmf_attention_pool_*              src/encoders.py:313-336
  late_weights_fwd / _bwd          mmf_late_fusion_*                 src/fusion.py:228-245
  lstm_layer_fwd / _bwd            mmf_lstm_forward / _backward      src/encoders.py:135-166
"""

from __future__ import annotations

import ctypes
import os
import sys
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch
from torch import Tensor

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import mmf_native as _nat  # noqa: E402

ALIGN = 64   # every tensor of a flat gradient buffer starts on a 256-byte boundary


_OFFS: Dict[tuple, Tuple[List[int], int]] = {}


def flat_offsets(numels: Sequence[int]) -> Tuple[List[int], int]:
    key = tuple(int(n) for n in numels)
    hit = _OFFS.get(key)
    if hit is not None:
        return hit
    offs, off = [], 0
    for n in key:
        offs.append(off)
        off += -(-n // ALIGN) * ALIGN
    _OFFS[key] = (offs, off)
    return offs, off


def _views(flat: Tensor, params: Sequence[Tensor], offsets: Sequence[int]) -> List[Tensor]:
    return [flat[o:o + p.numel()].view_as(p) for o, p in zip(offsets, params)]


# ============================================================================ HybridFusion
# idesc = [B, M, H, heads, C, training, return_attention, precision, P,
#          seq_len[0..M), in_dim[0..M), pair_q[0..P), pair_k[0..P)]
_HDESC: Dict[tuple, "_nat.HybridDesc"] = {}


def hybrid_idesc(batch: int, hidden: int, heads: int, classes: int, seq: Sequence[int], dims: Sequence[int],
                 pairs: Sequence[Tuple[int, int]], training: bool, return_attention: bool, precision: int) -> List[int]:
    M = len(seq)
    return ([batch, M, hidden, heads, classes, int(training), int(return_attention), precision, len(pairs)]
            + [int(s) for s in seq] + [int(x) for x in dims] + [q for q, _ in pairs] + [k for _, k in pairs])


def hybrid_desc(idesc: Sequence[int], dropout: float) -> "_nat.HybridDesc":
    """The C-ABI descriptor of an idesc, cached per (idesc, dropout, plan switches): its plan_flags
    are the MMF_* plan switches in force now (mmf_hybrid_plan_flags), so buffers sized from it match
    the layout the library computes; the callers set saved_capacity / workspace_capacity to the
    buffers they pass (include/mmfusion.h's buffer contract)."""
    flags = int(_nat.lib().mmf_hybrid_plan_flags())
    key = (tuple(idesc), float(dropout), flags)
    d = _HDESC.get(key)
    if d is not None:
        return d
    v = tuple(int(x) for x in key[0])
    B, M, H, heads, C, training, ret, prec, P = v[:9]
    d = _nat.HybridDesc()
    d.batch, d.num_modalities, d.hidden, d.num_heads, d.num_classes = B, M, H, heads, C
    for m in range(M):
        d.seq_len[m] = v[9 + m]
        d.in_dim[m] = v[9 + M + m]
    d.num_pairs = P
    for g in range(P):
        d.pair_q[g] = v[9 + 2 * M + g]
        d.pair_k[g] = v[9 + 2 * M + P + g]
    d.dropout, d.training, d.return_attention, d.matmul_precision = float(dropout), training, ret, prec
    d.plan_flags = flags
    _HDESC[key] = d
    return d


_HMETA: Dict[tuple, tuple] = {}


def _hybrid_meta(idesc: Sequence[int]):
    key = tuple(idesc)
    hit = _HMETA.get(key)
    if hit is None:
        hit = _HMETA[key] = _hybrid_meta_of(key)
    return hit


def _hybrid_meta_of(idesc: Sequence[int]):
    v = [int(x) for x in idesc]
    B, M, H, heads, C, _, ret, _, P = v[:9]
    seq = [max(s, 1) for s in v[9:9 + M]]
    pq, pk = v[9 + 2 * M:9 + 2 * M + P], v[9 + 2 * M + P:9 + 2 * M + 2 * P]
    maps = [(B, heads, seq[q], seq[k]) for q, k in zip(pq, pk)] if ret else []
    return B, M, C, maps


_PSTRUCT: Dict[tuple, "_nat.HybridParams"] = {}


def _hybrid_params_struct(params: Sequence[Tensor], M: int, P: int) -> "_nat.HybridParams":
    """The C-ABI parameter (or gradient) struct for these tensors' addresses, cached per address
    set (a training loop passes the same parameters every step; gradient buffers recur through
    the caching allocator)."""
    return _struct_from_ptrs(tuple(map(Tensor.data_ptr, params)), M, P)


def _grad_struct(flat: Tensor, offsets: Sequence[int], M: int, P: int) -> "_nat.HybridParams":
    """The gradient struct of a flat gradient buffer laid out at `offsets` (addresses by
    arithmetic: no per-parameter views to build)."""
    base = flat.data_ptr()
    return _struct_from_ptrs(tuple(base + 4 * o for o in offsets), M, P)


def _struct_from_ptrs(ptrs: tuple, M: int, P: int) -> "_nat.HybridParams":
    key = (M, P, ptrs)
    s = _PSTRUCT.get(key)
    if s is not None:
        return s
    s = _nat.HybridParams()
    it = iter(ptrs)
    nxt = lambda: next(it)  # noqa: E731
    for m in range(M):
        s.proj[m] = _nat.Linear(nxt(), nxt())
    for g in range(P):
        s.q[g] = _nat.Linear(nxt(), nxt())
        s.k[g] = _nat.Linear(nxt(), nxt())
        s.v[g] = _nat.Linear(nxt(), nxt())
        s.o[g] = _nat.Linear(nxt(), nxt())
    for m in range(M):
        s.gate[m] = _nat.Linear(nxt(), nxt())
    s.cls1 = _nat.Linear(nxt(), nxt())
    s.cls2 = _nat.Linear(nxt(), nxt())
    if len(_PSTRUCT) > 256:
        _PSTRUCT.clear()
    _PSTRUCT[key] = s
    return s


def hybrid_fwd_impl(idesc: Sequence[int], dropout: float, rng_state: Tensor, mask: Tensor, xs: Sequence[Tensor],
                    params: Sequence[Tensor], rng_inplace: bool = False):
    """mmf_hybrid_forward on the caller's stream -> logits (B, C), fusion_weights (B, M), saved
    (bytes), advanced rng state, attention maps.  (The hybrid_fwd operator's body, and the eager
    autograd functions': one implementation.)  The operator is functional: the library advances a
    clone of the dropout state, returned; rng_inplace (the eager functions) advances the caller's
    buffer itself and returns it."""
    L = _nat.lib()
    d = hybrid_desc(idesc, dropout)
    B, M, C, mshapes = _hybrid_meta(idesc)
    dev = mask.device
    saved = torch.empty(_nat.lib().mmf_hybrid_saved_bytes(ctypes.byref(d)), dtype=torch.uint8, device=dev)
    d.saved_capacity = saved.numel()
    logits = torch.empty(B, C, dtype=torch.float32, device=dev)
    fw = torch.empty(B, M, dtype=torch.float32, device=dev)
    maps = [torch.empty(s, dtype=torch.float32, device=dev) for s in mshapes]
    rng_next = rng_state if rng_inplace else rng_state.clone()   # snapshot into `saved`, then advanced
    pstruct = _hybrid_params_struct(params, M, d.num_pairs)
    xarr = _nat.ptr_array([x.data_ptr() for x in xs])
    marr = _nat.ptr_array([t.data_ptr() for t in maps]) if maps else None
    rc = L.mmf_hybrid_forward(ctypes.byref(d), ctypes.byref(pstruct), ctypes.cast(xarr, ctypes.c_void_p),
                              mask.data_ptr(), rng_next.data_ptr(), saved.data_ptr(), logits.data_ptr(),
                              fw.data_ptr(), ctypes.cast(marr, ctypes.c_void_p) if marr else None,
                              _nat.stream_ptr(dev))
    _nat.check(rc, "HybridFusion forward")
    return logits, fw, saved, rng_next, maps


def hybrid_bwd_impl(idesc: Sequence[int], dropout: float, mask: Tensor, xs: Sequence[Tensor],
                    params: Sequence[Tensor], saved: Tensor, dlogits: Tensor, need_dx: Sequence[bool],
                    offsets: Sequence[int], nelem: int, flat: Optional[Tensor] = None):
    """mmf_hybrid_backward -> dx per modality (an empty tensor where not needed), the flat
    parameter gradient.  The library writes every gradient; the buffer is zeroed for the padding
    between them, so a trainer whose flat layout matches (harness.FlatGradBuckets.direct_grad)
    can clip and update from it in place."""
    L = _nat.lib()
    d = hybrid_desc(idesc, dropout)
    M, P = d.num_modalities, d.num_pairs
    dev = mask.device
    ws = torch.empty(_nat.lib().mmf_hybrid_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device=dev)
    # (`saved` came from the forward: a plan switch flipped in between changes the layout this call
    # computes, which the library then finds larger than the forward's buffer, or a different
    # plan_flags descriptor -- refused, not read with another layout)
    d.saved_capacity, d.workspace_capacity = saved.numel(), ws.numel()
    if flat is None:
        flat = torch.zeros(nelem, dtype=torch.float32, device=dev)
    gstruct = _grad_struct(flat, offsets, M, P)
    pstruct = _hybrid_params_struct(params, M, P)
    dxs = [torch.empty_like(x) if need else x.new_empty(0) for x, need in zip(xs, need_dx)]
    xarr = _nat.ptr_array([x.data_ptr() for x in xs])
    dxarr = _nat.ptr_array([t.data_ptr() if need else None for t, need in zip(dxs, need_dx)])
    rc = L.mmf_hybrid_backward(ctypes.byref(d), ctypes.byref(pstruct), ctypes.cast(xarr, ctypes.c_void_p),
                               mask.data_ptr(), saved.data_ptr(), dlogits.data_ptr(), ws.data_ptr(),
                               ctypes.byref(gstruct), ctypes.cast(dxarr, ctypes.c_void_p), _nat.stream_ptr(dev))
    _nat.check(rc, "HybridFusion backward")
    return dxs, flat


@torch.library.custom_op("mmfusion::hybrid_fwd", mutates_args=(), device_types="cuda")
def hybrid_fwd(idesc: List[int], dropout: float, rng_state: Tensor, mask: Tensor, xs: List[Tensor],
               params: List[Tensor]) -> Tuple[Tensor, Tensor, Tensor, Tensor, List[Tensor]]:
    """-> logits (B, C), fusion_weights (B, M), saved (bytes), advanced rng state, attention maps."""
    return hybrid_fwd_impl(idesc, dropout, rng_state, mask, xs, params)


@hybrid_fwd.register_fake
def _(idesc, dropout, rng_state, mask, xs, params):
    d = hybrid_desc(idesc, dropout)
    B, M, C, mshapes = _hybrid_meta(idesc)
    nbytes = _nat.lib().mmf_hybrid_saved_bytes(ctypes.byref(d))
    return (mask.new_empty(B, C), mask.new_empty(B, M), mask.new_empty(nbytes, dtype=torch.uint8),
            torch.empty_like(rng_state), [mask.new_empty(s) for s in mshapes])


@torch.library.custom_op("mmfusion::hybrid_bwd", mutates_args=(), device_types="cuda")
def hybrid_bwd(idesc: List[int], dropout: float, mask: Tensor, xs: List[Tensor], params: List[Tensor],
               saved: Tensor, dlogits: Tensor, need_dx: List[bool], offsets: List[int],
               nelem: int) -> Tuple[List[Tensor], Tensor]:
    """-> dx per modality (an empty tensor where not needed), flat parameter gradient."""
    return hybrid_bwd_impl(idesc, dropout, mask, xs, params, saved, dlogits, need_dx, offsets, nelem)


@hybrid_bwd.register_fake
def _(idesc, dropout, mask, xs, params, saved, dlogits, need_dx, offsets, nelem):
    return [torch.empty_like(x) if need else x.new_empty(0) for x, need in zip(xs, need_dx)], mask.new_empty(nelem)


def _hybrid_setup(ctx, inputs, output):
    idesc, dropout, rng_state, mask, xs, params = inputs
    saved = output[2]
    # unused outputs (the saved bytes, the rng state, the maps) reach the backward as None, not as
    # materialised zeros (a 311 MB fill per C2 backward for `saved`)
    ctx.set_materialize_grads(False)
    ctx.idesc, ctx.dropout, ctx.nx = list(idesc), dropout, len(xs)
    ctx.need_dx = [bool(x.requires_grad) for x in xs]
    ctx.save_for_backward(mask, saved, *xs, *params)


def _hybrid_backward(ctx, dlogits, _dfw, _dsaved, _drng, _dmaps):
    if dlogits is None:
        return None, None, None, None, None, None
    mask, saved, *rest = ctx.saved_tensors
    xs, params = rest[:ctx.nx], rest[ctx.nx:]
    offsets, nelem = flat_offsets([p.numel() for p in params])
    dxs, flat = torch.ops.mmfusion.hybrid_bwd(ctx.idesc, ctx.dropout, mask, list(xs), list(params), saved,
                                              dlogits.contiguous(), ctx.need_dx, offsets, nelem)
    dx = [t if need else None for t, need in zip(dxs, ctx.need_dx)]
    return None, None, None, None, dx, _views(flat, params, offsets)


hybrid_fwd.register_autograd(_hybrid_backward, setup_context=_hybrid_setup)


class GradSink:
    """The flat gradient buffer of one HybridFusion module, for the eager grad-sink path
    (HybridSink): the operator's flat layout (flat_offsets of the operator's parameter order,
    which is the module's registration order), so every parameter's ``.grad`` is a view of it and
    a trainer with the same layout (harness.FlatGradBuckets.direct_grad) clips and updates from it
    in place.

    States between backwards: ``fresh`` -- the next backward WRITES the gradients into the buffer
    (after the parameters' ``.grad`` were set to None, or after ``consumed()``: a trainer that
    applied them); otherwise the parameters' ``.grad`` are the buffer's views holding gradients
    still to be accumulated into (the next backward writes into a scratch buffer and adds it)."""

    def __init__(self, params: Sequence[Tensor]):
        p0 = params[0]
        self.offsets, self.nelem = flat_offsets([p.numel() for p in params])
        self.flat = torch.zeros(self.nelem, dtype=torch.float32, device=p0.device)
        self.views = [self.flat.as_strided(tuple(p.shape), tuple(p.stride()), o) for p, o in zip(params, self.offsets)]
        self.fresh = True

    def matches(self, params: Sequence[Tensor]) -> bool:
        return len(params) == len(self.views) and params[0].device == self.flat.device


_EXT: Any = False   # mmf_torch once loaded and bound; None when not built or MMF_NO_TORCH_EXT is set


def torch_ext():
    """The mmf_torch extension (csrc/torch_bind.cpp: HybridFusion's and the cross-entropy's eager
    autograd nodes in C++ over this library's C-ABI), bound to the entry points of the library
    mmf_native loaded; None when it is not built (mmf_build.build_torch_ext) or MMF_NO_TORCH_EXT=1
    -- then the Python twins (HybridSink, CrossEntropyEager) run the same entry points."""
    global _EXT
    if _EXT is False:
        ext = None
        if not os.environ.get("MMF_NO_TORCH_EXT"):
            try:
                import mmf_torch as ext
            except ImportError:
                ext = None
        if ext is not None:
            L = _nat.lib()
            ext.bind({n: ctypes.cast(getattr(L, n), ctypes.c_void_p).value
                      for n in ("mmf_hybrid_saved_bytes", "mmf_hybrid_workspace_bytes", "mmf_hybrid_forward",
                                "mmf_hybrid_backward", "mmf_cross_entropy_ls", "mmf_last_error")})
        _EXT = ext
    return _EXT


def make_grad_sink(params: Sequence[Tensor], M: int, P: int):
    """The module's flat gradient buffer: mmf_torch.Sink (the C++ node writes into it) when the
    extension is loaded, GradSink otherwise -- one layout (flat_offsets), the same attributes."""
    ext = torch_ext()
    if ext is None:
        return GradSink(params)
    offsets, nelem = flat_offsets([p.numel() for p in params])
    return ext.Sink(list(params), offsets, nelem, M, P)


def _sink_ok(params: Sequence[Tensor]) -> bool:
    """The grad-sink path keeps autograd's semantics for these parameters: every one trainable,
    contiguous fp32 (the layout), and none with a tensor hook (register_hook can rewrite a
    gradient before accumulation: those parameters go through autograd's AccumulateGrad).
    Post-accumulate-grad hooks are called by the sink path itself, after the gradient lands."""
    return all(map(_TRAINABLE, params)) and not any(map(_TENSOR_HOOKS, params))


_TRAINABLE = Tensor.requires_grad.__get__
_TENSOR_HOOKS = Tensor._backward_hooks.__get__


class HybridSink(torch.autograd.Function):
    """Eager HybridFusion with the parameters OUTSIDE the autograd graph: the backward writes
    every parameter gradient straight into the module's GradSink and attaches the sink's views as
    ``.grad`` (what AccumulateGrad would leave there after a first backward, and the sum after
    further ones), so a step pays no per-parameter AccumulateGrad nodes, saved-tensor unpacking or
    gradient views per call -- at the reference's 2-D inputs (launch-bound) those were most of the
    step.  Only the modality inputs (and one anchor parameter, so a graph exists when
    no input requires grad) are autograd inputs.  Inputs: (idesc, dropout, rng_state, mask, owner,
    params, anchor, *xs) with `params` a Python list autograd does not look into."""

    @staticmethod
    def forward(ctx, idesc, dropout, rng_state, mask, owner, params, anchor, *xs):
        logits, fw, saved, _, maps = hybrid_fwd_impl(idesc, dropout, rng_state, mask, xs, params, rng_inplace=True)
        ctx.set_materialize_grads(False)
        ctx.idesc, ctx.dropout, ctx.owner, ctx.params = idesc, dropout, owner, params
        ctx.versions = [p._version for p in params]   # (autograd's in-place check for saved tensors)
        ctx.need_dx = [bool(n) for n in ctx.needs_input_grad[7:]]
        ctx.save_for_backward(mask, saved, *xs)
        ctx.mark_non_differentiable(fw, saved, *maps)
        return (logits, fw, saved, *maps)

    @staticmethod
    def backward(ctx, dlogits, *_unused):
        nx = len(ctx.need_dx)
        if dlogits is None:
            return (None,) * (7 + nx)
        mask, saved, *xs = ctx.saved_tensors
        params = ctx.params
        for i, (p, v) in enumerate(zip(params, ctx.versions)):
            if p._version != v:
                raise RuntimeError("one of the variables needed for gradient computation has been modified by an "
                                   f"inplace operation: HybridFusion parameter {i} (shape {tuple(p.shape)}) is at "
                                   f"version {p._version}; expected version {v} instead.")
        sink = ctx.owner._grad_sink(params)
        grads = [p.grad for p in params]
        if all(g is None for g in grads) or (sink.fresh and all(g is None or g is v for g, v in zip(grads, sink.views))):
            mode = 0          # write into the sink (set_to_none zero_grad, or a trainer consumed it)
        elif all(g is v for g, v in zip(grads, sink.views)):
            mode = 1          # add into the sink (gradients still to be applied)
        else:
            mode = 2          # someone else's .grad tensors: add into them
        dst = sink.flat if mode == 0 else torch.zeros(sink.nelem, dtype=torch.float32, device=sink.flat.device)
        dxs, _ = hybrid_bwd_impl(ctx.idesc, ctx.dropout, mask, xs, params, saved, dlogits.contiguous(), ctx.need_dx,
                                 sink.offsets, sink.nelem, flat=dst)
        if mode == 0:
            for p, g, v in zip(params, grads, sink.views):
                if g is None:
                    p.grad = v
            sink.fresh = False
        elif mode == 1:
            sink.flat.add_(dst)
        else:
            have = [(g, dst.as_strided(tuple(p.shape), tuple(p.stride()), o))
                    for p, g, o in zip(params, grads, sink.offsets) if g is not None]
            if have:
                torch._foreach_add_([g for g, _ in have], [v for _, v in have])
            for p, g, o in zip(params, grads, sink.offsets):
                if g is None:
                    p.grad = dst.as_strided(tuple(p.shape), tuple(p.stride()), o)
        for p in params:   # (what AccumulateGrad does after accumulating)
            hooks = p._post_accumulate_grad_hooks
            if hooks:
                for h in hooks.values():
                    h(p)
        dx = [t if need else None for t, need in zip(dxs, ctx.need_dx)]
        return (None, None, None, None, None, None, None, *dx)


class HybridEager(torch.autograd.Function):
    """The eager-mode twin of the hybrid_fwd / hybrid_bwd operators (HybridFusion.forward outside
    torch.compile): the same implementation functions and the same saved tensors and gradient
    formula, through autograd.Function.apply instead of the custom-op dispatch (the operator's
    Python dispatch, schema checks and argument flattening cost host time every call).  Inputs:
    (idesc, dropout, rng_state, mask, nx, *xs, *params)."""

    @staticmethod
    def forward(ctx, idesc, dropout, rng_state, mask, nx, *tensors):
        xs, params = tensors[:nx], tensors[nx:]
        logits, fw, saved, _, maps = hybrid_fwd_impl(idesc, dropout, rng_state, mask, xs, params, rng_inplace=True)
        ctx.set_materialize_grads(False)
        ctx.idesc, ctx.dropout, ctx.nx = idesc, dropout, nx
        ctx.need_dx = [bool(n) for n in ctx.needs_input_grad[5:5 + nx]]
        ctx.save_for_backward(mask, saved, *xs, *params)
        ctx.mark_non_differentiable(fw, saved, *maps)
        return (logits, fw, saved, *maps)

    @staticmethod
    def backward(ctx, dlogits, *_unused):
        if dlogits is None:
            return (None,) * len(ctx.needs_input_grad)
        mask, saved, *rest = ctx.saved_tensors
        xs, params = rest[:ctx.nx], rest[ctx.nx:]
        offsets, nelem = flat_offsets([p.numel() for p in params])
        dxs, flat = hybrid_bwd_impl(ctx.idesc, ctx.dropout, mask, xs, params, saved, dlogits.contiguous(),
                                    ctx.need_dx, offsets, nelem)
        dx = [t if need else None for t, need in zip(dxs, ctx.need_dx)]
        return (None, None, None, None, None, *dx, *_views(flat, params, offsets))


# ============================================================================ CrossModalAttention
# idesc = [B, lq, lk, query_dim, key_dim, H, heads, mask_mode, training, precision]
_CDESC: Dict[tuple, "_nat.CmaDesc"] = {}


def cma_desc(idesc: Sequence[int], dropout: float) -> "_nat.CmaDesc":
    key = (tuple(int(v) for v in idesc), float(dropout))
    d = _CDESC.get(key)
    if d is None:
        v = key[0]
        d = _nat.CmaDesc(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], float(dropout), v[8], v[9])
        _CDESC[key] = d
    return d


def _cma_struct(params: Sequence[Tensor]) -> "_nat.CmaParams":
    s = _nat.CmaParams()
    for i, name in enumerate(("q", "k", "v", "o")):
        setattr(s, name, _nat.Linear(params[2 * i].data_ptr(), params[2 * i + 1].data_ptr()))
    return s


@torch.library.custom_op("mmfusion::cma_fwd", mutates_args=(), device_types="cuda")
def cma_fwd(idesc: List[int], dropout: float, rng_state: Tensor, query: Tensor, key: Tensor, value: Tensor,
            mask: Optional[Tensor], params: List[Tensor]) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """-> attended (B, Lq, H), weights (B, h, Lq, Lk), saved, advanced rng state."""
    L = _nat.lib()
    d = cma_desc(idesc, dropout)
    dev = query.device
    saved = torch.empty(L.mmf_cma_saved_bytes(ctypes.byref(d)), dtype=torch.uint8, device=dev)
    attended = torch.empty(d.batch, d.lq, d.hidden, dtype=torch.float32, device=dev)
    attn = torch.empty(d.batch, d.num_heads, d.lq, d.lk, dtype=torch.float32, device=dev)
    rng_next = rng_state.clone()
    pstruct = _cma_struct(params)
    rc = L.mmf_cma_forward(ctypes.byref(d), ctypes.byref(pstruct), query.data_ptr(), key.data_ptr(),
                           value.data_ptr(), _nat.ptr(mask), rng_next.data_ptr(), saved.data_ptr(),
                           attended.data_ptr(), attn.data_ptr(), _nat.stream_ptr(dev))
    _nat.check(rc, "CrossModalAttention forward")
    return attended, attn, saved, rng_next


@cma_fwd.register_fake
def _(idesc, dropout, rng_state, query, key, value, mask, params):
    d = cma_desc(idesc, dropout)
    nbytes = _nat.lib().mmf_cma_saved_bytes(ctypes.byref(d))
    return (query.new_empty(d.batch, d.lq, d.hidden), query.new_empty(d.batch, d.num_heads, d.lq, d.lk),
            query.new_empty(nbytes, dtype=torch.uint8), torch.empty_like(rng_state))


@torch.library.custom_op("mmfusion::cma_bwd", mutates_args=(), device_types="cuda")
def cma_bwd(idesc: List[int], dropout: float, query: Tensor, key: Tensor, value: Tensor, mask: Optional[Tensor],
            params: List[Tensor], saved: Tensor, d_att: Tensor, need: List[bool], offsets: List[int],
            nelem: int) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """-> d query, d key, d value (empty where not needed), flat parameter gradient."""
    L = _nat.lib()
    d = cma_desc(idesc, dropout)
    dev = query.device
    ws = torch.empty(L.mmf_cma_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device=dev)
    flat = torch.zeros(nelem, dtype=torch.float32, device=dev)
    gstruct = _cma_struct(_views(flat, params, offsets))
    pstruct = _cma_struct(params)
    outs = [torch.empty_like(t) if n else t.new_empty(0) for t, n in zip((query, key, value), need)]
    ptrs = [t.data_ptr() if n else None for t, n in zip(outs, need)]
    rc = L.mmf_cma_backward(ctypes.byref(d), ctypes.byref(pstruct), query.data_ptr(), key.data_ptr(),
                            value.data_ptr(), _nat.ptr(mask), saved.data_ptr(), d_att.data_ptr(), ws.data_ptr(),
                            ctypes.byref(gstruct), ptrs[0], ptrs[1], ptrs[2], _nat.stream_ptr(dev))
    _nat.check(rc, "CrossModalAttention backward")
    return outs[0], outs[1], outs[2], flat


@cma_bwd.register_fake
def _(idesc, dropout, query, key, value, mask, params, saved, d_att, need, offsets, nelem):
    outs = [torch.empty_like(t) if n else t.new_empty(0) for t, n in zip((query, key, value), need)]
    return outs[0], outs[1], outs[2], query.new_empty(nelem)


def _cma_setup(ctx, inputs, output):
    idesc, dropout, rng_state, query, key, value, mask, params = inputs
    ctx.set_materialize_grads(False)
    ctx.idesc, ctx.dropout, ctx.has_mask = list(idesc), dropout, mask is not None
    ctx.need = [bool(t.requires_grad) for t in (query, key, value)]
    ctx.save_for_backward(query, key, value, mask if mask is not None else query.new_empty(0), output[2], *params)


def _cma_backward(ctx, d_att, _dw, _dsaved, _drng):
    if d_att is None:
        return None, None, None, None, None, None, None, None
    query, key, value, mask, saved, *params = ctx.saved_tensors
    offsets, nelem = flat_offsets([p.numel() for p in params])
    dq, dk, dv, flat = torch.ops.mmfusion.cma_bwd(ctx.idesc, ctx.dropout, query, key, value,
                                                  mask if ctx.has_mask else None, list(params), saved,
                                                  d_att.contiguous(), ctx.need, offsets, nelem)
    dq, dk, dv = (t if n else None for t, n in zip((dq, dk, dv), ctx.need))
    return None, None, None, dq, dk, dv, None, _views(flat, params, offsets)


cma_fwd.register_autograd(_cma_backward, setup_context=_cma_setup)


# ============================================================================ compute_adaptive_weights
def _gates(gparams: Sequence[Tensor]):
    M = len(gparams) // 2
    arr = (_nat.Linear * M)()
    for m in range(M):
        arr[m] = _nat.Linear(gparams[2 * m].data_ptr(), gparams[2 * m + 1].data_ptr())
    return arr


@torch.library.custom_op("mmfusion::adaptive_weights_fwd", mutates_args=(), device_types="cuda")
def adaptive_weights_fwd(mask: Tensor, feats: List[Tensor], gparams: List[Tensor]) -> Tensor:
    L = _nat.lib()
    B, M = mask.shape
    H = feats[0].size(1)
    dev = mask.device
    out = torch.empty(B, M, dtype=torch.float32, device=dev)
    ws = torch.empty(L.mmf_adaptive_weights_workspace_bytes(B, M, H), dtype=torch.uint8, device=dev)
    farr = _nat.ptr_array([f.data_ptr() for f in feats])
    rc = L.mmf_adaptive_weights(B, M, H, ctypes.cast(farr, ctypes.c_void_p), mask.data_ptr(),
                                ctypes.cast(_gates(gparams), ctypes.c_void_p), out.data_ptr(), ws.data_ptr(),
                                _nat.stream_ptr(dev))
    _nat.check(rc, "compute_adaptive_weights")
    return out


@adaptive_weights_fwd.register_fake
def _(mask, feats, gparams):
    return mask.new_empty(mask.shape)


@torch.library.custom_op("mmfusion::adaptive_weights_bwd", mutates_args=(), device_types="cuda")
def adaptive_weights_bwd(mask: Tensor, feats: List[Tensor], gparams: List[Tensor], dweights: Tensor,
                         need_x: bool, need_g: bool) -> Tuple[Tensor, List[Tensor]]:
    """-> dfeats (B, M, H) (empty unless need_x), gate gradients (w, b per modality; empty unless need_g)."""
    L = _nat.lib()
    B, M = mask.shape
    H = feats[0].size(1)
    dev = mask.device
    dfeats = torch.empty(B, M, H, dtype=torch.float32, device=dev) if need_x else mask.new_empty(0)
    ggrads = [torch.empty_like(p) for p in gparams] if need_g else [p.new_empty(0) for p in gparams]
    dgates = (_nat.Linear * M)()
    if need_g:
        for m in range(M):
            dgates[m] = _nat.Linear(ggrads[2 * m].data_ptr(), ggrads[2 * m + 1].data_ptr())
    ws = torch.empty(L.mmf_adaptive_weights_workspace_bytes(B, M, H), dtype=torch.uint8, device=dev)
    farr = _nat.ptr_array([f.data_ptr() for f in feats])
    rc = L.mmf_adaptive_weights_backward(B, M, H, ctypes.cast(farr, ctypes.c_void_p), mask.data_ptr(),
                                         ctypes.cast(_gates(gparams), ctypes.c_void_p), dweights.data_ptr(),
                                         dfeats.data_ptr() if need_x else None,
                                         ctypes.cast(dgates, ctypes.c_void_p) if need_g else None, ws.data_ptr(),
                                         _nat.stream_ptr(dev))
    _nat.check(rc, "compute_adaptive_weights backward")
    return dfeats, ggrads


@adaptive_weights_bwd.register_fake
def _(mask, feats, gparams, dweights, need_x, need_g):
    B, M = mask.shape
    H = feats[0].size(1)
    return (mask.new_empty(B, M, H) if need_x else mask.new_empty(0),
            [torch.empty_like(p) if need_g else p.new_empty(0) for p in gparams])


def _aw_setup(ctx, inputs, output):
    mask, feats, gparams = inputs
    ctx.M = len(feats)
    ctx.need_x = [bool(f.requires_grad) for f in feats]
    ctx.need_g = any(bool(p.requires_grad) for p in gparams)
    ctx.save_for_backward(mask, *feats, *gparams)


def _aw_backward(ctx, dweights):
    mask, *rest = ctx.saved_tensors
    feats, gparams = rest[:ctx.M], rest[ctx.M:]
    dfeats, gg = torch.ops.mmfusion.adaptive_weights_bwd(mask, list(feats), list(gparams), dweights.contiguous(),
                                                         any(ctx.need_x), ctx.need_g)
    dx = [dfeats[:, m] if n else None for m, n in enumerate(ctx.need_x)]
    return None, dx, (list(gg) if ctx.need_g else None)


adaptive_weights_fwd.register_autograd(_aw_backward, setup_context=_aw_setup)


# ============================================================================ FrameEncoder.attention_pool
@torch.library.custom_op("mmfusion::attention_pool_fwd", mutates_args=(), device_types="cuda")
def attention_pool_fwd(frames: Tensor, weight: Tensor, bias: Tensor, mask: Optional[Tensor]) -> Tuple[Tensor, Tensor]:
    """-> pooled (B, D), frame weights (B, T)."""
    L = _nat.lib()
    B, T, D = frames.shape
    dev = frames.device
    pooled = torch.empty(B, D, dtype=torch.float32, device=dev)
    weights = torch.empty(B, T, dtype=torch.float32, device=dev)
    rc = L.mmf_attention_pool_forward(B, T, D, frames.data_ptr(), weight.data_ptr(), bias.data_ptr(),
                                      _nat.ptr(mask), pooled.data_ptr(), weights.data_ptr(), _nat.stream_ptr(dev))
    _nat.check(rc, "FrameEncoder.attention_pool forward")
    return pooled, weights


@attention_pool_fwd.register_fake
def _(frames, weight, bias, mask):
    B, T, D = frames.shape
    return frames.new_empty(B, D), frames.new_empty(B, T)


@torch.library.custom_op("mmfusion::attention_pool_bwd", mutates_args=(), device_types="cuda")
def attention_pool_bwd(frames: Tensor, weight: Tensor, weights: Tensor, dpooled: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    L = _nat.lib()
    B, T, D = frames.shape
    dev = frames.device
    dx = torch.empty_like(frames)
    dw = torch.empty(D, dtype=torch.float32, device=dev)
    db = torch.empty(1, dtype=torch.float32, device=dev)
    ws = torch.empty(L.mmf_attention_pool_workspace_bytes(B, D), dtype=torch.uint8, device=dev)
    rc = L.mmf_attention_pool_backward(B, T, D, frames.data_ptr(), weight.data_ptr(), weights.data_ptr(),
                                       dpooled.data_ptr(), dx.data_ptr(), dw.data_ptr(), db.data_ptr(),
                                       ws.data_ptr(), _nat.stream_ptr(dev))
    _nat.check(rc, "FrameEncoder.attention_pool backward")
    return dx, dw, db


@attention_pool_bwd.register_fake
def _(frames, weight, weights, dpooled):
    return torch.empty_like(frames), frames.new_empty(frames.size(2)), frames.new_empty(1)


def _ap_setup(ctx, inputs, output):
    frames, weight, bias, mask = inputs
    ctx.wshape, ctx.bshape = weight.shape, bias.shape
    ctx.save_for_backward(frames, weight, output[1])


def _ap_backward(ctx, dpooled, _dweights):
    frames, weight, weights = ctx.saved_tensors
    dx, dw, db = torch.ops.mmfusion.attention_pool_bwd(frames, weight, weights, dpooled.contiguous())
    return dx, dw.view(ctx.wshape), db.view(ctx.bshape), None


attention_pool_fwd.register_autograd(_ap_backward, setup_context=_ap_setup)


# ============================================================================ LateFusion weighting
@torch.library.custom_op("mmfusion::late_weights_fwd", mutates_args=(), device_types="cuda")
def late_weights_fwd(stacked: Tensor, weight_logits: Tensor, mask: Tensor) -> Tuple[Tensor, Tensor]:
    """-> fused (B, C), weights (B, M)."""
    L = _nat.lib()
    B, M, C = stacked.shape
    dev = stacked.device
    fused = torch.empty(B, C, dtype=torch.float32, device=dev)
    weights = torch.empty(B, M, dtype=torch.float32, device=dev)
    rc = L.mmf_late_fusion_forward(B, M, C, stacked.data_ptr(), weight_logits.data_ptr(), mask.data_ptr(),
                                   fused.data_ptr(), weights.data_ptr(), _nat.stream_ptr(dev))
    _nat.check(rc, "LateFusion weighting forward")
    return fused, weights


@late_weights_fwd.register_fake
def _(stacked, weight_logits, mask):
    B, M, C = stacked.shape
    return stacked.new_empty(B, C), stacked.new_empty(B, M)


@torch.library.custom_op("mmfusion::late_weights_bwd", mutates_args=(), device_types="cuda")
def late_weights_bwd(stacked: Tensor, weight_logits: Tensor, mask: Tensor, weights: Tensor,
                     dfused: Tensor) -> Tuple[Tensor, Tensor]:
    L = _nat.lib()
    B, M, C = stacked.shape
    dev = stacked.device
    dstacked = torch.empty_like(stacked)
    dwl = torch.empty(M, dtype=torch.float32, device=dev)
    ws = torch.empty(L.mmf_late_fusion_workspace_bytes(B, M), dtype=torch.uint8, device=dev)
    rc = L.mmf_late_fusion_backward(B, M, C, stacked.data_ptr(), weight_logits.data_ptr(), mask.data_ptr(),
                                    weights.data_ptr(), dfused.data_ptr(), dstacked.data_ptr(), dwl.data_ptr(),
                                    ws.data_ptr(), _nat.stream_ptr(dev))
    _nat.check(rc, "LateFusion weighting backward")
    return dstacked, dwl


@late_weights_bwd.register_fake
def _(stacked, weight_logits, mask, weights, dfused):
    return torch.empty_like(stacked), stacked.new_empty(stacked.size(1))


def _lw_setup(ctx, inputs, output):
    stacked, weight_logits, mask = inputs
    ctx.save_for_backward(stacked, weight_logits, mask, output[1])


def _lw_backward(ctx, dfused, _dweights):
    stacked, weight_logits, mask, weights = ctx.saved_tensors
    ds, dwl = torch.ops.mmfusion.late_weights_bwd(stacked, weight_logits, mask, weights, dfused.contiguous())
    return ds, dwl, None


late_weights_fwd.register_autograd(_lw_backward, setup_context=_lw_setup)


# ============================================================================ LSTM layer (SequenceEncoder)
@torch.library.custom_op("mmfusion::lstm_layer_fwd", mutates_args=(), device_types="cuda")
def lstm_layer_fwd(xproj: List[Tensor], w_hh: List[Tensor]) -> Tuple[List[Tensor], List[Tensor], List[Tensor], Tensor]:
    """One layer of n independent LSTMs: xproj (B, T, 4H) = x W_ih^T + b_ih + b_hh per LSTM ->
    h, c (B, T, H), activated gates (B, T, 4H) per LSTM, and the launch's timeout word."""
    L = _nat.lib()
    n = len(xproj)
    dev = xproj[0].device
    B, T, H4 = xproj[0].shape
    H = H4 // 4
    hs = [torch.empty(B, T, H, dtype=torch.float32, device=dev) for _ in range(n)]
    cs = [torch.empty(B, T, H, dtype=torch.float32, device=dev) for _ in range(n)]
    gates = [torch.empty(B, T, 4 * H, dtype=torch.float32, device=dev) for _ in range(n)]
    sync = torch.empty(n, L.mmf_lstm_sync_bytes(B, H), dtype=torch.uint8, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    rc = L.mmf_lstm_forward(
        n, B, T, H, _nat.ptr_array([t.data_ptr() for t in xproj]), _nat.ptr_array([w.data_ptr() for w in w_hh]),
        _nat.ptr_array([t.data_ptr() for t in hs]), _nat.ptr_array([t.data_ptr() for t in cs]),
        _nat.ptr_array([t.data_ptr() for t in gates]), _nat.ptr_array([sync[i].data_ptr() for i in range(n)]),
        flag.data_ptr(), _nat.stream_ptr(dev))
    _nat.check(rc, "LSTM forward")
    return hs, cs, gates, flag


@lstm_layer_fwd.register_fake
def _(xproj, w_hh):
    B, T, H4 = xproj[0].shape
    H = H4 // 4
    n = len(xproj)
    x0 = xproj[0]
    return ([x0.new_empty(B, T, H) for _ in range(n)], [x0.new_empty(B, T, H) for _ in range(n)],
            [x0.new_empty(B, T, 4 * H) for _ in range(n)], x0.new_empty(1, dtype=torch.int32))


@torch.library.custom_op("mmfusion::lstm_layer_bwd", mutates_args=(), device_types="cuda")
def lstm_layer_bwd(w_hh: List[Tensor], cs: List[Tensor], gates: List[Tensor],
                   dh: List[Tensor]) -> Tuple[List[Tensor], Tensor]:
    """-> d(pre-activation gates) (B, T, 4H) per LSTM (= d xproj) and the timeout word."""
    L = _nat.lib()
    n = len(w_hh)
    dev = cs[0].device
    B, T, H = cs[0].shape
    dgates = [torch.empty(B, T, 4 * H, dtype=torch.float32, device=dev) for _ in range(n)]
    sync = torch.empty(n, L.mmf_lstm_sync_bytes(B, H), dtype=torch.uint8, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    rc = L.mmf_lstm_backward(
        n, B, T, H, _nat.ptr_array([w.data_ptr() for w in w_hh]), _nat.ptr_array([t.data_ptr() for t in cs]),
        _nat.ptr_array([t.data_ptr() for t in gates]),
        _nat.ptr_array([d.data_ptr() if d.numel() else 0 for d in dh]),
        _nat.ptr_array([t.data_ptr() for t in dgates]), _nat.ptr_array([sync[i].data_ptr() for i in range(n)]),
        flag.data_ptr(), _nat.stream_ptr(dev))
    _nat.check(rc, "LSTM backward")
    return dgates, flag


@lstm_layer_bwd.register_fake
def _(w_hh, cs, gates, dh):
    B, T, H = cs[0].shape
    return [cs[0].new_empty(B, T, 4 * H) for _ in w_hh], cs[0].new_empty(1, dtype=torch.int32)


def _lstm_setup(ctx, inputs, output):
    xproj, w_hh = inputs
    hs, cs, gates, _flag = output
    ctx.n = len(xproj)
    ctx.save_for_backward(*w_hh, *hs, *cs, *gates)


def _lstm_backward(ctx, dhs, _dcs, _dgates, _dflag):
    n = ctx.n
    sv = ctx.saved_tensors
    w_hh, hs, cs, gates = (list(sv[k * n:(k + 1) * n]) for k in range(4))
    dh = [hs[i].new_empty(0) if (dhs is None or dhs[i] is None) else dhs[i].contiguous() for i in range(n)]
    dgates, flag = torch.ops.mmfusion.lstm_layer_bwd(w_hh, cs, gates, dh)
    if eager_tensor(flag):
        LSTM_FLAGS.append(flag)
    B, T, H = hs[0].shape
    # dW_hh = sum_t dgates_t^T h_{t-1} (h_{-1} = 0)
    dw_hh = [dgates[i][:, 1:].reshape(-1, 4 * H).t() @ hs[i][:, :-1].reshape(-1, H) for i in range(n)]
    return list(dgates), dw_hh


lstm_layer_fwd.register_autograd(_lstm_backward, setup_context=_lstm_setup)

# timeout words of the eager LSTM launches, drained by encoders.lstm_timed_out (a compiled
# graph keeps only the NaN poisoning of values that never arrived, csrc/lstm.hip)
LSTM_FLAGS: List[Tensor] = []


def eager_tensor(t: Tensor) -> bool:
    """A real tensor of an eager call: not Dynamo tracing, and not one of the fake / functional
    tensors AOTAutograd traces the backward formula with (torch.compiler.is_compiling() is
    False there)."""
    return type(t) is torch.Tensor and not torch.compiler.is_compiling()


# ============================================================================ CrossEntropyLoss(label_smoothing)
def cross_entropy_impl(logits: Tensor, labels: Tensor, label_smoothing: float) -> Tuple[Tensor, Tensor]:
    L = _nat.lib()
    B, C = logits.shape
    dev = logits.device
    loss = torch.empty((), dtype=torch.float32, device=dev)
    dlogits = torch.empty(B, C, dtype=torch.float32, device=dev)
    rc = L.mmf_cross_entropy_ls(B, C, logits.data_ptr(), labels.data_ptr(), float(label_smoothing), 1.0,
                                loss.data_ptr(), dlogits.data_ptr(), _nat.stream_ptr(dev))
    _nat.check(rc, "CrossEntropyLoss(label_smoothing)")
    return loss, dlogits


@torch.library.custom_op("mmfusion::cross_entropy_ls_fwd", mutates_args=(), device_types="cuda")
def cross_entropy_ls_fwd(logits: Tensor, labels: Tensor, label_smoothing: float) -> Tuple[Tensor, Tensor]:
    """nn.CrossEntropyLoss(label_smoothing=eps) with reduction "mean" (src/train.py:185-186,
    310) in one launch of head.hip's cross_entropy_kernel: -> (mean loss, d loss / d logits).
    Rows labelled -100 (torch's default ignore_index) add nothing and get a zero gradient, the
    mean is over the other rows; a label outside [0, C) otherwise (torch raises) makes the loss
    NaN and is never used as an index."""
    return cross_entropy_impl(logits, labels, label_smoothing)


@cross_entropy_ls_fwd.register_fake
def _(logits, labels, label_smoothing):
    return logits.new_empty(()), torch.empty_like(logits)


def _ce_setup(ctx, inputs, output):
    ctx.save_for_backward(output[1])


def _ce_backward(ctx, dloss, _ddlogits):
    (dlogits,) = ctx.saved_tensors
    return dlogits * dloss, None, None


cross_entropy_ls_fwd.register_autograd(_ce_backward, setup_context=_ce_setup)


class CrossEntropyEager(torch.autograd.Function):
    """Eager twin of cross_entropy_ls_fwd (same implementation, autograd.Function dispatch)."""

    @staticmethod
    def forward(ctx, logits, labels, label_smoothing):
        loss, dlogits = cross_entropy_impl(logits, labels, label_smoothing)
        ctx.save_for_backward(dlogits)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        (dlogits,) = ctx.saved_tensors
        return dlogits * dloss, None, None


def cross_entropy(logits: Tensor, labels: Tensor, label_smoothing: float = 0.0, ignore_index: int = -100) -> Tensor:
    """Drop-in for torch.nn.functional.cross_entropy(logits, labels, label_smoothing=...,
    ignore_index=-100) on (B, C) fp32 logits, int64 labels, reduction "mean": the loss and its
    gradient in one HIP launch (torch's composes it from log_softmax, nll_loss and the smoothing
    term, about eight launches forward and backward).  Another ignore_index goes to torch's own
    (the kernel knows -100 only).  A label outside [0, C) that is not ignored gives a NaN loss
    (torch raises; checking on the host would synchronise every step)."""
    if logits.dim() != 2 or logits.dtype != torch.float32 or labels.dtype != torch.int64:
        raise ValueError("cross_entropy: (B, C) float32 logits and int64 labels")
    if ignore_index != -100:
        import torch.nn.functional as F
        return F.cross_entropy(logits, labels, label_smoothing=label_smoothing, ignore_index=ignore_index)
    if eager_tensor(logits):
        ext = torch_ext()
        if ext is not None:
            return ext.cross_entropy(logits.contiguous(), labels.contiguous(), float(label_smoothing))
        return CrossEntropyEager.apply(logits.contiguous(), labels.contiguous(), float(label_smoothing))
    return torch.ops.mmfusion.cross_entropy_ls_fwd(logits.contiguous(), labels.contiguous(), float(label_smoothing))[0]
