"""Shared test helpers: fixture loading and oracle evaluation (test infra)."""
from __future__ import annotations

from pathlib import Path
from typing import Dict

import numpy as np
import torch

from cases import (CMACase, HybridCase, cma_inputs, cma_state, hybrid_inputs,
                   hybrid_state, pair_names)

GOLDEN = Path(__file__).resolve().parent / "golden"


def load_fixture(name: str) -> Dict[str, np.ndarray]:
    with np.load(GOLDEN / f"{name}.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _bf16(x: torch.Tensor) -> torch.Tensor:
    return x.to(torch.bfloat16).to(torch.float32)


class _Bf16MatMul(torch.autograd.Function):
    """matmul with bf16-rounded operands and fp32 accumulation, forward AND backward:
    what torch.set_float32_matmul_precision("medium") permits for every fp32
    matmul (config/base.yaml:80).  Used to size the error a bf16 path must show."""

    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return torch.matmul(_bf16(a), _bf16(b))

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        ga = torch.matmul(_bf16(g), _bf16(b).transpose(-1, -2))
        gb = torch.matmul(_bf16(a).transpose(-1, -2), _bf16(g))
        while ga.dim() > a.dim():
            ga = ga.sum(0)
        while gb.dim() > b.dim():
            gb = gb.sum(0)
        return ga, gb


class bf16_matmul_mode(torch.overrides.TorchFunctionMode):
    """Routes every Tensor.matmul / torch.matmul of the oracle through _Bf16MatMul."""

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func in (torch.Tensor.matmul, torch.matmul) and not kwargs:
            with torch._C.DisableTorchFunction():
                return _Bf16MatMul.apply(*args)
        return func(*args, **kwargs)


def _split3(x: torch.Tensor):
    hi = _bf16(x)
    return hi, _bf16(x - hi)


class _Bf16x3MatMul(torch.autograd.Function):
    """matmul as matmul precision "high" computes it on the device (csrc/mmf_device.h, PR = 2):
    each fp32 operand split into hi = bf16(x) and lo = bf16(x - hi), the three products
    lo_a hi_b + hi_a lo_b + hi_a hi_b accumulated in fp32, lo_a lo_b dropped -- forward AND
    backward (every dS / dP / weight-gradient contraction takes the same split)."""

    @staticmethod
    def _mm(a, b):
        ah, al = _split3(a)
        bh, bl = _split3(b)
        return torch.matmul(al, bh) + torch.matmul(ah, bl) + torch.matmul(ah, bh)

    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return _Bf16x3MatMul._mm(a, b)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        ga = _Bf16x3MatMul._mm(g, b.transpose(-1, -2))
        gb = _Bf16x3MatMul._mm(a.transpose(-1, -2), g)
        while ga.dim() > a.dim():
            ga = ga.sum(0)
        while gb.dim() > b.dim():
            gb = gb.sum(0)
        return ga, gb


class bf16x3_matmul_mode(torch.overrides.TorchFunctionMode):
    """Routes every Tensor.matmul / torch.matmul of the oracle through _Bf16x3MatMul."""

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func in (torch.Tensor.matmul, torch.matmul) and not kwargs:
            with torch._C.DisableTorchFunction():
                return _Bf16x3MatMul.apply(*args)
        return func(*args, **kwargs)


def oracle_hybrid(case: HybridCase, dtype=torch.float32, bf16_matmul: bool = False):
    """Run the CPU oracle on the case; returns (outputs dict, param grads, input grads).
    bf16_matmul: every matmul with bf16 operands (bf16_matmul_mode)."""
    if bf16_matmul:
        with bf16_matmul_mode():
            return oracle_hybrid(case, dtype)
    from oracle.hybrid_cpu import hybrid_forward
    sd = hybrid_state(case.names, case.dims, case.hidden, case.classes, case.seed, case.deleted)
    params = {k: torch.from_numpy(v).to(dtype).requires_grad_(True) for k, v in sd.items()}
    feats_np, mask_np, grad_np = hybrid_inputs(case)
    feats = {m: torch.from_numpy(v).to(dtype).requires_grad_(True) for m, v in feats_np.items()}
    logits, info = hybrid_forward(params, case.names, feats, torch.from_numpy(mask_np).to(dtype),
                                  case.heads)
    (logits * torch.from_numpy(grad_np).to(dtype)).sum().backward()
    out = {"logits": logits.detach(), "fusion_weights": info["fusion_weights"].detach(),
           "pooled": info["pooled"].detach()}
    for k, v in info["attention_maps"].items():
        out[f"attn/{k}"] = v.detach()
    grads = {k: (p.grad if p.grad is not None else torch.zeros_like(p)).detach()
             for k, p in params.items()}
    dx = {m: t.grad.detach() for m, t in feats.items()}
    return out, grads, dx


def oracle_cma(case: CMACase, dtype=torch.float32, bf16_matmul: bool = False):
    if bf16_matmul:
        with bf16_matmul_mode():
            return oracle_cma(case, dtype)
    from oracle.hybrid_cpu import cma_forward
    sd = cma_state(case.query_dim, case.key_dim, case.hidden, case.seed)
    params = {k: torch.from_numpy(v).to(dtype).requires_grad_(True) for k, v in sd.items()}
    q, k, v, mask, grad = cma_inputs(case)
    qt, kt, vt = (torch.from_numpy(a).to(dtype).requires_grad_(True) for a in (q, k, v))
    mt = torch.from_numpy(mask).to(dtype) if mask is not None else None
    att, w = cma_forward(params, "", qt, kt, vt, case.heads, mask=mt)
    (att * torch.from_numpy(grad).to(dtype)).sum().backward()
    out = {"attended": att.detach(), "weights": w.detach(), "dquery": qt.grad, "dkey": kt.grad,
           "dvalue": vt.grad}
    for name, p in params.items():
        out[f"grad/{name}"] = p.grad
    return out


def rel_err(got, ref) -> float:
    """max|got-ref| / max(max|ref|, 1e-6)  (SURVEY §8d parity metric)."""
    got = torch.as_tensor(np.asarray(got) if not torch.is_tensor(got) else got).double().cpu()
    ref = torch.as_tensor(np.asarray(ref) if not torch.is_tensor(ref) else ref).double().cpu()
    assert got.shape == ref.shape, (tuple(got.shape), tuple(ref.shape))
    if ref.numel() == 0:
        return 0.0
    return float((got - ref).abs().max() / max(float(ref.abs().max()), 1e-6))


def diff_report(got, ref, rtol: float, atol: float = 0.0) -> str:
    """For an assertion message: the largest |got - ref|, where it is, the two values there and
    the bound close() applies."""
    got = torch.as_tensor(got).double().cpu()
    ref = torch.as_tensor(ref).double().cpu()
    if got.shape != ref.shape or ref.numel() == 0:
        return f"shapes {tuple(got.shape)} vs {tuple(ref.shape)}"
    d = (got - ref).abs()
    i = int(d.argmax())
    idx = np.unravel_index(i, tuple(ref.shape))
    bound = rtol * float(ref.abs().max()) + atol
    nbad = int((d > bound).sum())
    return (f"max|diff| {float(d.flatten()[i]):.3e} at {tuple(int(v) for v in idx)} (got "
            f"{float(got.flatten()[i]):.6e}, ref {float(ref.flatten()[i]):.6e}), bound {bound:.3e}, "
            f"{nbad} of {ref.numel()} elements over")


def device_relu_gates(taps: dict, weights: dict, dev_acts: dict, rel: float = 1e-5):
    """The device's ReLU'(z) decisions for the pre-activations within rounding of zero, for
    hybrid_forward(relu_gate=...) (the ReLU kink).

    taps: an oracle pass's taps (z/<layer>, in/<layer>); weights: layer -> its weight (H_out,
    H_in); dev_acts: layer -> the device's activation after ReLU and dropout (the values its
    backward takes ReLU' from, as value > 0; HybridTrainStep.saved_activation).  Where
    |z| <= rel * (|x| @ |W|^T) two fp32 summation orders may disagree on the sign of z; there the
    oracle is given the device's decision, everywhere else it keeps its own.  Asserted on the way:
    outside that band every element the device passed (value > 0) has z > 0 in the oracle.
    Returns ({layer: (sel, pos)}, {layer: number of elements in the band})."""
    gates, counts = {}, {}
    for layer, a_dev in dev_acts.items():
        w = weights[layer].detach().double()
        z = taps[f"z/{layer}"].double()
        x = taps[f"in/{layer}"].double().reshape(-1, w.shape[1])
        scale = (x.abs() @ w.abs().t()).reshape(z.shape)
        sel = z.abs() <= rel * scale
        pos = a_dev.detach().cpu().reshape(z.shape) > 0
        bad = pos & ~sel & ~(z > 0)
        assert not bool(bad.any()), (layer, int(bad.sum()), "device passed a z the oracle puts clearly <= 0")
        gates[layer] = (sel, pos)
        counts[layer] = int(sel.sum())
    return gates, counts


def close(got, ref, rtol: float, atol: float = 0.0) -> bool:
    """max|got-ref| <= rtol*max|ref| + atol.  atol only matters for tensors whose
    reference is mathematically zero (e.g. key_proj.bias grads: softmax is
    shift-invariant) and holds pure rounding noise."""
    got = torch.as_tensor(np.asarray(got) if not torch.is_tensor(got) else got).double().cpu()
    ref = torch.as_tensor(np.asarray(ref) if not torch.is_tensor(ref) else ref).double().cpu()
    assert got.shape == ref.shape, (tuple(got.shape), tuple(ref.shape))
    if ref.numel() == 0:
        return True
    return float((got - ref).abs().max()) <= rtol * float(ref.abs().max()) + atol
