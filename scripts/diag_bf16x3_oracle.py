"""Diagnostic (CPU): how far matmul precision "high" (bf16x3) moves the REFERENCE algorithm.

Runs one TRAIN_CASES case through the oracle three ways -- float64 (the truth), float32, and
float32 with every matmul (forward and backward) on bf16x3-split operands
(tests/_util.bf16x3_matmul_mode) -- and prints max|x - x64| / max|x64| per tensor for the
fp32 and the bf16x3 runs, plus the worst samples of each input gradient.
usage: python scripts/diag_bf16x3_oracle.py <case> [p]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
from _philox import mask_provider  # noqa: E402
from _util import bf16x3_matmul_mode  # noqa: E402
from cases import hybrid_inputs, hybrid_state  # noqa: E402
from oracle.hybrid_cpu import hybrid_forward  # noqa: E402
from test_gpu_train_mode import OFFSET, SEED, TRAIN_CASES  # noqa: E402

case = next(c for c in TRAIN_CASES if c.name == sys.argv[1])
P = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
torch.set_num_threads(8)


def run(dtype, emu=False):
    sd = hybrid_state(case.names, case.dims, case.hidden, case.classes, case.seed)
    params = {k: torch.from_numpy(v).to(dtype).requires_grad_(True) for k, v in sd.items()}
    feats_np, mask_np, grad_np = hybrid_inputs(case)
    xs = {m: torch.from_numpy(v).to(dtype).requires_grad_(True) for m, v in feats_np.items()}
    gen = mask_provider(SEED, OFFSET, P) if P > 0 else None

    def go():
        ref, _ = hybrid_forward(params, case.names, xs, torch.from_numpy(mask_np).to(dtype), case.heads,
                                p=P, train=P > 0, gen=gen)
        (ref * torch.from_numpy(grad_np).to(dtype)).sum().backward()
        return ref

    if emu:
        with bf16x3_matmul_mode():
            ref = go()
    else:
        ref = go()
    out = {"logits": ref.detach()}
    for m in case.names:
        out[f"dx/{m}"] = xs[m].grad.detach()
    for k, v in params.items():
        out[k] = v.grad.detach() if v.grad is not None else torch.zeros_like(v)
    return out


t64 = run(torch.float64)
f32 = run(torch.float32)
emu = run(torch.float32, emu=True)
print(f"case {case.name} p={P}")
print(f"{'tensor':50s} {'fp32':>10s} {'bf16x3':>10s}")
for k, v in t64.items():
    s = max(float(v.abs().max()), 1e-30)
    e32 = float((f32[k].double() - v).abs().max()) / s
    e3 = float((emu[k].double() - v).abs().max()) / s
    print(f"{k:50s} {e32:10.3e} {e3:10.3e}")
for m in case.names:
    v = t64[f"dx/{m}"]
    d = (emu[f"dx/{m}"].double() - v).abs().flatten(1).max(1).values / float(v.abs().max())
    top = torch.topk(d, 4)
    print(f"worst samples dx/{m} (bf16x3):", [(int(i), f"{float(x):.2e}") for x, i in zip(top.values, top.indices)])
