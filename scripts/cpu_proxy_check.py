#!/usr/bin/env python3
"""Is the CPU baseline's proxy faithful?  (SURVEY §8d "CPU reference timing")

bench.py's ``cpu_baseline`` times the oracle (oracle/hybrid_cpu.py, a from-scratch torch-CPU
restatement) on the GPU box's host cores, because the reference cannot travel there.  This
container-only script (it imports /root/reference/src) times the REFERENCE itself beside the
oracle on the same inputs, threads and batch -- one training step = forward + CE(label
smoothing 0.05) + backward, train mode (dropout 0.1), fp32 "highest" -- and reports the ratio.
The proxy is accepted when every leg agrees within +-15 %.

Legs (C2: M = 3, D = H = 128, 4 heads, C = 5, B = 256):
  * L = 1 (2-D inputs): the reference's own HybridFusion.forward;
  * L = 128 (sequence mode, the bench workload): the reference's sub-modules composed as in
    SURVEY §8c (tests/golden/gen_golden.py composed_seq_forward);
  at 8 threads (this container) and 4 threads (the reference's own cap, src/train.py:446).

usage: python scripts/cpu_proxy_check.py [--out profiles/r03_cpu_proxy_check.json] [--steps 3]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
REF_SRC = "/root/reference/src"


def timed(fn, steps, min_s=3.0):
    """Mean seconds per call over >= `steps` calls and >= min_s seconds, after one warm-up call."""
    fn()
    n, t0 = 0, time.perf_counter()
    while n < steps or time.perf_counter() - t0 < min_s:
        fn()
        n += 1
    return (time.perf_counter() - t0) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_cpu_proxy_check.json"))
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    torch.set_float32_matmul_precision("highest")
    sys.path.insert(0, REF_SRC)
    import fusion as ref_fusion               # the reference (read-only, imported in place)
    from gen_golden import composed_seq_forward
    from oracle.hybrid_cpu import hybrid_train_step

    M, B, D, H, heads, C = 3, 256, 128, 128, 4, 5
    names = [f"m{i}" for i in range(M)]
    torch.manual_seed(0)
    ref = ref_fusion.HybridFusion({n: D for n in names}, hidden_dim=H, num_classes=C, num_heads=heads,
                                  dropout=0.1).train()
    params = {k: v.detach().clone().requires_grad_(True) for k, v in ref.state_dict().items()}
    g = torch.Generator().manual_seed(1)
    legs = []
    for L in (1, 128):
        shape = (B, D) if L == 1 else (B, L, D)
        x = {n: torch.randn(shape, generator=g) for n in names}
        mask = torch.ones(B, M)
        labels = torch.randint(0, C, (B,), generator=g)
        feats_r = {n: t.clone().requires_grad_(True) for n, t in x.items()}
        feats_o = {n: t.clone().requires_grad_(True) for n, t in x.items()}

        def ref_step():
            ref.zero_grad(set_to_none=True)
            for t in feats_r.values():
                t.grad = None
            logits = ref(feats_r, mask) if L == 1 else composed_seq_forward(ref, feats_r, mask)[0]
            F.cross_entropy(logits, labels, label_smoothing=0.05).backward()

        gen = torch.Generator().manual_seed(5)

        def oracle_step():
            for t in list(params.values()) + list(feats_o.values()):
                t.grad = None
            hybrid_train_step(params, names, feats_o, mask, labels, heads, 0.1, gen)

        for threads in (8, 4):
            torch.set_num_threads(threads)
            t_ref = timed(ref_step, args.steps)
            t_orc = timed(oracle_step, args.steps)
            leg = {"L": L, "B": B, "threads": threads, "reference_ms": round(t_ref * 1e3, 2),
                   "oracle_ms": round(t_orc * 1e3, 2), "oracle_over_reference": round(t_orc / t_ref, 4),
                   "reference_samples_per_s": round(B / t_ref, 2), "oracle_samples_per_s": round(B / t_orc, 2)}
            leg["within_15pct"] = abs(leg["oracle_over_reference"] - 1.0) <= 0.15
            print(json.dumps(leg), flush=True)
            legs.append(leg)
    out = {"what": "reference HybridFusion (L=1) / composed reference sub-modules (L=128) vs oracle/hybrid_cpu.py, "
                   "one fwd+CE+bwd train step, fp32, same inputs",
           "host": f"{os.cpu_count()} CPUs (this container)", "torch": torch.__version__, "steps": args.steps,
           "legs": legs, "all_within_15pct": all(x["within_15pct"] for x in legs)}
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({"all_within_15pct": out["all_within_15pct"]}))


if __name__ == "__main__":
    main()
