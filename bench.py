#!/usr/bin/env python3
"""HybridFusion fwd+bwd training-step throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], "C2"): synthetic 3-modality HybridFusion,
B=256 samples per GPU, T=L=128 tokens per modality, d_model=D=H=128, 4 heads,
5 classes, fp32, train mode (dropout 0.1).  Inputs are the (B, L, D) encoder
outputs of each modality (sequence mode), resident in HBM.
One step = HybridFusion forward -> CrossEntropy(label_smoothing=0.05) ->
backward (all parameter grads + input grads) -> [RCCL all-reduce of the flat
gradient when N > 1] -> AdamW.  Weak scaling: every rank runs B=256.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c2_l1]
N > 1 is launched by torch.distributed.run (one process per GPU, RCCL).
Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "multimodal-sensor-fusion-with-attention-rajeevatla_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)

METRIC = "HybridFusion fwd+bwd samples/sec at 1/2/4/8 MI355X; CPU-ref parity"
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak

WORKLOADS = {
    # name: (M, B per GPU, L (0 => 2-D reference semantics), D, H, heads, C)
    "c2": (3, 256, 128, 128, 128, 4, 5),
    "c2_l1": (3, 256, 0, 128, 128, 4, 5),
}


def pooled_plan(L, heads):
    """csrc/hybrid.hip use_pool(): key lengths <= 128 and <= 8 heads."""
    return max(L, 1) <= 128 and heads <= 8


def stage_flops(M, B, L, D, H, heads, C):
    """Algorithmic FLOPs of each launch group (no recompute counted)."""
    Le = max(L, 1)
    P = M * (M - 1)
    rows = B * Le
    if pooled_plan(L, heads):
        # pooled-output plan: no V / O / attended (B, L, H) tensors
        return {
            "fwd.proj_gemm": 2 * rows * D * H * M,
            "fwd.qkv_gemm": 2 * 2 * rows * H * H * P,
            "fwd.attn": 2 * B * Le * Le * H * P,             # S = Q K^T (+ softmax, column mean)
            "fwd.pool_u": 2 * B * heads * Le * H * P,         # U_h = pbar_h P_k
            "fwd.vbar_gemm": 2 * B * H * H * P,
            "fwd.out_gemm": 2 * B * H * H * P,
            "fwd.cls1_gemm": 2 * B * H * H,
            "fwd.cls2_gemm": 2 * B * H * C,
            "fwd.tail": 2 * 2 * B * H * H * P + 2 * B * H * H + 2 * B * H * C,   # fused V/O/head/classifier
            "bwd.tail": 2 * B * C * H + 2 * B * H * H + 2 * 2 * B * H * H * P,
            "bwd.cls_dz1_gemm": 2 * B * C * H,
            "bwd.cls_dfused_gemm": 2 * B * H * H,
            "bwd.out_dO_gemm": 2 * B * H * H * P,
            "bwd.du_gemm": 2 * B * H * H * P,
            "bwd.pool_dpbar": 2 * B * heads * Le * H * P,
            "bwd.attn_dq": 2 * B * Le * Le * H * P,          # dQ = dS K (S recompute not counted)
            "bwd.attn_dk": 2 * B * Le * Le * H * P,          # dK = dS^T Q
            "bwd.pool_e": 2 * B * heads * Le * H * P,
            "bwd.dZ_gemm": 2 * rows * H * H * 2 * P,         # dQ W_q + dK W_k into every modality
            "bwd.dx_gemm": 2 * rows * H * D * M,
            "bwd.wgrad_gemm": 2 * rows * H * D * M + 2 * 2 * rows * H * H * P + 2 * 2 * B * H * H * P
                              + 2 * B * H * (H + C),
        }
    f = {
        "fwd.proj_gemm": 2 * rows * D * H * M,
        "fwd.qkv_gemm": 3 * 2 * rows * H * H * P,
        "fwd.attn": 4 * B * Le * Le * H * P,
        "fwd.out_gemm": 2 * rows * H * H * P,
        "fwd.cls1_gemm": 2 * B * H * H,
        "fwd.cls2_gemm": 2 * B * H * C,
        "bwd.cls_dz1_gemm": 2 * B * C * H,
        "bwd.cls_dfused_gemm": 2 * B * H * H,
        "bwd.out_dO_gemm": 2 * rows * H * H * P,
        "bwd.attn_dkv": 6 * B * Le * Le * H * P,     # dP, dV, dK
        "bwd.attn_dq": 2 * B * Le * Le * H * P,      # dQ
        "bwd.dZ_gemm": 3 * 2 * rows * H * H * P,     # dP_m from dQ, dK, dV
        "bwd.dx_gemm": 2 * rows * H * D * M,
        # dW for proj (M), q/k/v/out (4P), classifier (2)
        "bwd.wgrad_gemm": 2 * rows * H * D * M + 4 * 2 * rows * H * H * P + 2 * B * H * (H + C),
    }
    return f


def total_step_flops(M, B, L, D, H, heads, C):
    """SURVEY §8d formula: 3 x forward (projections + P*(8BLH^2 + 4BL^2H) + head)."""
    Le = max(L, 1)
    P = M * (M - 1)
    fwd = 2 * B * Le * D * H * M
    if L > 0:
        fwd += P * (8 * B * Le * H * H + 4 * B * Le * Le * H)
    else:
        fwd += P * 4 * B * H * H      # reference semantics: Q/K dead at L=1
    fwd += 2 * B * H * H + 2 * B * H * C + 4 * M * B * H + B * Le * H * M
    return 3 * fwd


def make_inputs(M, B, L, D, C, seed, device):
    g = torch.Generator().manual_seed(seed)
    shape = (B, L, D) if L > 0 else (B, D)
    feats = [torch.randn(shape, generator=g) for _ in range(M)]
    mask = torch.ones(B, M)
    labels = torch.randint(0, C, (B,), generator=g)
    return [f.to(device) for f in feats], mask.to(device), labels.to(device)


def cpu_baseline(M, L, D, H, heads, C, budget_s=15.0, max_steps=20):
    """Time the oracle (torch-CPU restatement, oracle/hybrid_cpu.py) on a bounded sample."""
    from oracle.hybrid_cpu import hybrid_train_step
    from fusion import HybridFusion
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    torch.set_num_threads(threads)
    bs = 16 if L > 0 else 256
    torch.manual_seed(0)
    names = [f"m{i}" for i in range(M)]
    model = HybridFusion({n: D for n in names}, hidden_dim=H, num_classes=C, num_heads=heads, dropout=0.1)
    params = {k: v.detach().clone().requires_grad_(True) for k, v in model.state_dict().items()}
    feats_l, mask, labels = make_inputs(M, bs, L, D, C, 1234, "cpu")
    feats = {n: f.requires_grad_(True) for n, f in zip(names, feats_l)}
    gen = torch.Generator().manual_seed(5)
    hybrid_train_step(params, names, feats, mask, labels, heads, 0.1, gen)   # warm-up
    n, t0 = 0, time.perf_counter()
    while n < max_steps and (time.perf_counter() - t0) < budget_s:
        for p in list(params.values()) + list(feats.values()):
            p.grad = None
        hybrid_train_step(params, names, feats, mask, labels, heads, 0.1, gen)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(bs * n / dt, 2), "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"{n} oracle steps of B={bs} (same per-sample work: M={M}, L={max(L, 1)}, "
                      f"D=H={H}, h={heads}, fwd+CE+bwd, fp32, torch {torch.__version__} CPU), {dt:.1f}s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--skip-cpu", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=5)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
        pg = dist.group.WORLD

    import mmf_native
    from fusion import HybridFusion
    from train_step import HybridTrainStep

    M, B, L, D, H, heads, C = WORKLOADS[args.workload]
    torch.manual_seed(0)                      # identical initial weights on every rank
    names = [f"m{i}" for i in range(M)]
    model = HybridFusion({n: D for n in names}, hidden_dim=H, num_classes=C, num_heads=heads,
                         dropout=0.1).to(dev)
    model._rng_state[0] ^= rank * 0x9E3779B1  # distinct dropout streams per rank
    feats, mask, labels = make_inputs(M, B, L, D, C, 42 + rank, dev)
    trainer = HybridTrainStep(model, feats, mask, labels, process_group=pg)

    # kernel-level timing (eager, hipEvents around each launch group on the launch stream)
    trainer.forward_backward()
    torch.cuda.synchronize(dev)
    mmf_native.profile_begin()
    for _ in range(args.profile_steps):
        trainer.forward_backward()
    stages = mmf_native.profile_end()
    per_stage = {}
    for name, ms in stages:
        t, n = per_stage.get(name, (0.0, 0))
        per_stage[name] = (t + ms, n + 1)
    avg_ms = {k: t / n for k, (t, n) in per_stage.items()}

    if not args.no_graph:
        trainer.capture()
    for _ in range(args.warmup):
        trainer.step()
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        trainer.step()
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    dt_t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(dt_t, op=torch.distributed.ReduceOp.MAX)
    dt = float(dt_t.item())
    ms_per_step = dt / args.steps * 1e3
    value = world * B * args.steps / dt
    loss = float(trainer.loss.item())

    if rank == 0:
        fl = stage_flops(M, B, L, D, H, heads, C)
        dom = max(avg_ms, key=lambda k: avg_ms[k])
        dom_flops = fl.get(dom, 0)
        achieved = dom_flops / (avg_ms[dom] * 1e-3) / 1e12 if dom_flops else None
        roofline = {
            "bound": "mfma", "kernel": dom, "achieved": round(achieved, 2) if achieved else None,
            "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4) if achieved else None,
            "traffic": None, "avg_launch_ms": round(avg_ms[dom], 4),
            "algorithmic_gflop_per_launch": round(dom_flops / 1e9, 3),
        }
        step_fl = total_step_flops(M, B, L, D, H, heads, C)
        cpu = None
        if world == 1 and not args.skip_cpu:
            cpu = cpu_baseline(M, L, D, H, heads, C)
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "samples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (N(0,1) encoder outputs, random-init weights, seeded)",
            "config": {"workload": f"{args.workload}: HybridFusion M={M} B={B}/gpu L={L or 1}"
                                   f"{'' if L else ' (2-D reference semantics)'} D=H={H} heads={heads} "
                                   f"C={C} dropout=0.1 train, fwd+CE(ls=0.05)+bwd+AdamW",
                       "global_batch": B * world, "seq_len": L or 1, "parallelism": f"dp{world}",
                       "graph": not args.no_graph},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "step_tflops_algorithmic": round(step_fl / (ms_per_step * 1e-3) / 1e12, 3),
            "step_gflop_algorithmic": round(step_fl / 1e9, 2),
            "stage_ms": {k: round(v, 4) for k, v in sorted(avg_ms.items(), key=lambda kv: -kv[1])},
            "loss": round(loss, 5),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
