#!/usr/bin/env python3
"""HybridFusion fwd+bwd training-step throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], "C2"): synthetic 3-modality HybridFusion,
B=256 samples per GPU, T=L=128 tokens per modality, d_model=D=H=128, 4 heads,
5 classes, fp32, train mode (dropout 0.1).  Inputs are the (B, L, D) encoder
outputs of each modality (sequence mode), resident in HBM.
One step = HybridFusion forward -> CrossEntropy(label_smoothing=0.05) ->
backward (all parameter grads + input grads) -> [RCCL all-reduce of the flat
gradient when N > 1] -> global-norm gradient clipping (1.0) -> AdamW
(lr 1e-3, weight decay 1e-4: config/base.yaml:69-74).  Weak scaling: every rank runs B=256.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c2_l1|c4|c5]
                       [--scaling weak|strong] [--path step|module] [--precision highest|high|medium]
N > 1: one process per GPU over RCCL.  Under torch.distributed.run (WORLD_SIZE set) the
ranks join directly; a plain `python bench.py --gpus N` starts
`python -m torch.distributed.run --nproc-per-node N ... bench.py ...` as a CHILD process
before this process touches the GPU, and exits with its return code.
--scaling weak (default): every rank runs the workload's per-GPU batch (C2: B = 256 per GPU).
--scaling strong: the workload's global batch (C2: 256, C5: 1024) is split over the ranks
(128 / 64 / 32 per GPU at 2 / 4 / 8), each rank running its shard of the same
global batch.
--path step (default): the fused training step (train_step.HybridTrainStep: flat buffers,
one hipGraph per step).  --path module: what src/train.py calls -- the nn.Module forward,
torch CrossEntropyLoss, autograd backward, eager, no graph -- timed the same way (diagnostic:
the gap to the captured step).  --path compiled: the same under the reference trainer's
torch.compile(mode="reduce-overhead", fullgraph=True).
Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import re
import os
import socket
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "multimodal-sensor-fusion-with-attention-rajeevatla_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)

METRIC = "HybridFusion fwd+bwd samples/sec at 1/2/4/8 MI355X; CPU-ref parity"
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
BF16_MFMA_PEAK_TFLOPS = 16 * FP32_MFMA_PEAK_TFLOPS   # ~2.5 PF dense: v_mfma_f32_32x32x16_bf16 (16x the f32 rate)
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E ~8 TB/s

# Per-GPU workloads (BASELINE.json configs; the headline is configs[1] = "c2").
#   L: per-modality sequence lengths (0 => 2-D (B, D) inputs, reference semantics)
#   keep: per-(sample, modality) keep probability of the modality mask (>= 1 kept
#         per row) plus 1 % all-masked rows when < 1
#   B: per-GPU batch under weak scaling; GB: the global batch strong scaling splits
WORKLOADS = {
    "c2": dict(M=3, B=256, GB=256, L=[128] * 3, D=128, H=128, heads=4, C=5, keep=1.0),
    "c2_l1": dict(M=3, B=256, GB=256, L=[0] * 3, D=128, H=128, heads=4, C=5, keep=1.0),
    # C4 shape: video (30 frame embeddings) + IMU (50 steps), Lq != Lk, H = 256, 11 classes
    "c4": dict(M=2, B=256, GB=256, L=[30, 50], D=256, H=256, heads=4, C=11, keep=1.0),
    # C5: 6 modalities, global B = 1024 over 8 GPUs, T = 512, d_model = 256, missing-modality masks
    "c5": dict(M=6, B=128, GB=1024, L=[512] * 6, D=256, H=256, heads=4, C=5, keep=0.9),
}


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_command(gpus: int, argv, port: int, script: str = None):
    """The child command a plain `bench.py --gpus N` (N > 1) runs: torch.distributed.run with
    one process per GPU on this node, rendezvous on 127.0.0.1, the same bench arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", script or os.path.abspath(__file__)] + list(argv)


def rank_batch(w, scaling: str, world: int) -> int:
    """Per-rank batch: the per-GPU batch (weak) or the rank's share of the global batch (strong)."""
    if scaling == "weak":
        return w["B"]
    if w["GB"] % world:
        raise ValueError(f"strong scaling: global batch {w['GB']} is not divisible by {world} ranks")
    return w["GB"] // world


def total_step_flops(w):
    """SURVEY §8d formula: 3 x forward (projections + per pair Q,K,V,out + QK^T + AV + head)."""
    B, D, H, C, M = w["B"], w["D"], w["H"], w["C"], w["M"]
    Ls = w["L"]
    fwd = sum(2 * B * max(l, 1) * D * H for l in Ls)
    for q in range(M):
        for k in range(M):
            if q == k:
                continue
            lq, lk = Ls[q], Ls[k]
            if lq == 0 and lk == 0:
                fwd += 4 * B * H * H          # reference semantics: Q/K dead at L=1
            else:
                lq, lk = max(lq, 1), max(lk, 1)
                fwd += 4 * B * lq * H * H + 4 * B * lk * H * H + 4 * B * lq * lk * H
    fwd += 2 * B * H * H + 2 * B * H * C + 4 * M * B * H + sum(B * max(l, 1) * H for l in Ls)
    return 3 * fwd


def kernel_precision(kname):
    """The int matmul-precision template argument of a library MFMA kernel's profiler name
    (0 fp32, 1 bf16 "medium", 2 bf16x3 "high"): the last integer argument, optionally
    followed by a trailing bool (e.g. "attn_poolL_lse_kernel<64, 1, true>",
    "gemm_lds_kernel<0, 1, 16, 3, 2>", "gemm_wsr_kernel<1>"); the bf16-only kernels are named
    "..._bf16<...>".  Kernels without one (the generic GEMM, the tail / head kernels) run fp32."""
    if kname.startswith("gemm_generic"):
        return 0
    if "_bf16<" in kname or "_b16_kernel" in kname:   # the bf16-only kernels (attn_poolL_*_fused_bf16<DROP>,
        return 1                                       # gemm_wsr_b16_kernel<NS>)
    if kname.startswith("gemm_lds_kernel<") and kname.count(",") in (5, 6):
        return 1                   # the bf16-operand forms: <A, B, 32, 3, 1, B16 form 1 | 2 | 3[, WIDE]>
    m = re.search(r"[<, ]([012])(?:, (?:true|false)){0,3}>$", kname)
    return int(m.group(1)) if m else 0


def mfma_peak(kname):
    """Dense MFMA peak for a kernel's algorithmic FLOPs: fp32 MFMA, bf16 MFMA, or for the
    bf16x3 form one third of the bf16 peak (three bf16 MFMAs per fp32-equivalent product)."""
    return {0: FP32_MFMA_PEAK_TFLOPS, 1: BF16_MFMA_PEAK_TFLOPS, 2: BF16_MFMA_PEAK_TFLOPS / 3.0}[kernel_precision(kname)]


def kernel_table(launches, steps):
    """Per kernel name: time per step, average launch duration and the roofline
    of its launches (algorithmic FLOPs / bytes from the library's per-launch
    records over the measured durations), sorted by time per step."""
    acc = {}
    for _stage, kname, ms, flops, nbytes in launches:
        a = acc.setdefault(kname, [0.0, 0, 0.0, 0.0])
        a[0] += ms
        a[1] += 1
        a[2] += flops
        a[3] += nbytes
    out = {}
    for kname, (ms, n, flops, nbytes) in sorted(acc.items(), key=lambda kv: -kv[1][0]):
        sec = ms * 1e-3
        fpeak = mfma_peak(kname)
        t_f = flops / (fpeak * 1e12)
        t_b = nbytes / (HBM_PEAK_GBS * 1e9)
        if t_f >= t_b:
            bound, ach, peak, unit = "mfma", flops / sec / 1e12 if sec else 0.0, fpeak, "TFLOP/s"
        else:
            bound, ach, peak, unit = "hbm", nbytes / sec / 1e9 if sec else 0.0, HBM_PEAK_GBS, "GB/s"
        # the other roof's fraction beside it: a kernel at a small fraction of both (issue- or
        # latency-bound, e.g. the C5 long-key backward) shows that here, not only its nominal bound
        mfma_frac = (flops / sec / 1e12) / fpeak if sec else 0.0
        hbm_frac = (nbytes / sec / 1e9) / HBM_PEAK_GBS if sec else 0.0
        out[kname] = {
            "ms_per_step": round(ms / steps, 4), "launches_per_step": round(n / steps, 2),
            "avg_launch_ms": round(ms / n, 5), "bound": bound, "achieved": round(ach, 2), "peak": peak,
            "unit": unit, "frac": round(ach / peak, 4),
            "mfma_frac": round(mfma_frac, 4), "hbm_frac": round(hbm_frac, 4),
            "flops_per_launch": flops / n, "bytes_per_launch": nbytes / n,
        }
    return out


def pmc_traffic(workload="c2", precision="highest"):
    """HBM bytes per launch by kernel name from the committed PMC summary of THIS workload
    and precision (profiles/pmc_traffic.py output: FETCH_SIZE x2 (gfx950 correction) +
    WRITE_SIZE, KiB -> bytes, averaged over the dispatches of an eager run of this bench):
    profiles/pmc_traffic.json for the C2 headline, profiles/pmc_traffic_<workload>_<precision>.json
    otherwise; none (traffic null) when no pass of that workload is committed -- the kernel
    names repeat across workloads, their bytes do not."""
    name = "pmc_traffic.json" if (workload, precision) == ("c2", "highest") else \
        f"pmc_traffic_{workload}_{precision}.json"
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return {}, None
    with open(path) as f:
        d = json.load(f)
    return d.get("kernels", {}), d.get("source")


def dominant_roofline(kernels, workload="c2", precision="highest"):
    """Roofline of the kernel with the most time per step."""
    kname = next(iter(kernels))
    k = kernels[kname]
    traffic, src = pmc_traffic(workload, precision)
    t = traffic.get(kname, {}).get("hbm_bytes_per_launch")
    per_launch = k["flops_per_launch"] if k["bound"] == "mfma" else k["bytes_per_launch"]
    return {
        "bound": k["bound"], "achieved": k["achieved"], "peak": k["peak"], "unit": k["unit"],
        "frac": k["frac"], "mfma_frac": k["mfma_frac"], "hbm_frac": k["hbm_frac"],
        "traffic": round(t) if t is not None else None,
        "kernel": kname, "avg_launch_ms": k["avg_launch_ms"], "launches_per_step": k["launches_per_step"],
        "algorithmic_per_launch": round(per_launch),
        "algorithmic_bytes_per_launch": round(k["bytes_per_launch"]),
        "traffic_source": src if t is not None else None,
    }


def make_inputs(w, B, seed, device):
    g = torch.Generator().manual_seed(seed)
    feats = [torch.randn((B, l, w["D"]) if l > 0 else (B, w["D"]), generator=g) for l in w["L"]]
    mask = torch.ones(B, w["M"])
    if w["keep"] < 1.0:
        mask = (torch.rand(B, w["M"], generator=g) < w["keep"]).float()
        first = torch.randint(0, w["M"], (B,), generator=g)
        mask[torch.arange(B), first] = 1.0            # >= 1 modality kept per row ...
        mask[torch.randperm(B, generator=g)[: max(1, B // 100)]] = 0.0   # ... except 1 % all-masked rows
    labels = torch.randint(0, w["C"], (B,), generator=g)
    return [f.to(device) for f in feats], mask.to(device), labels.to(device)


def _cpu_leg(w, bs, threads, budget_s, max_steps):
    """Oracle train steps (fwd + CE + bwd, dropout 0.1) at `threads` threads for ~budget_s."""
    from oracle.hybrid_cpu import hybrid_train_step
    from fusion import HybridFusion
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    names = [f"m{i}" for i in range(w["M"])]
    model = HybridFusion({n: w["D"] for n in names}, hidden_dim=w["H"], num_classes=w["C"], num_heads=w["heads"],
                         dropout=0.1)
    params = {k: v.detach().clone().requires_grad_(True) for k, v in model.state_dict().items()}
    feats_l, mask, labels = make_inputs(w, bs, 1234, "cpu")
    feats = {n: f.requires_grad_(True) for n, f in zip(names, feats_l)}
    gen = torch.Generator().manual_seed(5)
    hybrid_train_step(params, names, feats, mask, labels, w["heads"], 0.1, gen)   # warm-up
    n, t0 = 0, time.perf_counter()
    while n < max_steps and (n == 0 or (time.perf_counter() - t0) < budget_s):
        for p in list(params.values()) + list(feats.values()):
            p.grad = None
        hybrid_train_step(params, names, feats, mask, labels, w["heads"], 0.1, gen)
        n += 1
    dt = time.perf_counter() - t0
    return bs * n / dt, n, dt


def cpu_baseline(w, budget_s=10.0, max_steps=400):
    """The reference CPU path timed on this host's cores: the oracle (oracle/hybrid_cpu.py, a
    torch-CPU restatement of src/fusion.py / src/attention.py) on the workload's per-GPU batch,
    at every host thread and at 4 threads (the reference's own cap, src/train.py:446-447).  The
    proxy is checked against the reference itself in scripts/cpu_proxy_check.py (same ATen ops,
    within +-15 %: profiles/r03_cpu_proxy_check.json).  C5 (L = 512) is infeasible on a CPU at its
    batch: B = 2 there, per-sample work identical (samples/s scale linearly in B)."""
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    lmax = max(w["L"])
    bs = w["B"] if lmax <= 128 else 2
    v_all, n_all, dt_all = _cpu_leg(w, bs, threads, budget_s, max_steps)
    v_4, n_4, dt_4 = _cpu_leg(w, bs, min(4, threads), budget_s, max_steps)
    torch.set_num_threads(threads)
    return {"value": round(v_all, 2), "unit": "samples/s", "cores": threads, "kind": "port",
            "value_4_threads": round(v_4, 2),
            "sample": f"{n_all} oracle steps of B={bs} at {threads} threads ({dt_all:.1f}s) and {n_4} at 4 threads "
                      f"({dt_4:.1f}s); per step the workload's fwd+CE+bwd (M={w['M']}, L={w['L']}, D={w['D']}, "
                      f"H={w['H']}, h={w['heads']}, dropout 0.1, fp32, torch {torch.__version__} CPU); proxy "
                      f"validated against the reference within 15% (scripts/cpu_proxy_check.py)"}


class ModuleRunner:
    """--path module: the nn.Module path src/train.py drives -- HybridFusion.forward under
    autograd, cross_entropy(label_smoothing=0.05) (mmf_ops.cross_entropy, the HIP kernel
    behind torch's functional signature), loss.backward() (parameter and input
    grads), then the exchange + clip + AdamW of harness.DPTrainer (flat buffers, bucketed
    all-reduce).  Eager; no graph."""

    def __init__(self, model, feats, mask, labels, pg, compiled=False, traceable=False):
        from harness import DPTrainer
        import mmf_ops
        self.ce = mmf_ops.cross_entropy
        self.model = model.train()
        # --path compiled: the reference trainer's own call, torch.compile(module, backend="inductor",
        # mode="reduce-overhead") (src/train.py:101-122, 193-231); the optimizer step stays outside.
        # HybridFusion is opaque to TorchDynamo by default; --traceable compiles its traced form
        # (custom operators, fullgraph) instead
        model.traceable = bool(traceable)
        self.fwd = (torch.compile(model, mode="reduce-overhead", fullgraph=bool(traceable)) if compiled else model)
        self.names = list(model.modality_names)
        self.feats = [f.clone().requires_grad_(True) for f in feats]
        self.mask, self.labels = mask, labels
        self.trainer = DPTrainer(model, accumulate=1, process_group=pg)
        self.loss = torch.zeros(())

    def forward_backward(self, eager=False):
        for f in self.feats:
            f.grad = None
        feats = dict(zip(self.names, self.feats))
        self.trainer.flat.arm()
        logits = (self.model if eager else self.fwd)(feats, self.mask)
        # (mmf_ops.cross_entropy: torch's cross_entropy(label_smoothing) in one HIP launch)
        loss = self.ce(logits, self.labels, label_smoothing=0.05)
        loss.backward()
        self.loss = loss.detach()

    def step(self):
        self.forward_backward()
        self.trainer.optimizer_step()


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    ap.add_argument("--path", default="step", choices=["step", "module", "compiled"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--traceable", action="store_true",
                    help="--path compiled: compile HybridFusion's traced form (custom operators, fullgraph) "
                         "instead of the default opaque module")
    ap.add_argument("--dropout", type=float, default=0.1,
                    help="diagnostics only: the benchmark workload is dropout 0.1")
    ap.add_argument("--skip-cpu", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=30,
                    help="eager steps of the kernel-level profile pass (untimed; after the capture, right "
                         "before the warm-up: they also bring the GPU to its steady clocks)")
    ap.add_argument("--dump-launches", default=None,
                    help="write every profiled launch (stage, kernel, ms, flops, bytes) of the last profile step "
                         "to this JSON file")
    ap.add_argument("--precision", default="highest", choices=["highest", "high", "medium"],
                    help="torch.set_float32_matmul_precision for the run: 'highest' = fp32 MFMA (the "
                         "fp32-parity headline), 'high' = bf16x3 (operands split into bf16 hi + lo, "
                         "three bf16 MFMAs, fp32 accumulate), 'medium' = bf16 MFMA operands, fp32 "
                         "accumulate (config/base.yaml:80)")
    args = ap.parse_args(argv)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: torch.distributed.run as a child, started before this process
        # touches the GPU (never an exec from a GPU-initialised process)
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        return subprocess.call(launcher_command(args.gpus, argv, free_port()), env=env)
    torch.set_float32_matmul_precision(args.precision)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
        pg = dist.group.WORLD
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, expected {args.gpus}")

    import mmf_native
    from fusion import HybridFusion
    from train_step import HybridTrainStep, shard_batch

    w = WORKLOADS[args.workload]
    M, D, H, heads, C = w["M"], w["D"], w["H"], w["heads"], w["C"]
    B = rank_batch(w, args.scaling, world)
    wr = dict(w, B=B)                         # the per-rank workload
    torch.manual_seed(0)                      # identical initial weights on every rank
    names = [f"m{i}" for i in range(M)]
    model = HybridFusion({n: D for n in names}, hidden_dim=H, num_classes=C, num_heads=heads,
                         dropout=args.dropout).to(dev)
    if args.scaling == "strong":
        # every rank takes its contiguous shard of ONE global batch (train_step.shard_batch)
        gf, gm, gl = make_inputs(w, w["GB"], 42, "cpu")
        feats, mask, labels = shard_batch(gf, gm, gl, rank, world)
        feats, mask, labels = [f.to(dev) for f in feats], mask.to(dev), labels.to(dev)
    else:
        feats, mask, labels = make_inputs(w, B, 42 + rank, dev)
    if args.path in ("module", "compiled"):
        trainer = ModuleRunner(model, feats, mask, labels, pg, compiled=args.path == "compiled",
                               traceable=args.traceable)
    else:
        trainer = HybridTrainStep(model, feats, mask, labels, process_group=pg)

    # the graph is captured first: its host work (about 17 ms at C2) leaves the GPU idle, and the
    # GPU's clocks then take ~30 ms of sustained load to ramp back up (kernel trace of
    # the driver's command, profiles/r06/timed_gap/).  The kernel-level profile pass that follows
    # keeps the GPU busy right up to the warm-up, so the timed region starts at the steady-state
    # rate a training loop runs at after its first few tens of milliseconds.
    # (the launch-lean L = 1 step runs eagerly: HybridTrainStep.replay_pays)
    graph = args.path == "step" and not args.no_graph and trainer.replay_pays()
    if graph:
        trainer.capture()

    # kernel-level timing (eager): hipEvents around each launch group and each
    # kernel launch, on the launch stream (mmf_profile_begin/end)
    # (the compiled path's profile steps run its module eagerly: the same library launches,
    # outside the graphs the compiled module captures)
    prof_fb = (lambda: trainer.forward_backward(eager=True)) if isinstance(trainer, ModuleRunner) \
        else trainer.forward_backward
    prof_fb()
    torch.cuda.synchronize(dev)
    mmf_native.profile_begin()
    for _ in range(args.profile_steps):
        prof_fb()
    stages, launches = mmf_native.profile_end()
    if args.dump_launches and rank == 0:
        per = len(launches) // max(1, args.profile_steps)
        with open(args.dump_launches, "w") as f:
            json.dump([{"stage": st_, "kernel": k_, "ms": ms_, "gflop": fl_ / 1e9, "mb": by_ / 1e6,
                        "tflops": fl_ / (ms_ * 1e-3) / 1e12 if ms_ > 0 else None}
                       for st_, k_, ms_, fl_, by_ in launches[-per:]], f, indent=1)
    per_stage = {}
    for name, ms in stages:
        t, n = per_stage.get(name, (0.0, 0))
        per_stage[name] = (t + ms, n + 1)
    avg_ms = {k: t / n for k, (t, n) in per_stage.items()}
    kernels = kernel_table(launches, args.profile_steps)

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
    # the per-step spread (median, p10 / p90): a separate pass after the timed region with one event
    # per step on the stream the steps run on -- an event recorded between graph replays costs
    # ~5 us of GPU time per step on this stack (scripts/replay_gap_probe.py), so the timed region
    # above has none
    n_spread = min(args.steps, 50)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n_spread + 1)]
    for i in range(n_spread):
        evs[i].record()
        trainer.step()
    evs[-1].record()
    torch.cuda.synchronize(dev)
    per_step = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(n_spread))
    med = per_step[len(per_step) // 2] if len(per_step) % 2 else 0.5 * (per_step[len(per_step) // 2 - 1] +
                                                                          per_step[len(per_step) // 2])
    loss = float(trainer.loss.item())

    if rank == 0:
        roofline = dominant_roofline(kernels, args.workload, args.precision)
        step_fl = total_step_flops(wr)
        cpu = None
        if world == 1 and not args.skip_cpu:
            cpu = cpu_baseline(w)
        Ls = w["L"]
        lens = Ls[0] if len(set(Ls)) == 1 else Ls
        mask_note = "" if w["keep"] >= 1 else f", modality masks keep={w['keep']} (+1% all-masked rows)"
        path_note = ("fused step (flat buffers, one hipGraph)" if graph else
                     "fused step, eager launches (the 3-launch L = 1 step: a graph replay's boundary costs "
                     "more than the dispatches it saves)" if args.path == "step" and not args.no_graph else
                     "fused step, eager" if args.path == "step" else
                     "nn.Module forward + autograd backward, eager (src/train.py's call path)"
                     if args.path == "module" else
                     ("torch.compile(module, mode='reduce-overhead', fullgraph=True) of the traced form "
                      "(HybridFusion.traceable) forward + backward" if args.traceable else
                      "torch.compile(module, mode='reduce-overhead') forward + backward (src/train.py's "
                      "compiled call path; HybridFusion opaque to TorchDynamo)"))
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "samples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
            "dtype": {"highest": "fp32", "high": "bf16x3 (fp32 operands split into bf16 hi + lo, three bf16 MFMAs, fp32 accumulate)",
                      "medium": "bf16 (fp32 accumulate)"}[args.precision],
            "data": "synthetic (N(0,1) encoder outputs, random-init weights, seeded)",
            "config": {"workload": f"{args.workload}: HybridFusion M={M} B={B}/gpu L={lens or 1}"
                                   f"{'' if max(Ls) else ' (2-D reference semantics)'} D={D} H={H} heads={heads} "
                                   f"C={C} dropout={args.dropout} train"
                                   f"{mask_note}"
                                   f", fwd+CE(ls=0.05)+bwd+clip(1.0)+AdamW; {path_note}",
                       "global_batch": B * world, "per_gpu_batch": B, "seq_len": lens or 1,
                       "parallelism": f"dp{world}", "path": args.path + ("+traceable" if args.traceable else ""),
                       "graph": graph, "matmul_precision": args.precision},
            "ms_per_step_median": round(med, 4),
            "ms_per_step_spread_source": f"a separate pass of {n_spread} event-timed steps after the timed region",
            "ms_per_step_p10_p90": [round(per_step[len(per_step) // 10], 4),
                                    round(per_step[min(len(per_step) - 1, (9 * len(per_step)) // 10)], 4)],
            "roofline": roofline,
            "cpu_baseline": cpu,
            "step_tflops_algorithmic": round(step_fl / (ms_per_step * 1e-3) / 1e12, 3),
            "step_gflop_algorithmic": round(step_fl / 1e9, 2),
            "step_gflop_executed_plan": round(sum(v["flops_per_launch"] * v["launches_per_step"]
                                                  for v in kernels.values()) / 1e9, 2),
            "stage_ms": {k: round(v, 4) for k, v in sorted(avg_ms.items(), key=lambda kv: -kv[1])},
            "kernels": {k: {kk: v[kk] for kk in ("ms_per_step", "launches_per_step", "avg_launch_ms",
                                                 "bound", "achieved", "unit", "frac", "mfma_frac", "hbm_frac")}
                        for k, v in list(kernels.items())[:12]},
            "loss": round(loss, 5),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
