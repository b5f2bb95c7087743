#!/usr/bin/env python3
"""Where the drop-in module path's host time goes (VERDICT r04 "next" #1).

Builds bench.py's ModuleRunner for a workload (default c2_l1: the reference's own 2-D
inputs) on the eager and the torch.compile(mode="reduce-overhead") paths and reports, per
step in steady state:
  * the host wall time of each phase (forward call, loss, backward, optimizer step), timed
    without synchronising (the GPU work of these steps is shorter than their host work, so
    the host phases are the step);
  * the whole step with a synchronize at the end;
  * the cudagraph skip counters of inductor and torch.profiler's top CPU ops.
usage: python scripts/host_phase_profile.py [--workload c2_l1] [--steps 50] [--out file.json]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multimodal-sensor-fusion-with-attention-rajeevatla_amd"))

import bench  # noqa: E402


def phases(runner, steps):
    acc = {"fwd": 0.0, "loss": 0.0, "bwd": 0.0, "opt": 0.0}
    torch.cuda.synchronize()
    t_all = time.perf_counter()
    for _ in range(steps):
        t0 = time.perf_counter()
        for f in runner.feats:
            f.grad = None
        feats = dict(zip(runner.names, runner.feats))
        runner.trainer.flat.arm()
        logits = runner.fwd(feats, runner.mask)
        t1 = time.perf_counter()
        loss = runner.ce(logits, runner.labels, label_smoothing=0.05)
        t2 = time.perf_counter()
        loss.backward()
        t3 = time.perf_counter()
        runner.trainer.optimizer_step()
        t4 = time.perf_counter()
        acc["fwd"] += t1 - t0
        acc["loss"] += t2 - t1
        acc["bwd"] += t3 - t2
        acc["opt"] += t4 - t3
    torch.cuda.synchronize()
    total = time.perf_counter() - t_all
    out = {k: round(v / steps * 1e3, 4) for k, v in acc.items()}
    out["step_synced_ms"] = round(total / steps * 1e3, 4)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2_l1")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--out", default=None)
    ap.add_argument("--paths", default="module,compiled,compiled_traceable")
    ap.add_argument("--trace", default=None, help="directory: write each path's 10-step CPU chrome trace there")
    args = ap.parse_args()
    from fusion import HybridFusion
    dev = torch.device("cuda", 0)
    w = bench.WORKLOADS[args.workload]
    res = {"workload": args.workload}
    for path in args.paths.split(","):
        try:
            run_path(args, w, dev, path, res, HybridFusion)
        except Exception as e:  # noqa: BLE001  (one path failing must not lose the others' numbers)
            res[path] = {"error": repr(e)[:2000]}
            print(path, "failed:", repr(e)[:500], flush=True)
        if args.out:
            with open(args.out, "w") as f:
                json.dump(res, f, indent=1, default=str)
    try:
        from torch._dynamo.utils import counters
        res["inductor_counters"] = {k: dict(v) for k, v in counters.items() if v}
    except Exception as e:  # noqa: BLE001
        res["inductor_counters"] = repr(e)
    txt = json.dumps(res, indent=1, default=str)
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt)
    print(txt)


def run_path(args, w, dev, path, res, HybridFusion):
    if True:
        torch.manual_seed(0)
        names = [f"m{i}" for i in range(w["M"])]
        model = HybridFusion({n: w["D"] for n in names}, hidden_dim=w["H"], num_classes=w["C"],
                             num_heads=w["heads"], dropout=0.1).to(dev)
        feats, mask, labels = bench.make_inputs(w, w["B"], 42, dev)
        r = bench.ModuleRunner(model, feats, mask, labels, None, compiled=path.startswith("compiled"),
                               traceable=path.endswith("traceable"))
        for _ in range(10):
            r.step()
        torch.cuda.synchronize()
        res[path] = phases(r, args.steps)
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
            for _ in range(10):
                r.step()
            torch.cuda.synchronize()
        if args.trace:
            os.makedirs(args.trace, exist_ok=True)
            prof.export_chrome_trace(os.path.join(args.trace, path + ".json"))
        ka = prof.key_averages()
        top = sorted(ka, key=lambda e: -e.self_cpu_time_total)[:25]
        res[path + "_top_self_cpu_us_per_step"] = [
            (e.key, round(e.self_cpu_time_total / 10, 1), round(e.count / 10, 2)) for e in top]
        print(path, json.dumps(res[path]), flush=True)


if __name__ == "__main__":
    main()
