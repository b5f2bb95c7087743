#!/usr/bin/env python3
"""Where the driver's headline loses its ~1 ms.

BENCH_r05: 20 timed steps averaged 0.9857 ms while the same run's per-step median (a separate
event-timed pass after the timed region) was 0.9362 ms: about 1 ms of fixed cost per timed region.
This replays bench.py's sequence for C2 exactly (eager profile steps, capture, W warm-up replays,
synchronize, then K replays bracketed by synchronize) and splits the timed region's wall time:

  * host: perf_counter at t0, after every step() returned (the enqueue side), after the final
    synchronize;
  * device: one hipEvent before the first replay and one after the last (2 events: ~10 us), so
    wall - span = the time the GPU was NOT running the region's work (the first replay's
    submission before its first kernel + the synchronize's wake-up after the last);
  * per-step device times of the same region in a second pass with an event per step (the ~5 us
    an event costs between replays is stated in bench.py), to see whether the first replays after
    the warm-up are slower (clock ramp) or the steps are uniform.

Repeated R times in one process (the first region is bench.py's; the later ones show whether the
cost is per region or only the first).  Prints one JSON object.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-sensor-fusion-with-attention-rajeevatla_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--repeats", type=int, default=4)
    ap.add_argument("--idle-ms", type=float, default=0.0, help="host sleep between warm-up and region")
    args = ap.parse_args()
    import bench
    import mmf_native
    from fusion import HybridFusion
    from train_step import HybridTrainStep
    torch.set_float32_matmul_precision("highest")
    dev = torch.device("cuda", 0)
    w = bench.WORKLOADS["c2"]
    torch.manual_seed(0)
    names = [f"m{i}" for i in range(w["M"])]
    model = HybridFusion({n: w["D"] for n in names}, hidden_dim=w["H"], num_classes=w["C"], num_heads=w["heads"],
                         dropout=0.1).to(dev)
    feats, mask, labels = bench.make_inputs(w, w["B"], 42, dev)
    st = HybridTrainStep(model, feats, mask, labels)
    # bench.py: one eager step, 5 profiled eager steps, capture, warm-up
    st.forward_backward()
    torch.cuda.synchronize(dev)
    mmf_native.profile_begin()
    for _ in range(5):
        st.forward_backward()
    mmf_native.profile_end()
    st.capture()
    for _ in range(args.warmup):
        st.step()
    torch.cuda.synchronize(dev)
    out = {"steps": args.steps, "warmup": args.warmup, "regions": []}
    stream = torch.cuda.current_stream(dev)
    for r in range(args.repeats):
        if args.idle_ms:
            time.sleep(args.idle_ms / 1e3)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        e0.record(stream)
        enq = []
        for _ in range(args.steps):
            st.step()
            enq.append(time.perf_counter())
        e1.record(stream)
        t_enq = time.perf_counter()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        wall = (t1 - t0) * 1e3
        span = e0.elapsed_time(e1)
        # the same region with an event per step
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        torch.cuda.synchronize(dev)
        for i in range(args.steps):
            evs[i].record(stream)
            st.step()
        evs[-1].record(stream)
        torch.cuda.synchronize(dev)
        per = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
        out["regions"].append({
            "wall_ms": round(wall, 4), "gpu_span_ms": round(span, 4), "wall_minus_span_ms": round(wall - span, 4),
            "ms_per_step_wall": round(wall / args.steps, 4), "ms_per_step_span": round(span / args.steps, 4),
            "enqueue_ms": round((t_enq - t0) * 1e3, 4),
            "first_step_enqueue_ms": round((enq[0] - t0) * 1e3, 4),
            "per_step_ms_first5": [round(x, 4) for x in per[:5]],
            "per_step_ms_median": round(statistics.median(per), 4),
            "per_step_ms_max": round(max(per), 4),
        })
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
