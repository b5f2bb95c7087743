#!/usr/bin/env python3
"""Phase shares of the fused attention backward from the diagnostic stamp build.

Build: make -C <pkg>/csrc stamps (stampsf for the forward, argument "fwd").  Run (box):
  MMF_LIB_PATH=<pkg>/csrc/libmmfusion_stamps.so MMF_ATTN_BWD=v1 python scripts/attn_stamps.py
Long-key fused kernels (attn_long.hip, C5 medium; make stampsl):
  MMF_LIB_PATH=<pkg>/csrc/libmmfusion_stampsl.so python scripts/attn_stamps.py long   (backward)
  MMF_LIB_PATH=<pkg>/csrc/libmmfusion_stampsl.so MMF_NO_LONG_BWD_STAMP=1 ... longf  (forward: the
  forward's stamps are overwritten by the backward's, so the bwd stamps are read after a forward-only
  pass: see main_long)
Stamps (s_memtime, wave 0 of every workgroup): 0 start, 1 K/Q images loaded, 2 S/P/D,
3 dS, 4 dQ stored, 5 dK quarters, 6 dK stored.  Prints per-phase mean cycles, the
workgroup lifetime, and how the start times of the workgroups on one CU are spread
(lockstep or not).  Shares, not lengths: the stamps themselves cost cycles.
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "multimodal-sensor-fusion-with-attention-rajeevatla_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)

import mmf_native  # noqa: E402
from fusion import HybridFusion  # noqa: E402
from train_step import HybridTrainStep  # noqa: E402
import bench  # noqa: E402


def main_long(kernel):
    """attn_long.hip stamps: per workgroup, phase sums over the query blocks of wave 0 (slots 0-4:
    to barrier A, barrier A wait, to barrier B, barrier B wait, after B) and of the first wave of
    the younger half (slots 5-8), the s_memrealtime lifetime in slot 9.  The last launch of the
    step is read: the backward's last launch ("long"), or for "longf" a forward-only pass."""
    w = bench.WORKLOADS["c5"]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    names = [f"m{i}" for i in range(w["M"])]
    model = HybridFusion({n: w["D"] for n in names}, hidden_dim=w["H"], num_classes=w["C"], num_heads=w["heads"],
                         dropout=0.1).to(dev)
    torch.set_float32_matmul_precision("medium")
    feats, mask, labels = bench.make_inputs(w, w["B"], 42, dev)
    step = HybridTrainStep(model, feats, mask, labels)
    L = mmf_native.lib()
    reader = L.mmf_long_stamps_read
    reader.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    for _ in range(int(os.environ.get("STAMPS_WARM", "3"))):
        step.forward_backward()
    if kernel == "longf":
        model.train()
        with torch.no_grad():
            model(dict(zip(names, feats)), mask)
    torch.cuda.synchronize()
    buf = np.zeros((8192, 10), dtype=np.uint64)
    assert reader(buf.ctypes.data, buf.nbytes) == 0
    nwg = w["B"] * w["heads"] * 10
    st = buf[:nwg].astype(np.int64)
    ok = st[:, 9] > 0
    st = st[ok]
    if kernel == "long":
        ph = ["S/P/D partial", "barrier A", "dS + dQ/dK MFMA + partial dQ", "barrier B", "dQ reduce + store"]
    else:
        ph = ["loads + max", "barrier A", "next S + exp + sums", "barrier B", "P' tile + colsum"]
    tot0 = st[:, 0:5].sum(axis=1)
    out = {"kernel": kernel, "workgroups": int(ok.sum()),
           "wave0_loop_cycles_mean": float(tot0.mean()),
           "wave0_phase_mean_cycles": {n: float(st[:, i].mean()) for i, n in enumerate(ph)},
           "wave0_phase_share": {n: round(float(st[:, i].mean() / tot0.mean()), 3) for i, n in enumerate(ph)},
           "younger_phase_mean_cycles": {n: float(st[:, 5 + i].mean()) for i, n in enumerate(ph[:4])},
           "wg_lifetime_us_median": float(np.median(st[:, 9]) * 0.01),
           "shader_clock_ghz_median": float(np.median(tot0 / st[:, 9] * 0.1))}
    print(json.dumps(out, indent=1))


def main():
    kernel = sys.argv[1] if len(sys.argv) > 1 else "attn"
    if kernel in ("long", "longf"):
        return main_long(kernel)
    w = bench.WORKLOADS["c2"]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    names = [f"m{i}" for i in range(w["M"])]
    model = HybridFusion({n: w["D"] for n in names}, hidden_dim=w["H"], num_classes=w["C"], num_heads=w["heads"],
                         dropout=0.1).to(dev)
    feats, mask, labels = bench.make_inputs(w, w["B"], 42, dev)
    if os.environ.get("STAMPS_ZERO") == "1":   # trivial operands (the DVFS check, MICROARCH 'give-back' 1)
        feats = [torch.zeros_like(f) for f in feats]
        with torch.no_grad():
            for prm in model.parameters():
                prm.zero_()
    step = HybridTrainStep(model, feats, mask, labels)
    L = mmf_native.lib()
    occ = (ctypes.c_int * 2)()
    L.mmf_attn_occupancy(occ)
    print("runtime occupancy (blocks/CU): fused bwd", occ[0], "pooled fwd", occ[1], flush=True)
    reader = L.mmf_stamps_read if kernel in ("attn", "fwd") else L.mmf_tail_stamps_read
    reader.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    # STAMPS_WARM back-to-back steps first (the clock the chip holds under sustained load;
    # the stamps of the last step are read)
    for _ in range(int(os.environ.get("STAMPS_WARM", "3"))):
        step.forward_backward()
    torch.cuda.synchronize()
    buf = np.zeros((8192, 10), dtype=np.uint64)
    assert reader(buf.ctypes.data, buf.nbytes) == 0
    if kernel == "attn":
        nwg, nst = 6 * w["B"] * w["heads"], 7
        names_ph = ["load", "S/P/D", "dS", "dQ", "dK quarters", "dK store"]
    elif kernel == "fwd":   # attn_pool_fwd_lean, libmmfusion_stampsf.so (make stampsf)
        nwg, nst = 6 * w["B"] * w["heads"], 6
        names_ph = ["K/Q load", "S = K Q^T + max", "exp + sum", "dropout + colsum", "pbar store"]
    else:   # tail_pair_fwd_kernel: grid (B, pairs)
        nwg, nst = 6 * w["B"], 6
        names_ph = ["pbar + r", "U = pbar P_k", "Obar GEMV", "Abar GEMV", "stores"]
    st = buf[:nwg, :nst].astype(np.int64)
    hw = buf[:nwg, 9]
    t0 = st[:, 0].min()
    ph = np.diff(st, axis=1)
    last = nst - 1
    out = {"kernel": kernel, "workgroups": int(nwg),
           "kernel_cycles": int(st[:, last].max() - t0),
           "wg_lifetime_mean": float((st[:, last] - st[:, 0]).mean()),
           "phase_mean_cycles": {n: float(ph[:, i].mean()) for i, n in enumerate(names_ph)},
           "phase_share": {n: round(float(ph[:, i].mean() / (st[:, last] - st[:, 0]).mean()), 3)
                           for i, n in enumerate(names_ph)}}
    # s_memtime counters are per XCD: spans and residency per XCC
    xcc_all = ((hw >> 32).astype(np.int64)) & 0xF
    spans, resid = [], []
    for x in np.unique(xcc_all):
        sel = xcc_all == x
        span = int(st[sel, last].max() - st[sel, 0].min())
        spans.append(span)
        # mean workgroups resident = sum of lifetimes / span
        resid.append(float((st[sel, last] - st[sel, 0]).sum() / span))
    if kernel in ("attn", "fwd"):
        rt = (buf[:nwg, 8].astype(np.int64) - buf[:nwg, 7].astype(np.int64))
        ok = rt > 0
        out["shader_clock_ghz_median"] = float(np.median((st[ok, last] - st[ok, 0]) / rt[ok] * 0.1))
        out["wg_lifetime_us_median"] = float(np.median(rt[ok]) * 0.01)
    out["xcc_span_cycles_mean"] = float(np.mean(spans))
    out["resident_wgs_per_xcc_mean"] = float(np.mean(resid))
    out["resident_wgs_per_cu_mean"] = float(np.mean(resid)) / 32.0
    # workgroups sharing a CU: HW_ID cu / sh / se fields + XCC id
    hw32 = (hw & 0xFFFFFFFF).astype(np.int64)
    xcc = (hw >> 32).astype(np.int64) & 0xF
    cu_key = xcc * 4096 + ((hw32 >> 8) & 0xFF) + (((hw32 >> 12) & 0xF) << 8) * 0   # cu_id | sh_id | se_id (tg_id dropped)
    cu_key = xcc * 65536 + (((hw32 >> 8) & 0xF) | (((hw32 >> 12) & 0x1) << 4) | (((hw32 >> 13) & 0x7) << 5))
    starts = {}
    for k, s0 in zip(cu_key, st[:, 0] - t0):
        starts.setdefault(int(k), []).append(int(s0))
    spreads = []
    for k, v in starts.items():
        v = sorted(v)
        # first 4 residents of this CU: how far apart did they start?
        if len(v) >= 4:
            spreads.append(v[3] - v[0])
    # residency: the most workgroups alive at once on one CU (start / end stamps share that CU's
    # XCD clock), and the mean number alive over the CU's busy span
    ev = {}
    for k, s0, s1 in zip(cu_key, st[:, 0], st[:, last]):
        ev.setdefault(int(k), []).append((int(s0), int(s1)))
    peak, mean_alive = [], []
    for k, v in ev.items():
        pts = sorted([(a, 1) for a, _ in v] + [(b, -1) for _, b in v])
        cur = best = 0
        for _, d in pts:
            cur += d
            best = max(best, cur)
        peak.append(best)
        span = max(b for _, b in v) - min(a for a, _ in v)
        mean_alive.append(sum(b - a for a, b in v) / span if span > 0 else 0.0)
    out["resident_wgs_per_cu_peak_median"] = float(np.median(peak))
    out["resident_wgs_per_cu_mean_alive"] = float(np.mean(mean_alive))
    out["cus_seen"] = len(starts)
    out["wgs_per_cu_mean"] = float(np.mean([len(v) for v in starts.values()]))
    out["first4_start_spread_cycles_median"] = float(np.median(spreads)) if spreads else None
    # start-time histogram in units of the mean lifetime
    life = out["wg_lifetime_mean"]
    hist = np.histogram((st[:, 0] - t0) / life, bins=12)[0].tolist()
    out["start_hist_per_lifetime"] = hist
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
