#!/usr/bin/env python3
"""Phase stamps of the launch-lean L = 1 step (csrc/l1.hip) from the diagnostic stamp build.

Build: make -C <pkg>/csrc stampsl1.  Run (box):
  MMF_LIB_PATH=<pkg>/csrc/libmmfusion_stampsl1.so python scripts/l1_stamps.py
The C2-L1 train step (bench.py's c2_l1 workload) is captured into a hipGraph as bench.py does
and replayed; the stamps of the last replay are read.  Per kernel: the workgroups' phase means
(s_memtime cycles between the stamps of thread 0; slot 0 is taken after the first global loads
are issued) and, from s_memrealtime (100 MHz, one clock for the chip), the kernel's span from its
first workgroup's start to its last workgroup's end and the gap to the next stamped kernel (the
cross-entropy and clip / AdamW launches are not stamped: they sit in the gaps they follow).
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

KERNELS = [
    ("l1_pair_fwd (l1_fwd_loss: pair part)", ["loads+keep+P'", "X'", "P = relu(X'Wk)", "O = P'(PWv)", "A = OWo + store",
                                              "store drain", "arrival count"]),
    ("l1_head_fwd (last pair workgroup of a tile)", ["loads+keep", "pooled", "gating+adaptive+fused", "h1",
                                                     "logits+loss+dz1"]),
    ("l1_head_bwd (head backward)", ["dfused", "dw+adaptive bwd+cvec"]),
    ("l1_key_bwd (pair part, after the head)", ["cvec + W_o/W_v + dO/dV/dP + count"]),
    ("l1_wgrad", ["main loop", "reduce + store"]),
]


def main():
    w = bench.WORKLOADS["c2_l1"]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    names = [f"m{i}" for i in range(w["M"])]
    model = HybridFusion({n: w["D"] for n in names}, hidden_dim=w["H"], num_classes=w["C"], num_heads=w["heads"],
                         dropout=0.1).to(dev)
    feats, mask, labels = bench.make_inputs(w, w["B"], 42, dev)
    step = HybridTrainStep(model, feats, mask, labels)
    step.capture()
    for _ in range(int(os.environ.get("STAMPS_WARM", "20"))):
        step.step()
    torch.cuda.synchronize()
    L = mmf_native.lib()
    L.mmf_l1_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros((5, 1024, 10), dtype=np.uint64)
    assert L.mmf_l1_stamps_read(buf.ctypes.data, buf.nbytes) == 0
    tiles = (w["B"] + 15) // 16
    nwg = [tiles * 6, None, None, tiles * 6, None]
    out = {"kernels": {}}
    spans = []
    t_first = int(buf[0, :tiles * 6, 8].astype(np.int64).min())   # this replay's first pair workgroup
    for k, (kn, ph) in enumerate(KERNELS):
        b = buf[k].astype(np.int64)
        n = nwg[k] if nwg[k] is not None else int(len(b))
        b = b[:n]
        # (the one-launch step's head phases are stamped by whichever pair workgroup finished its
        # tile last, at that workgroup's slot: keep the rows of this replay)
        b = b[(b[:, 8] >= t_first) & (b[:, 9] > 0)]
        if k == 4:   # zero-fill workgroups carry only the start stamps
            b = b[b[:, 2] > 0]
        st = b[:, :len(ph) + 1]
        d = np.diff(st, axis=1)
        rt0, rt1 = b[:, 8], b[:, 9]
        spans.append((kn, int(rt0.min()), int(rt1.max())))
        out["kernels"][kn] = {
            "workgroups": int(len(b)),
            "phase_mean_cycles": {p: round(float(d[:, i].mean()), 1) for i, p in enumerate(ph)},
            "wg_cycles_mean": round(float((st[:, -1] - st[:, 0]).mean()), 1),
            "wg_us_mean_realtime": round(float((rt1 - rt0).mean()) * 0.01, 2),
            "start_spread_us": round(float(rt0.max() - rt0.min()) * 0.01, 2),
            "span_us": round(float(rt1.max() - rt0.min()) * 0.01, 2),
        }
    t0 = spans[0][1]
    out["timeline_us"] = [{"kernel": kn, "start": round((a - t0) * 0.01, 2), "end": round((e - t0) * 0.01, 2)}
                          for kn, a, e in spans]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
