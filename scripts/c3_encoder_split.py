#!/usr/bin/env python3
"""C3 step anatomy ("keep the LSTM on MIOpen, but measure it").

BASELINE.json configs[2]: PAMAP2 3-IMU + heart-rate, SequenceEncoder (LSTM)
per modality, HybridFusion.  One training step of the reference's
MultimodalFusionModule (src/train.py:233-324): per modality
SequenceEncoder(lstm, 1 layer, hidden 256 -> 128) (src/encoders.py:34-166,
config/base.yaml:37-56) + LayerNorm(128) (src/train.py:170-171, 267-268),
then HybridFusion(H=256, C=25, 4 heads) on the HIP path, CrossEntropy(0.05),
backward.  Encoders stay on PyTorch-ROCm (nn.LSTM -> MIOpen).

Synthetic inputs of the PAMAP2 manifest shape (the shards do not travel to the
GPU box): chunk_size 1024 steps (config/base.yaml:20), imu_* 17 features,
heart_rate 1.  The manifest loader's batch is 1 chunk (src/data.py:564-566);
B = 32 (config batch_size) is timed too.  Each phase is timed with hipEvents
on the current stream; prints one JSON line.

--encoders miopen,hip times both LSTM implementations: torch nn.LSTM (MIOpen)
and the package's SequenceEncoder on the persistent HIP recurrence
(csrc/lstm.hip), all four modalities' LSTMs in one launch per layer.

usage: python scripts/c3_encoder_split.py [--steps 20] [--batches 1,32] [--encoders miopen,hip]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-sensor-fusion-with-attention-rajeevatla_amd"))

MODALITIES = {"imu_hand": 17, "imu_chest": 17, "imu_ankle": 17, "heart_rate": 1}


class SeqEnc(nn.Module):
    """The reference SequenceEncoder's LSTM branch (src/encoders.py:67-75, 135-166)."""

    def __init__(self, input_dim: int, hidden: int = 256, out: int = 128, dropout: float = 0.1):
        super().__init__()
        self.rnn = nn.LSTM(input_dim, hidden, num_layers=1, batch_first=True)
        self.dropout_layer = nn.Dropout(dropout)
        self.projection = nn.Linear(hidden, out)

    def forward(self, x):
        _, (h, _) = self.rnn(x)
        return self.projection(self.dropout_layer(h[-1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batches", default="1,32")
    ap.add_argument("--chunk", type=int, default=1024)
    ap.add_argument("--encoders", default="miopen,hip")
    ap.add_argument("--precision", default="highest", choices=["highest", "medium"],
                    help="torch.set_float32_matmul_precision (config/base.yaml:80 sets 'medium')")
    args = ap.parse_args()
    torch.set_float32_matmul_precision(args.precision)
    from fusion import HybridFusion
    import encoders as hip_encoders

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    lns = nn.ModuleDict({m: nn.LayerNorm(128) for m in MODALITIES}).to(dev)
    fusion = HybridFusion({m: 128 for m in MODALITIES}, hidden_dim=256, num_classes=25, num_heads=4,
                          dropout=0.1).to(dev).train()
    results = []
    for kind in args.encoders.split(","):
        torch.manual_seed(0)
        if kind == "miopen":
            enc = nn.ModuleDict({m: SeqEnc(d) for m, d in MODALITIES.items()}).to(dev).train()
            run_enc = lambda xs: {m: enc[m](xs[m]) for m in MODALITIES}  # noqa: E731
        else:
            enc = nn.ModuleDict({m: hip_encoders.SequenceEncoder(d, 256, 128, num_layers=1)
                               for m, d in MODALITIES.items()}).to(dev).train()
            run_enc = lambda xs: hip_encoders.encode_sequences(dict(enc.items()), xs)  # noqa: E731
        for B in [int(b) for b in args.batches.split(",")]:
            g = torch.Generator().manual_seed(B)
            xs = {m: torch.randn(B, args.chunk, d, generator=g).to(dev) for m, d in MODALITIES.items()}
            labels = torch.randint(0, 25, (B,), generator=g).to(dev)
            mask = torch.ones(B, len(MODALITIES), device=dev)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
            acc = [0.0] * 4
            for it in range(args.warmup + args.steps):
                for p in list(enc.parameters()) + list(lns.parameters()) + list(fusion.parameters()):
                    p.grad = None
                ev[0].record()
                encoded = {m: lns[m](e) for m, e in run_enc(xs).items()}
                ev[1].record()
                leaf = {m: e.detach().requires_grad_(True) for m, e in encoded.items()}
                logits = fusion(leaf, mask)
                loss = F.cross_entropy(logits, labels, label_smoothing=0.05)
                ev[2].record()
                loss.backward()
                ev[3].record()
                torch.autograd.backward([encoded[m] for m in MODALITIES], [leaf[m].grad for m in MODALITIES])
                ev[4].record()
                torch.cuda.synchronize(dev)
                if it >= args.warmup:
                    for i in range(4):
                        acc[i] += ev[i].elapsed_time(ev[i + 1])
            n = args.steps
            enc_f, fus_f, fus_b, enc_b = (a / n for a in acc)
            total = enc_f + fus_f + fus_b + enc_b
            results.append({
                "encoders": kind, "batch": B, "chunk": args.chunk,
                "ms": {"encoders_fwd": round(enc_f, 3), "fusion_fwd": round(fus_f, 3),
                       "fusion_bwd": round(fus_b, 3), "encoders_bwd": round(enc_b, 3), "step": round(total, 3)},
                "fusion_share": round((fus_f + fus_b) / total, 4),
                "samples_per_s_step": round(B / (total * 1e-3), 2),
                "fusion_fwd_bwd_samples_per_s": round(B / ((fus_f + fus_b) * 1e-3), 1),
            })
    print(json.dumps({"config": "c3: PAMAP2 3-IMU+HR, SequenceEncoder(LSTM 1x256 -> 128)+LayerNorm, "
                                "HybridFusion(H=256, C=25, 4 heads), synthetic chunks, matmul precision "
                                + args.precision + (" (fp32)" if args.precision == "highest" else
                                                    " (bf16 MFMA operands in the fusion, fp32 LSTM recurrence)"),
                      "encoders": {"miopen": "torch nn.LSTM on ROCm (MIOpen)",
                                   "hip": "SequenceEncoder on the persistent HIP LSTM (csrc/lstm.hip)"},
                      "fusion": "mmfusion HIP",
                      "results": results}), flush=True)


if __name__ == "__main__":
    main()
