"""Generate the PAMAP2 logits / calibration parity fixture by running the REFERENCE.

Container-only tool (never run on the GPU box): it imports ``/root/reference/src``
(read-only, never copied) and reads the PAMAP2 ``.pt`` shards that ship with the
reference (``data/processed_tensors``), each loaded with
``torch.load(..., weights_only=True)``.  It writes ``pamap2_test.npz`` next to this
file.  Only derived tensors are stored (encoder outputs, labels, logits, metrics).

Pipeline (reference behaviour; the manifest loader yields one chunk per step):
  1. Present shards only (64 of the 91 manifest entries are missing):
     train = 18 shards, test = 3 shards (subject_102/12, 103/13, 107/2).
     Chunking at ``chunk_size: 1024`` (config/base.yaml:20, src/data.py:212-225),
     columns chosen by the reference's own ``_resolve_modality_columns``
     (src/data.py:180-210), ``nan_to_num`` (src/data.py:298-303).
  2. Encoders: ``build_encoder`` per ``config/base.yaml`` (LSTM, 1 layer, hidden 256,
     output 128; src/encoders.py:400-451) + ``nn.LayerNorm(128)``
     (src/train.py:158-171), seeded ``torch.manual_seed(42)`` (config seed), eval
     mode.  The encoders stay on PyTorch in the MI355X build (out of scope), so
     their OUTPUTS are this fixture's inputs: the (B, 128) per-modality features
     ``HybridFusion`` consumes (src/train.py:261-279).  ``enc_zero`` holds the
     encodings of all-zero raw inputs, the features
     ``_evaluate_with_modality_subset`` feeds for a missing modality
     (src/eval.py:400-404).
  3. HybridFusion(hidden 256, heads 4, 25 classes; config/base.yaml:12,28-31) with
     the seeded weights of ``cases.hybrid_state(seed=PAMAP2_SEED)`` (rebuildable on
     the GPU box).  Its fusion head (``gating_layers`` + ``classifier``) is then
     fitted BY THE REFERENCE MODULE on the present train chunks (eval mode, full
     batch, Adam 1e-2, ``PAMAP2_HEAD_STEPS`` steps, CE with label smoothing 0.05,
     src/train.py:185-186), so the calibration metrics are not those of a
     uniform-output model; the fitted head tensors are stored (0.3 MB).
  4. The reference eval chain on the 44 test chunks: logits (src/eval.py:80) ->
     softmax / max (:89-90) -> ``CalibrationMetrics`` ECE / MCE (15 bins, last bin
     closed; src/uncertainty.py:84-171) and NLL (:173-192); accuracy (:103).
     Missing-modality sweep: logits for each of the 2^M - 1 subsets
     (src/eval.py:342-424).

Run:  python tests/golden/gen_pamap2.py
"""

from __future__ import annotations

import itertools
import math
import sys
import time
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
REF = Path("/root/reference")

from cases import (PAMAP2_CHUNK, PAMAP2_CLASSES, PAMAP2_HEADS, PAMAP2_HIDDEN,  # noqa: E402
                   PAMAP2_MODALITIES, PAMAP2_OUT_DIM, PAMAP2_SEED, hybrid_state)

PAMAP2_HEAD_STEPS = 300

# Present shards of data/splits/{train,test}.txt.
TRAIN_SHARDS = [
    "subject_101/activity_12", "subject_101/activity_13", "subject_101/activity_24",
    "subject_102/activity_13", "subject_102/activity_5",
    "subject_104/activity_12", "subject_104/activity_13", "subject_104/activity_5",
    "subject_105/activity_12", "subject_105/activity_13", "subject_105/activity_24",
    "subject_106/activity_12", "subject_106/activity_13", "subject_106/activity_24",
    "subject_107/activity_12",
    "subject_108/activity_13", "subject_108/activity_24", "subject_108/activity_5",
]
TEST_SHARDS = ["subject_102/activity_12", "subject_103/activity_13", "subject_107/activity_2"]

# config/base.yaml:36-56 (encoders of the four PAMAP2 modalities)
ENCODER_CFG = {
    "imu_hand": {"type": "sequence", "input_dim": 17, "encoder_type": "lstm", "num_layers": 1},
    "imu_chest": {"type": "sequence", "input_dim": 17, "encoder_type": "lstm", "num_layers": 1},
    "imu_ankle": {"type": "sequence", "input_dim": 17, "encoder_type": "lstm", "num_layers": 1},
    "heart_rate": {"type": "sequence", "input_dim": 1, "encoder_type": "lstm", "num_layers": 1},
}


def load_reference():
    sys.path.insert(0, str(REF / "src"))
    import data as ref_data
    import encoders as ref_encoders
    import fusion as ref_fusion
    import uncertainty as ref_unc
    return ref_data, ref_encoders, ref_fusion, ref_unc


def chunks_of(ref_data, shard: str):
    payload = torch.load(REF / "data" / "processed_tensors" / f"{shard}.pt", weights_only=True)
    columns = list(payload["columns"])
    data = payload["data"]
    # the reference's own column resolution (src/data.py:180-210)
    mapping = ref_data.MultimodalDataset._resolve_modality_columns(
        SimpleNamespace(modalities=PAMAP2_MODALITIES), columns)
    col = {c: i for i, c in enumerate(columns)}
    idx = {m: torch.tensor([col[c] for c in mapping[m]], dtype=torch.long) for m in PAMAP2_MODALITIES}
    act = col["activity_id"]
    rows = data.shape[0]
    out = []
    for start in range(0, rows, PAMAP2_CHUNK):
        end = min(start + PAMAP2_CHUNK, rows)
        batch = data[start:end]
        lab = batch[:, act]
        assert torch.all(lab == lab[0]), "activity varies within chunk (src/data.py:295-296)"
        feats = {m: torch.nan_to_num(batch.index_select(1, ix).clone().float(), nan=0.0, posinf=0.0,
                                     neginf=0.0).unsqueeze(0) for m, ix in idx.items()}
        out.append((feats, int(lab[0].item()), (start, end)))
    return out


def build_encoders(ref_encoders):
    torch.manual_seed(42)   # config/base.yaml:117
    encs, norms = {}, {}
    for m in PAMAP2_MODALITIES:
        cfg = dict(ENCODER_CFG[m])
        input_dim = cfg.pop("input_dim")
        encs[m] = ref_encoders.build_encoder(m, input_dim, PAMAP2_OUT_DIM, cfg).eval()
        norms[m] = torch.nn.LayerNorm(PAMAP2_OUT_DIM).eval()
    return encs, norms


@torch.no_grad()
def encode(encs, norms, chunks, with_zero: bool):
    enc = np.zeros((len(chunks), len(PAMAP2_MODALITIES), PAMAP2_OUT_DIM), np.float32)
    enc_zero = np.zeros_like(enc)
    for i, (feats, _, _) in enumerate(chunks):
        for j, m in enumerate(PAMAP2_MODALITIES):
            enc[i, j] = norms[m](encs[m](feats[m]))[0].numpy()
            if with_zero:
                enc_zero[i, j] = norms[m](encs[m](torch.zeros_like(feats[m])))[0].numpy()
    return enc, enc_zero


def main():
    torch.set_float32_matmul_precision("highest")
    torch.set_num_threads(8)
    ref_data, ref_encoders, ref_fusion, ref_unc = load_reference()
    t0 = time.time()
    train_chunks = [c for s in TRAIN_SHARDS for c in chunks_of(ref_data, s)]
    test_chunks, test_index = [], []
    for si, s in enumerate(TEST_SHARDS):
        for c in chunks_of(ref_data, s):
            test_chunks.append(c)
            test_index.append((si, c[2][0], c[2][1]))
    print(f"chunks: train {len(train_chunks)} test {len(test_chunks)}", flush=True)
    encs, norms = build_encoders(ref_encoders)
    tr_enc, _ = encode(encs, norms, train_chunks, with_zero=False)
    te_enc, te_zero = encode(encs, norms, test_chunks, with_zero=True)
    tr_lab = torch.tensor([c[1] for c in train_chunks], dtype=torch.long)
    te_lab = torch.tensor([c[1] for c in test_chunks], dtype=torch.long)
    print(f"encoded in {time.time() - t0:.1f}s", flush=True)

    names = list(PAMAP2_MODALITIES)
    dims = {m: PAMAP2_OUT_DIM for m in names}
    model = ref_fusion.HybridFusion(dims, hidden_dim=PAMAP2_HIDDEN, num_classes=PAMAP2_CLASSES,
                                    num_heads=PAMAP2_HEADS, dropout=0.1)
    sd = hybrid_state(names, dims, PAMAP2_HIDDEN, PAMAP2_CLASSES, PAMAP2_SEED)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    model.eval()

    # fit the fusion head on the present train chunks (reference module, eval mode)
    head_prefix = ("gating_layers.", "classifier.")
    for k, p in model.named_parameters():
        p.requires_grad_(k.startswith(head_prefix))
    head = [p for k, p in model.named_parameters() if k.startswith(head_prefix)]
    opt = torch.optim.Adam(head, lr=1e-2)
    crit = torch.nn.CrossEntropyLoss(label_smoothing=0.05)
    tr_feats = {m: torch.from_numpy(tr_enc[:, j]) for j, m in enumerate(names)}
    tr_mask = torch.ones(len(train_chunks), len(names))
    for step in range(PAMAP2_HEAD_STEPS):
        opt.zero_grad()
        loss = crit(model(tr_feats, tr_mask), tr_lab)
        loss.backward()
        opt.step()
        if step % 50 == 0 or step == PAMAP2_HEAD_STEPS - 1:
            print(f"head step {step}: train loss {loss.item():.4f}", flush=True)
    for p in model.parameters():
        p.requires_grad_(True)

    out = {"enc": te_enc, "enc_zero": te_zero, "labels": te_lab.numpy(),
           "chunk_index": np.asarray(test_index, np.int64)}
    for k, v in model.state_dict().items():
        if k.startswith(head_prefix):
            out[f"head/{k}"] = v.detach().numpy().copy()

    CM = ref_unc.CalibrationMetrics
    with torch.no_grad():
        feats = {m: torch.from_numpy(te_enc[:, j]) for j, m in enumerate(names)}
        mask = torch.ones(len(test_chunks), len(names))
        logits = model(feats, mask)
        probs = torch.softmax(logits, dim=1)                     # src/eval.py:89-90
        conf, preds = torch.max(probs, dim=1)
        out["logits"] = logits.numpy()
        out["confidences"] = conf.numpy()
        out["preds"] = preds.numpy()
        out["ece"] = np.asarray([CM.expected_calibration_error(conf, preds, te_lab, num_bins=15)])
        out["mce"] = np.asarray([CM.maximum_calibration_error(conf, preds, te_lab, num_bins=15)])
        out["nll"] = np.asarray([CM.negative_log_likelihood(logits, te_lab)])
        out["accuracy"] = np.asarray([(preds == te_lab).float().mean().item()])
        # missing-modality sweep (src/eval.py:342-424): zeroed raw inputs + subset mask
        subsets = []
        for r in range(1, len(names) + 1):
            subsets.extend(itertools.combinations(range(len(names)), r))
        sub_logits = np.zeros((len(subsets), len(test_chunks), PAMAP2_CLASSES), np.float32)
        sub_acc = np.zeros(len(subsets), np.float64)
        for si, sub in enumerate(subsets):
            f = {m: torch.from_numpy(te_enc[:, j] if j in sub else te_zero[:, j]) for j, m in enumerate(names)}
            mk = torch.zeros(len(test_chunks), len(names))
            for j in sub:
                mk[:, j] = 1
            lg = model(f, mk)
            sub_logits[si] = lg.numpy()
            sub_acc[si] = (torch.argmax(lg, dim=1) == te_lab).float().mean().item()
        out["subset_mask"] = np.asarray([[1.0 if j in s else 0.0 for j in range(len(names))] for s in subsets],
                                        np.float32)
        out["subset_logits"] = sub_logits
        out["subset_accuracy"] = sub_acc
    np.savez_compressed(HERE / "pamap2_test.npz", **out)
    print(f"wrote pamap2_test.npz: acc {out['accuracy'][0]:.4f} ece {out['ece'][0]:.5f} "
          f"mce {out['mce'][0]:.5f} nll {out['nll'][0]:.5f} ({time.time() - t0:.1f}s)")
    assert math.isfinite(float(out["ece"][0]))


if __name__ == "__main__":
    main()
