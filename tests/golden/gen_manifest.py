"""Golden fixture for the manifest data path, produced by the REFERENCE dataset.

Container-only tool (imports /root/reference/src).  It slices two present
PAMAP2 shards (the first rows of subject_102/activity_12 and
subject_103/activity_13, with a NaN and an inf planted to exercise
nan_to_num), writes them as .pt shards + a manifest in a temp directory, runs
the reference ``MultimodalDataset`` (src/data.py:110-343, manifest branch,
chunk_size 64, modalities imu_hand / imu_chest / imu_ankle / heart_rate), and
stores the shard slices (inputs) and the reference's chunk table and
per-chunk features / labels (outputs) in manifest_pamap2.npz.

Run:  python tests/golden/gen_manifest.py
"""
from __future__ import annotations

import sys
import tempfile
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REF = Path("/root/reference")
SHARDS = [("subject_102/activity_12.pt", 150), ("subject_103/activity_13.pt", 100)]
MODALITIES = ["imu_hand", "imu_chest", "imu_ankle", "heart_rate"]
CHUNK = 64


def main():
    sys.path.insert(0, str(REF / "src"))
    import data as ref_data
    out = {}
    with tempfile.TemporaryDirectory() as td:
        root = Path(td) / "a" / "b"           # manifest.parents[2] = td/a (project root of relative paths)
        (root / "splits").mkdir(parents=True)
        lines = []
        for i, (rel, rows) in enumerate(SHARDS):
            pl = torch.load(REF / "data" / "processed_tensors" / rel, weights_only=True)
            d = pl["data"][:rows].clone().float()
            if i == 0:
                cols = list(pl["columns"])
                d[3, cols.index("hand_acc16_x_ms2")] = float("nan")
                d[70, cols.index("heart_rate_bpm")] = float("inf")
            out[f"shard{i}/data"] = d.numpy()
            path = Path(td) / f"shard{i}.pt"
            torch.save({"columns": list(pl["columns"]), "data": d}, path)
            lines.append(f"{path},{rows}")
        lines.insert(1, "ignored.pt,0")         # rows <= 0: skipped before the existence check
        (root / "splits" / "test.txt").write_text("\n".join(lines) + "\n")
        ds = ref_data.MultimodalDataset(str(root), modalities=MODALITIES, split="test", chunk_size=CHUNK,
                                        modality_dropout=0.0, prefetch_shards=True)
        out["columns"] = np.array(list(pl["columns"]))
        out["chunks"] = np.array(ds._chunks, dtype=np.int64)
        for idx in range(len(ds)):
            feats, label, mask = ds[idx]
            for m in MODALITIES:
                out[f"chunk{idx}/{m}"] = feats[m].numpy()
            out[f"chunk{idx}/label"] = label.numpy()
            out[f"chunk{idx}/mask"] = mask.numpy()
    np.savez_compressed(HERE / "manifest_pamap2.npz", **out)
    print("wrote manifest_pamap2.npz", len(out), "arrays")


if __name__ == "__main__":
    main()
