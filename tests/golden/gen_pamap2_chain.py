"""Raw-input fixture for the end-to-end PAMAP2 chain (config C3), made from the REFERENCE.

Container-only tool (imports ``/root/reference/src``; never run on the GPU box).  It
complements ``pamap2_test.npz`` (gen_pamap2.py: the reference's encoder outputs,
fitted fusion head, logits and calibration metrics for the 44 present test chunks)
with the RAW rows of the first chunk of each present test shard, so a GPU test can
run the whole C3 chain on the HIP path -- manifest chunk gather (mmf_gather_chunks)
-> SequenceEncoder LSTMs (csrc/lstm.hip) -> LayerNorm -> HybridFusion -- and compare
against the reference's logits for those chunks.

Stored (derived data only, no source):
  * ``table`` (3 x 1024, 54) fp32: rows [0, 1024) of subject_102/activity_12,
    subject_103/activity_13, subject_107/activity_2 (``torch.load(weights_only=True)``);
    ``columns`` (54,) str: the shards' column names (data/preprocess.py:41-58);
  * ``test_index`` (3,): positions of those chunks in pamap2_test.npz's chunk list;
  * ``encoder_checksum/{m}`` (float64): the sum of every parameter of the reference's
    encoder for modality m built as gen_pamap2.build_encoders does
    (``torch.manual_seed(42)``, build_encoder per config/base.yaml).  The drop-in
    SequenceEncoder has the reference's construction order, so the same seed gives the
    same weights; the test rebuilds them and checks these sums before comparing.

Run:  python tests/golden/gen_pamap2_chain.py
"""

from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))

from cases import PAMAP2_CHUNK, PAMAP2_MODALITIES  # noqa: E402
from gen_pamap2 import REF, TEST_SHARDS, build_encoders, load_reference  # noqa: E402


def main():
    _, ref_encoders, _, _ = load_reference()
    with np.load(HERE / "pamap2_test.npz", allow_pickle=False) as z:
        index = z["chunk_index"]
    out = {}
    rows, test_index, columns = [], [], None
    for si, shard in enumerate(TEST_SHARDS):
        pl = torch.load(REF / "data" / "processed_tensors" / f"{shard}.pt", weights_only=True)
        if columns is None:
            columns = list(pl["columns"])
        assert list(pl["columns"]) == columns
        rows.append(pl["data"][:PAMAP2_CHUNK].float().numpy())
        pos = [i for i, (s, a, _) in enumerate(index) if s == si and a == 0]
        assert len(pos) == 1
        test_index.append(pos[0])
    out["table"] = np.concatenate(rows, axis=0).astype(np.float32)
    out["columns"] = np.array(columns)
    out["test_index"] = np.asarray(test_index, np.int64)
    encs, _ = build_encoders(ref_encoders)
    for m in PAMAP2_MODALITIES:
        out[f"encoder_checksum/{m}"] = np.asarray(
            [sum(float(p.detach().double().sum()) for p in encs[m].parameters())])
        out[f"encoder_keys/{m}"] = np.array(list(encs[m].state_dict().keys()))
    np.savez_compressed(HERE / "pamap2_chain.npz", **out)
    print(f"wrote pamap2_chain.npz: table {out['table'].shape}, test_index {test_index}")


if __name__ == "__main__":
    main()
