"""CPU restatement of the manifest data path (ORACLE; test infrastructure only).

Only ``tests/`` may import it, as the checker of the HIP gather
(``mmf_gather_chunks``) and of the package's ``manifest.py`` host logic.
Pinned by ``tests/golden/manifest_pamap2.npz``, produced by the reference's own
``MultimodalDataset`` (``tests/golden/gen_manifest.py``).

  chunk windows                 src/data.py:205-217 (_build_chunks)
  __getitem__ (manifest branch) src/data.py:275-298: rows [start, end) of the shard,
                                label = activity_id of the first row (constant per chunk),
                                per modality index_select(columns) -> nan_to_num -> (1, T, c)
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np


def chunk_windows(shard_rows: Sequence[int], chunk_size: int) -> List[Tuple[int, int, int]]:
    out = []
    for s, rows in enumerate(shard_rows):
        start = 0
        while start < rows:
            end = min(start + chunk_size, rows)
            out.append((s, start, end))
            start = end
    return out


def gather_chunk(shards: Sequence[np.ndarray], chunk: Tuple[int, int, int], cols: Dict[str, List[int]],
                 activity_col: int):
    s, a, b = chunk
    rows = shards[s][a:b]
    lab = rows[:, activity_col]
    if not np.all(lab == lab[0]):
        raise ValueError("Activity id varies within shard chunk.")
    feats = {}
    for m, idx in cols.items():
        v = rows[:, idx].astype(np.float32)
        feats[m] = np.where(np.isfinite(v), v, 0.0).astype(np.float32)[None]
    return feats, int(lab[0])
