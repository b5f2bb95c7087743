"""GPU-resident manifest data path.

Mirrors the manifest branch of the reference's ``MultimodalDataset``
(src/data.py:110-343) over the ``.pt`` shard format written by
data/preprocess.py:130-139 (``{"columns": List[str], "data": float32 (rows, ncols)}``):

  * manifest ``{data_dir}/splits/{split}.txt``, one ``path,rows`` per line;
    relative paths resolve against ``manifest.parents[2]``; entries with
    ``rows <= 0`` are skipped (src/data.py:113-141), with the reference's
    errors: ``ValueError("Malformed manifest entry ...")``,
    ``FileNotFoundError("Shard referenced in manifest not found: ...")``,
    ``ValueError("No shards found in manifest ...")``;
  * modality -> column resolution by prefix (``imu_hand`` -> ``hand_*``,
    ``*_imu`` suffixes, ``heart_rate`` -> ``heart_rate_bpm``) and its
    ``ValueError("Could not resolve modality ...")`` (src/data.py:171-203);
    ``ValueError("activity_id column missing from tensor shards.")`` (:151-152);
  * chunk windows ``(shard, start, end)`` of ``chunk_size`` rows per shard, the
    last one ragged (``_build_chunks``, :205-217);
  * ``__getitem__`` -> ``({m: (1, T, c_m)}, label (1,), mask (1, M))``:
    nan_to_num'd features, the chunk's activity_id (``ValueError("Activity id
    varies within shard chunk.")`` otherwise), modality dropout with at least
    one modality kept (:275-343).

MI355X-first differences: every shard of the split is loaded once
(``torch.load(weights_only=True)``) into ONE (rows, ncols) fp32 table in HBM,
the chunk table lives on the device, and ``gather(chunk_ids)`` builds a whole
batch of windows (B, T, c_m) per modality in one HIP launch
(``mmf_gather_chunks``, csrc/chunks.hip), zero-padded past each chunk's length
(returned), so the encoders see batches instead of the reference's
batch-of-one loader (src/data.py:564-566).  The chunk cache file and the
host-RAM shard LRU of the reference are not needed: the table is resident.
"""

from __future__ import annotations

import ctypes
import os
import sys
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import mmf_native as _nat  # noqa: E402


def parse_manifest(manifest_path: Path) -> List[Tuple[Path, int]]:
    """(shard path, rows) entries of a manifest, with the reference's checks (src/data.py:113-141)."""
    entries: List[Tuple[Path, int]] = []
    project_root = manifest_path.parents[2] if len(manifest_path.parents) >= 3 else Path(".")
    with manifest_path.open("r", encoding="utf-8") as handle:
        for line in handle:
            line = line.strip()
            if not line:
                continue
            if "," not in line:
                raise ValueError(f"Malformed manifest entry '{line}' in {manifest_path}")
            path_str, rows_str = line.split(",", 1)
            shard_path = Path(path_str)
            if not shard_path.is_absolute():
                shard_path = (project_root / shard_path).resolve()
            rows = int(rows_str)
            if rows <= 0:
                continue
            if not shard_path.exists():
                raise FileNotFoundError(f"Shard referenced in manifest not found: {shard_path}")
            entries.append((shard_path, rows))
    if not entries:
        raise ValueError(f"No shards found in manifest {manifest_path}")
    return entries


def resolve_modality_columns(columns: Sequence[str], modalities: Sequence[str]) -> Dict[str, List[str]]:
    """Modality -> shard columns (src/data.py:171-203)."""
    column_set = set(columns)
    mapping: Dict[str, List[str]] = {}
    for modality in modalities:
        normalized = modality.lower()
        candidate: List[str] = []
        if normalized in {"heart_rate", "heart", "hr"}:
            if "heart_rate_bpm" in column_set:
                candidate = ["heart_rate_bpm"]
        else:
            prefix = normalized
            if prefix.startswith("imu_"):
                prefix = prefix.split("imu_", 1)[1]
            if prefix.endswith("_imu"):
                prefix = prefix.rsplit("_imu", 1)[0]
            prefix = prefix.replace(" ", "")
            candidate = [col for col in columns if col.startswith(f"{prefix}_")]
        if not candidate:
            raise ValueError(f"Could not resolve modality '{modality}'. Available columns: {list(columns)}")
        mapping[modality] = candidate
    return mapping


def build_chunks(shard_rows: Sequence[int], chunk_size: Optional[int]) -> List[Tuple[int, int, int]]:
    """(shard_idx, start, end) windows (src/data.py:205-217)."""
    chunks: List[Tuple[int, int, int]] = []
    for shard_idx, rows in enumerate(shard_rows):
        if chunk_size is None:
            chunks.append((shard_idx, 0, rows))
            continue
        start = 0
        while start < rows:
            end = min(start + chunk_size, rows)
            chunks.append((shard_idx, start, end))
            start = end
    return chunks


class ManifestShards:
    """The shards of one split, resident in HBM, with batched chunk gathers."""

    def __init__(self, data_dir, split: str, modalities: Sequence[str], chunk_size: Optional[int] = 1024,
                 modality_dropout: float = 0.0, device="cuda"):
        self.data_dir = Path(data_dir)
        self.split = split
        self.modalities = list(modalities)
        self.chunk_size = chunk_size
        self.modality_dropout = float(modality_dropout)
        self.device = torch.device(device)
        manifest_path = self.data_dir / "splits" / f"{split}.txt"
        entries = parse_manifest(manifest_path)
        payloads = [torch.load(p, weights_only=True) for p, _ in entries]
        columns = list(payloads[0]["columns"])
        self.columns = columns
        col_index = {name: i for i, name in enumerate(columns)}
        self.modality_columns = resolve_modality_columns(columns, self.modalities)
        if "activity_id" not in col_index:
            raise ValueError("activity_id column missing from tensor shards.")
        self.activity_col = col_index["activity_id"]
        # the manifest's row counts define the chunking (as in the reference); the table
        # holds each shard's first `rows` rows
        self.shard_rows = [r for _, r in entries]
        datas = []
        for (path, rows), pl in zip(entries, payloads):
            if list(pl["columns"]) != columns:
                raise ValueError(f"Shard {path} has different columns than {entries[0][0]}")
            d = pl["data"]
            if d.shape[0] < rows:
                raise ValueError(f"Shard {path} has {d.shape[0]} rows, manifest says {rows}")
            datas.append(d[:rows].float())
        self.shard_offsets = [0]
        for r in self.shard_rows:
            self.shard_offsets.append(self.shard_offsets[-1] + r)
        self.table = torch.cat(datas, dim=0).contiguous().to(self.device)
        self.ncols = self.table.shape[1]
        self.chunks = build_chunks(self.shard_rows, chunk_size)
        row0 = [self.shard_offsets[s] + a for s, a, _ in self.chunks]
        lens = [b - a for _, a, b in self.chunks]
        self.chunk_row0 = torch.tensor(row0, dtype=torch.int64, device=self.device)
        self.chunk_len = torch.tensor(lens, dtype=torch.int32, device=self.device)
        self.max_len = max(lens)
        cols: List[int] = []
        self.col_offsets = [0]
        for m in self.modalities:
            cols += [col_index[c] for c in self.modality_columns[m]]
            self.col_offsets.append(len(cols))
        self.cols = torch.tensor(cols, dtype=torch.int32, device=self.device)
        self.modality_dims = {m: len(self.modality_columns[m]) for m in self.modalities}

    def __len__(self) -> int:
        return len(self.chunks)

    def gather(self, chunk_ids: torch.Tensor, T: Optional[int] = None, check_labels: bool = True):
        """Batch of chunk windows: ({m: (B, T, c_m)}, labels (B,) int64, lengths (B,) int32).

        T defaults to the longest chunk of the split; shorter chunks are zero-padded."""
        _nat.require_device(self.table, "manifest table")
        ids = chunk_ids.to(device=self.device, dtype=torch.int64)
        B = int(ids.numel())
        T = int(T or self.max_len)
        row0 = self.chunk_row0.index_select(0, ids).contiguous()
        lens = self.chunk_len.index_select(0, ids).contiguous()
        if B and int(lens.max()) > T:
            raise ValueError(f"chunk longer than T={T}")
        feats = {m: torch.empty(B, T, self.modality_dims[m], dtype=torch.float32, device=self.device)
                 for m in self.modalities}
        labels = torch.empty(B, dtype=torch.int64, device=self.device)
        mismatch = torch.zeros(1, dtype=torch.int32, device=self.device)
        offs = (ctypes.c_int32 * len(self.col_offsets))(*self.col_offsets)
        outs = _nat.ptr_array([feats[m].data_ptr() for m in self.modalities])
        rc = _nat.lib().mmf_gather_chunks(
            self.table.data_ptr(), self.table.shape[0], self.ncols, row0.data_ptr(), lens.data_ptr(), B, T,
            len(self.modalities), self.cols.data_ptr(), ctypes.cast(offs, ctypes.c_void_p),
            ctypes.cast(outs, ctypes.c_void_p), self.activity_col, labels.data_ptr(), mismatch.data_ptr(),
            _nat.stream_ptr(self.device))
        _nat.check(rc, "manifest gather")
        if check_labels and B and int(mismatch.item()) != 0:
            raise ValueError("Activity id varies within shard chunk.")
        return feats, labels, lens

    def modality_mask(self, B: int, generator: Optional[torch.Generator] = None) -> torch.Tensor:
        """(B, M) availability mask with the reference's modality dropout (src/data.py:318-341):
        each modality kept with prob 1 - modality_dropout, and one random modality forced on
        when a row would otherwise be empty."""
        M = len(self.modalities)
        mask = torch.ones(B, M, device=self.device)
        if self.modality_dropout > 0:
            keep = (torch.rand(B, M, generator=generator, device=self.device) > self.modality_dropout).float()
            empty = keep.sum(dim=1) == 0
            pick = torch.randint(0, M, (B,), generator=generator, device=self.device)
            keep[empty, pick[empty]] = 1.0
            mask = mask * keep
        return mask

    def __getitem__(self, idx: int):
        """Reference-compatible single sample: ({m: (1, T_i, c_m)}, label (1,), mask (1, M))."""
        feats, labels, lens = self.gather(torch.tensor([idx]), T=self.chunks[idx][2] - self.chunks[idx][1])
        return feats, labels, self.modality_mask(1)

    def rank_chunk_ids(self, rank: int = 0, world: int = 1, shuffle: bool = False, seed: int = 0,
                       epoch: int = 0) -> List[int]:
        """The chunks rank `rank` of `world` data-parallel ranks visits in one epoch: torch's
        DistributedSampler partition of the split's chunk list (harness.shard_indices).  The
        manifest loader's batch is one chunk (src/data.py:560-566), so each rank takes every
        world-th chunk of the (shuffled) list and all ranks run ceil(n / world) steps."""
        from harness import shard_indices
        return shard_indices(len(self.chunks), rank, world, shuffle=shuffle, seed=seed, epoch=epoch)

    def batches(self, batch_size: int, shuffle: bool = False, generator: Optional[torch.Generator] = None,
                drop_last: bool = False, rank: int = 0, world: int = 1, seed: int = 0, epoch: int = 0):
        """Iterate ({m: (B, T, c_m)}, labels, mask, lengths) batches over every chunk of the split
        (world > 1: over this rank's shard of the chunks, rank_chunk_ids)."""
        if world > 1:
            order = torch.tensor(self.rank_chunk_ids(rank, world, shuffle, seed, epoch), dtype=torch.int64)
        else:
            n = len(self.chunks)
            order = torch.randperm(n, generator=generator) if shuffle else torch.arange(n)
        n = int(order.numel())
        for i in range(0, n, batch_size):
            ids = order[i:i + batch_size]
            if drop_last and ids.numel() < batch_size:
                break
            feats, labels, lens = self.gather(ids)
            yield feats, labels, self.modality_mask(int(ids.numel())), lens
