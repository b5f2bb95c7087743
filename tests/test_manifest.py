"""Manifest data path: the package's manifest.py host logic
and the HIP chunk gather (mmf_gather_chunks) against the reference's
MultimodalDataset outputs (tests/golden/manifest_pamap2.npz, made by
tests/golden/gen_manifest.py from two sliced PAMAP2 shards) and the CPU oracle.
The gather is pure data movement: results are compared bit-exactly."""
import numpy as np
import pytest
import torch

from _util import load_fixture

MODALITIES = ["imu_hand", "imu_chest", "imu_ankle", "heart_rate"]
CHUNK = 64


@pytest.fixture(scope="module")
def man(pkg_on_path):
    import manifest
    return manifest


def _write_split(tmp_path, fx, extra_lines=()):
    root = tmp_path / "a" / "b"
    (root / "splits").mkdir(parents=True)
    cols = [str(c) for c in fx["columns"]]
    lines = []
    for i in range(2):
        d = torch.from_numpy(fx[f"shard{i}/data"])
        path = tmp_path / f"shard{i}.pt"
        torch.save({"columns": cols, "data": d}, path)
        lines.append(f"{path},{d.shape[0]}")
    lines[1:1] = list(extra_lines)
    (root / "splits" / "test.txt").write_text("\n".join(lines) + "\n")
    return root, cols


def test_oracle_matches_reference_dataset(tmp_path):
    from oracle.manifest_cpu import chunk_windows, gather_chunk
    fx = load_fixture("manifest_pamap2")
    cols = [str(c) for c in fx["columns"]]
    shards = [fx["shard0/data"], fx["shard1/data"]]
    chunks = chunk_windows([s.shape[0] for s in shards], CHUNK)
    assert np.array_equal(np.array(chunks), fx["chunks"])
    sel = {"imu_hand": [i for i, c in enumerate(cols) if c.startswith("hand_")],
           "imu_chest": [i for i, c in enumerate(cols) if c.startswith("chest_")],
           "imu_ankle": [i for i, c in enumerate(cols) if c.startswith("ankle_")],
           "heart_rate": [cols.index("heart_rate_bpm")]}
    for idx, ch in enumerate(chunks):
        feats, label = gather_chunk(shards, ch, sel, cols.index("activity_id"))
        assert label == int(fx[f"chunk{idx}/label"][0])
        for m in MODALITIES:
            assert np.array_equal(feats[m], fx[f"chunk{idx}/{m}"]), (idx, m)


def test_host_logic_matches_reference(man, tmp_path):
    fx = load_fixture("manifest_pamap2")
    root, cols = _write_split(tmp_path, fx, ["ignored.pt,0"])
    entries = man.parse_manifest(root / "splits" / "test.txt")
    assert [r for _, r in entries] == [150, 100]
    mapping = man.resolve_modality_columns(cols, MODALITIES)
    assert mapping["heart_rate"] == ["heart_rate_bpm"] and len(mapping["imu_hand"]) == 17
    assert np.array_equal(np.array(man.build_chunks([150, 100], CHUNK)), fx["chunks"])
    # the reference's suffix form and errors (tests/test_data.py:306-393 of the reference)
    assert man.resolve_modality_columns(cols, ["chest_imu"])["chest_imu"][0] == "chest_temp_c"
    with pytest.raises(ValueError, match="Could not resolve modality"):
        man.resolve_modality_columns(cols, ["video"])
    bad = tmp_path / "x" / "y" / "z"
    (bad / "splits").mkdir(parents=True)
    (bad / "splits" / "test.txt").write_text("missing_comma_entry\n")
    with pytest.raises(ValueError, match="Malformed manifest entry"):
        man.parse_manifest(bad / "splits" / "test.txt")
    (bad / "splits" / "test.txt").write_text("ghost.pt,2\n")
    with pytest.raises(FileNotFoundError, match="Shard referenced in manifest not found"):
        man.parse_manifest(bad / "splits" / "test.txt")
    (bad / "splits" / "test.txt").write_text("ignored.pt,0\n")
    with pytest.raises(ValueError, match="No shards found in manifest"):
        man.parse_manifest(bad / "splits" / "test.txt")


def test_rank_sharding_of_chunks(man, tmp_path):
    """DP over the PAMAP2 chunk list (one chunk per rank per step): every rank gets
    ceil(n / world) chunks (DistributedSampler's wrap padding), together they cover the split."""
    fx = load_fixture("manifest_pamap2")
    root, _ = _write_split(tmp_path, fx)
    ds = man.ManifestShards(root, "test", MODALITIES, chunk_size=CHUNK, device="cpu")
    n = len(ds)
    assert n == 5
    for world in (1, 2, 4):
        parts = [ds.rank_chunk_ids(r, world, shuffle=True, seed=42, epoch=1) for r in range(world)]
        assert all(len(p) == -(-n // world) for p in parts)
        assert set(i for p in parts for i in p) == set(range(n))
    # epochs reshuffle, the same epoch is reproducible
    assert ds.rank_chunk_ids(0, 2, True, 42, 1) == ds.rank_chunk_ids(0, 2, True, 42, 1)
    assert ds.rank_chunk_ids(0, 2, True, 42, 1) != ds.rank_chunk_ids(0, 2, True, 42, 2) or n < 3


@pytest.mark.gpu
def test_gpu_gather_matches_reference(man, tmp_path):
    fx = load_fixture("manifest_pamap2")
    root, _ = _write_split(tmp_path, fx, ["ignored.pt,0"])
    ds = man.ManifestShards(root, "test", MODALITIES, chunk_size=CHUNK, device="cuda")
    assert len(ds) == len(fx["chunks"])
    feats, labels, lens = ds.gather(torch.arange(len(ds)))
    assert feats["imu_hand"].shape == (len(ds), CHUNK, 17)
    for idx in range(len(ds)):
        n = int(lens[idx])
        assert labels[idx].item() == int(fx[f"chunk{idx}/label"][0])
        for m in MODALITIES:
            got = feats[m][idx].cpu().numpy()
            assert np.array_equal(got[:n][None], fx[f"chunk{idx}/{m}"]), (idx, m)
            assert not got[n:].any()          # zero padding past the chunk
    # reference-compatible single sample, ragged last chunk
    f2, lab2, mask2 = ds[2]
    assert f2["heart_rate"].shape == (1, 22, 1) and lab2.item() == 12 and mask2.shape == (1, 4)
    assert np.array_equal(f2["imu_ankle"].cpu().numpy(), fx["chunk2/imu_ankle"])
    # batch iteration covers every chunk once
    seen = sum(int(b[1].numel()) for b in ds.batches(2, shuffle=True, generator=torch.Generator().manual_seed(0)))
    assert seen == len(ds)


@pytest.mark.gpu
def test_gpu_gather_label_check_and_dropout(man, tmp_path):
    fx = load_fixture("manifest_pamap2")
    d0 = fx["shard0/data"].copy()
    cols = [str(c) for c in fx["columns"]]
    d0[10, cols.index("activity_id")] = 99.0          # activity id varies within chunk 0
    fx2 = dict(fx)
    fx2["shard0/data"] = d0
    root, _ = _write_split(tmp_path, fx2)
    ds = man.ManifestShards(root, "test", MODALITIES, chunk_size=CHUNK, modality_dropout=0.9, device="cuda")
    with pytest.raises(ValueError, match="Activity id varies within shard chunk"):
        ds.gather(torch.tensor([0, 1]))
    ds.gather(torch.tensor([1, 3]))                   # the other chunks are fine
    mask = ds.modality_mask(4096)
    assert (mask.sum(dim=1) >= 1).all() and mask.mean() < 0.5
