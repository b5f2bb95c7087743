"""Module-path data parallelism (harness.py) and the bench launcher, on the CPU.

* ``shard_indices`` is torch's DistributedSampler partition (the PAMAP2 chunk list is
  sharded with it: the manifest loader's batch is one chunk, src/data.py:560-566).
* ``FlatGradBuckets`` over an encoder + fusion model, world size 2 on gloo: each rank
  back-propagates its shard, the fusion bucket is all-reduced from the post-accumulate
  hooks while the encoders' backward is still running, the encoder bucket after; the
  rank average of the flat gradient equals the single-process full-batch gradient
  (SURVEY §8e).  The fusion model is the oracle's HybridFusion restatement (CPU test
  infrastructure; the HIP fusion has no CPU path) and the encoders are torch LSTMs --
  the gradient exchange is what is under test.  Gradient accumulation over two
  micro-batches exchanges once and equals the sum of the micro-batch gradients.
* ``bench.py --gpus N``: the torch.distributed.run child command and the strong-scaling
  batch split (global 256 -> 128 / 64 / 32 per GPU).
"""
from __future__ import annotations

import os
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn
import torch.nn.functional as F

from test_dp import PKG, ROOT, _free_port, _setup

B, T, FEAT, OUT, HID, HEADS, C = 8, 12, 5, 16, 16, 2, 4
NAMES = ["imu_hand", "imu_chest", "heart_rate"]


def _pkg():
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)


class _OracleFusion(nn.Module):
    """HybridFusion's parameters (reference names) around the oracle's forward (CPU)."""

    def __init__(self):
        super().__init__()
        _pkg()
        from fusion import HybridFusion
        torch.manual_seed(5)
        ref = HybridFusion({m: OUT for m in NAMES}, hidden_dim=HID, num_classes=C, num_heads=HEADS, dropout=0.0)
        self.keys = list(ref.state_dict().keys())
        self.p = nn.ParameterList([nn.Parameter(v.detach().clone()) for v in ref.state_dict().values()])

    def forward(self, feats, mask=None):
        from oracle.hybrid_cpu import hybrid_forward
        if mask is None:
            mask = torch.ones(next(iter(feats.values())).size(0), len(NAMES))
        logits, _ = hybrid_forward(dict(zip(self.keys, self.p)), NAMES, feats, mask, HEADS)
        return logits


class _LstmEncoder(nn.Module):
    def __init__(self, in_dim):
        super().__init__()
        self.rnn = nn.LSTM(in_dim, 16, batch_first=True)
        self.projection = nn.Linear(16, OUT)

    def forward(self, x):
        _, (h, _) = self.rnn(x)
        return self.projection(h[-1])


def _model():
    _pkg()
    from harness import MultimodalFusionModel
    torch.manual_seed(7)
    encs = {m: _LstmEncoder(FEAT if m != "heart_rate" else 1) for m in NAMES}
    return MultimodalFusionModel(encs, _OracleFusion(), OUT, layer_norm=True)


def _batch(seed=3, n=B):
    g = torch.Generator().manual_seed(seed)
    feats = {m: torch.randn(n, T, FEAT if m != "heart_rate" else 1, generator=g) for m in NAMES}
    mask = torch.ones(n, len(NAMES))
    mask[2, 1] = 0.0
    labels = torch.randint(0, C, (n,), generator=g)
    return feats, mask, labels


def _loss(model, feats, mask, labels):
    return F.cross_entropy(model(feats, mask), labels, label_smoothing=0.05)


def _rank(rank: int, world: int, port: int, out: str) -> None:
    _setup(rank, world, port)
    try:
        from harness import FlatGradBuckets, shard_indices
        model = _model()
        fb = FlatGradBuckets([list(model.fusion_model.parameters()),
                              [p for n, p in model.named_parameters() if not n.startswith("fusion_model.")]],
                             dist.group.WORLD)
        feats, mask, labels = _batch()
        idx = shard_indices(B, rank, world)
        sf = {m: f[idx] for m, f in feats.items()}
        # two micro-batches (accumulation): only the last one exchanges
        half = len(idx) // 2
        for mb, sync in ((slice(0, half), False), (slice(half, None), True)):
            if sync:
                fb.arm()
            loss = _loss(model, {m: f[mb] for m, f in sf.items()}, mask[idx][mb], labels[idx][mb])
            (loss / 2).backward()
        hooked = [w is not None for w in fb._works]
        fb.finish()
        if rank == 0:
            torch.save({"dp": fb.grad / world, "hooked": hooked, "spans": fb.spans}, out)
    finally:
        dist.destroy_process_group()


def test_flat_buckets_encoder_fusion_gloo_matches_full_batch(tmp_path):
    out = str(tmp_path / "dp.pt")
    mp.spawn(_rank, args=(2, _free_port(), out), nprocs=2, join=True)
    r = torch.load(out, weights_only=True)
    # both buckets were issued by the hooks during the backward (nothing left for finish())
    assert r["hooked"] == [True, True]
    # single process: the same accumulation over the whole batch (each rank's two
    # micro-batches of B/4 => 4 micro-batches of the global batch, loss / 2 each, / world)
    _pkg()
    from harness import FlatGradBuckets, shard_indices
    model = _model()
    fb = FlatGradBuckets([list(model.fusion_model.parameters()),
                          [p for n, p in model.named_parameters() if not n.startswith("fusion_model.")]])
    feats, mask, labels = _batch()
    for rank in range(2):
        idx = shard_indices(B, rank, 2)
        half = len(idx) // 2
        for mb in (slice(0, half), slice(half, None)):
            loss = _loss(model, {m: f[idx][mb] for m, f in feats.items()}, mask[idx][mb], labels[idx][mb])
            (loss / 4).backward()
    fb.finish()      # (unarmed: gathers the accumulated .grad tensors into the flat gradient)
    full = fb.grad
    assert r["spans"] == fb.spans
    enc0 = fb.spans[1][0]
    assert full[:enc0].abs().max() > 0 and full[enc0:].abs().max() > 0   # fusion and encoder buckets live
    err = (r["dp"] - full).abs().max() / full.abs().max()
    assert err <= 1e-5, float(err)


def test_flat_buckets_views_and_layout():
    _pkg()
    from harness import FlatGradBuckets
    model = _model()
    fb = FlatGradBuckets([list(model.fusion_model.parameters()), list(model.encoders.parameters())])
    for p in model.fusion_model.parameters():
        assert p.data.data_ptr() >= fb.flat.data_ptr()
        assert (p.data.data_ptr() - fb.flat.data_ptr()) % 256 == 0          # 256-byte aligned tensors
        assert p.grad is None                                                 # set-to-none gradients
    feats, mask, labels = _batch()
    _loss(model, feats, mask, labels).backward()
    want = [p.grad.clone() for p in fb.params]
    fb.finish()            # unarmed: gather (a copy into the fresh flat gradient), .grad -> None
    assert all(p.grad is None for p in fb.params)
    it = iter(want)
    for views in fb._gviews:
        for v in views:
            assert torch.equal(v, next(it))
    assert fb.grad.abs().sum() > 0
    # a second backward without zero_grad accumulates (an add into the flat gradient)
    _loss(model, feats, mask, labels).backward()
    fb.gather()
    it = iter(want)
    for views in fb._gviews:
        for v in views:
            assert torch.allclose(v, 2 * next(it), rtol=1e-6, atol=1e-7)
    # after zero_grad the next gather copies; a parameter without a gradient reads zero
    fb.zero_grad()
    fb.params[0].grad = torch.ones_like(fb.params[0])
    fb.gather()
    assert torch.equal(fb._gviews[0][0], torch.ones_like(fb.params[0]))
    assert fb.grad[fb.params[0].numel():].abs().sum() == 0
    with pytest.raises(ValueError):
        FlatGradBuckets([[]])


@pytest.mark.parametrize("n,world", [(44, 2), (44, 4), (216, 8), (7, 3), (1, 2), (216, 1)])
@pytest.mark.parametrize("shuffle", [False, True])
def test_shard_indices_matches_distributed_sampler(n, world, shuffle):
    _pkg()
    from harness import shard_indices
    from torch.utils.data import DistributedSampler
    data = list(range(n))
    covered = set()
    for rank in range(world):
        s = DistributedSampler(data, num_replicas=world, rank=rank, shuffle=shuffle, seed=17)
        s.set_epoch(3)
        got = shard_indices(n, rank, world, shuffle=shuffle, seed=17, epoch=3)
        assert got == list(iter(s))
        covered.update(got)
    assert covered == set(data)
    with pytest.raises(ValueError):
        shard_indices(4, 2, 2)


def test_bench_launcher_and_strong_split():
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.launcher_command(8, ["--gpus", "8", "--steps", "20"], 29511, script="/x/bench.py")
    assert cmd[1:] == ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8", "--master-addr=127.0.0.1",
                       "--master-port=29511", "/x/bench.py", "--gpus", "8", "--steps", "20"]
    w = bench.WORKLOADS["c2"]
    assert [bench.rank_batch(w, "strong", n) for n in (1, 2, 4, 8)] == [256, 128, 64, 32]
    assert [bench.rank_batch(w, "weak", n) for n in (1, 2, 4, 8)] == [256] * 4
    assert bench.rank_batch(bench.WORKLOADS["c5"], "strong", 8) == 128
    with pytest.raises(ValueError):
        bench.rank_batch(w, "strong", 3)
    assert 1024 < bench.free_port() < 65536


def test_bench_gpus_mismatch_refused(monkeypatch):
    """Under a launcher, --gpus must equal WORLD_SIZE (checked before any GPU call)."""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.main(["--gpus", "4"])


def test_model_from_base_config_keys():
    """MultimodalFusionModel.from_config builds config/base.yaml's PAMAP2 model (the keys of
    src/train.py:150-182): four LSTM SequenceEncoders, LayerNorms, HybridFusion H=256, h=4."""
    _pkg()
    from harness import MultimodalFusionModel
    enc = {m: {"type": "sequence", "input_dim": 17 if m != "heart_rate" else 1, "encoder_type": "lstm",
               "num_layers": 1} for m in ("imu_hand", "imu_chest", "imu_ankle", "heart_rate")}
    cfg = {"dataset": {"modalities": list(enc), "num_classes": 25},
           "model": {"fusion_type": "hybrid", "hidden_dim": 256, "output_dim": 128, "num_heads": 4,
                     "dropout": 0.1, "layer_norm": True, "encoders": enc}}
    m = MultimodalFusionModel.from_config(cfg)
    assert list(m.encoders) == list(enc) and list(m.layer_norms) == list(enc)
    assert m.fusion_model.hidden_dim == 256 and m.fusion_model.num_heads == 4
    assert m.encoders["heart_rate"].rnn.input_size == 1
    keys = set(m.state_dict())
    assert "fusion_model.attention_modules.imu_hand_to_heart_rate.query_proj.weight" in keys
    assert "encoders.imu_chest.rnn.weight_hh_l0" in keys and "layer_norms.imu_ankle.weight" in keys
    cfg["dataset"]["modalities"] = ["mystery"]
    with pytest.raises(NotImplementedError):
        MultimodalFusionModel.from_config(cfg)




def test_direct_grad_reads_the_operator_buffer_in_place():
    """FlatGradBuckets.direct_grad (one process, one bucket): when every parameter's .grad is a
    view of one buffer at this buffer's offsets -- what the HIP operators return (mmf_ops
    flat_offsets: the same 256-byte alignment; HybridFusion's operator order is its registration
    order) -- the optimizer reads that buffer in place; any other layout, a missing gradient or two
    buckets fall back to the gather."""
    _pkg()
    import mmf_ops
    from fusion import HybridFusion
    from harness import FlatGradBuckets
    torch.manual_seed(0)
    model = HybridFusion({m: OUT for m in NAMES}, hidden_dim=HID, num_classes=C, num_heads=HEADS, dropout=0.0)
    params = [p for p in model.parameters()]
    names = [n for n, _ in model.named_parameters()]
    pairs = model.present_pairs()
    assert names == model._param_names(pairs)   # the operator's order is the registration order
    fb = FlatGradBuckets([params])
    offs, n = mmf_ops.flat_offsets([p.numel() for p in params])
    assert n == fb.numel
    src = torch.zeros(n + 64)[32:]            # (a storage offset of its own, as a pooled output has)
    src.normal_()
    for p, o in zip(params, offs):
        p.grad = src[o:o + p.numel()].view_as(p)
    d = fb.direct_grad()
    assert d is not None and d.data_ptr() == src.data_ptr() and d.numel() == fb.numel
    params[3].grad = params[3].grad.clone()   # one gradient elsewhere
    assert fb.direct_grad() is None
    params[3].grad = None
    assert fb.direct_grad() is None
    fb2 = FlatGradBuckets([params[:4], params[4:]])
    for p, o in zip(params, offs):
        p.grad = src[o:o + p.numel()].view_as(p)
    assert fb2.direct_grad() is None          # (two buckets: gathered)
