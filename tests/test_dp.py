"""Data-parallel path: world_size-2 runs over torch.distributed.

The one exchange of DP training is the all-reduce of the flat gradient
(train_step.allreduce_flat); samples are independent, so the average of the
ranks' gradients on equal shards must equal the full-batch gradient up to
summation order.

* CPU (gloo): the sharding, flat-gradient layout (the plan's parameter order)
  and the collective, with per-rank gradients from the oracle.
* GPU (gloo, two ranks sharing cuda:0; the box has one GPU, and RCCL refuses
  two ranks on one device): the real HybridTrainStep on each shard through
  the HIP library vs a single-process step on the whole batch.
"""
from __future__ import annotations

import os
import socket
import sys
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "multimodal-sensor-fusion-with-attention-rajeevatla_amd")

M, B, L, D, H, HEADS, C = 3, 8, 6, 16, 16, 2, 5
TOL = 1e-5


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _setup(rank: int, world: int, port: int) -> None:
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _global_batch(seed: int = 11):
    g = torch.Generator().manual_seed(seed)
    feats = [torch.randn(B, L, D, generator=g) for _ in range(M)]
    mask = torch.ones(B, M)
    mask[1, 0] = 0.0
    mask[5, 2] = 0.0
    labels = torch.randint(0, C, (B,), generator=g)
    return feats, mask, labels


def _model():
    from fusion import HybridFusion
    torch.manual_seed(3)
    return HybridFusion({f"m{i}": D for i in range(M)}, hidden_dim=H, num_classes=C, num_heads=HEADS,
                        dropout=0.0)


def _oracle_flat_grad(model, feats, mask, labels) -> torch.Tensor:
    """Oracle fwd+CE+bwd gradient flattened in the kernel plan's parameter order."""
    from oracle.hybrid_cpu import hybrid_train_step
    names = model.modality_names
    params = {k: v.detach().clone().requires_grad_(True) for k, v in model.state_dict().items()}
    fd = {n: f.clone() for n, f in zip(names, feats)}
    hybrid_train_step(params, names, fd, mask, labels, HEADS, 0.0)
    plan = model._plan(feats, False)
    plan.params(model)
    flat = torch.zeros(plan.num_param_elems)
    for n, o in zip(plan.names, plan.offsets):
        g = params[n].grad if params[n].grad is not None else torch.zeros_like(params[n])
        flat[o:o + g.numel()] = g.reshape(-1)
    return flat


def _cpu_rank(rank: int, world: int, port: int, out: str, accumulate: int = 1) -> None:
    _setup(rank, world, port)
    try:
        from train_step import allreduce_flat, shard_batch
        model = _model()
        feats, mask, labels = _global_batch()
        lf, lm, ll = shard_batch(feats, mask, labels, rank, world)
        assert lm.size(0) == B // world
        if accumulate == 1:
            flat = _oracle_flat_grad(model, lf, lm, ll)
        else:
            # Lightning's accumulate_grad_batches (config/base.yaml:75): the shard as `accumulate`
            # equal micro-batches, each loss scaled by 1 / accumulate, gradients summed before the
            # one exchange (what HybridTrainStep's forward_backward does on the device)
            flat = None
            for i in range(accumulate):
                mf, mm, ml = shard_batch(lf, lm, ll, i, accumulate)
                g = _oracle_flat_grad(model, mf, mm, ml) / accumulate
                flat = g if flat is None else flat + g
        allreduce_flat(flat, dist.group.WORLD, world)
        flat /= world
        if rank == 0:
            torch.save({"dp": flat, "full": _oracle_flat_grad(model, feats, mask, labels)}, out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("accumulate", [1, 4])
def test_dp_gloo_cpu_matches_full_batch(tmp_path, accumulate):
    out = str(tmp_path / "dp.pt")
    mp.spawn(_cpu_rank, args=(2, _free_port(), out, accumulate), nprocs=2, join=True)
    r = torch.load(out, weights_only=True)
    err = (r["dp"] - r["full"]).abs().max() / r["full"].abs().max()
    assert err <= TOL, float(err)


def test_cosine_annealing_lr_matches_torch():
    """train_step.cosine_annealing_lr == CosineAnnealingLR(T_max=max_epochs, eta_min=lr/100),
    the reference's scheduler (src/train.py:394-402), stepped per epoch."""
    sys.path.insert(0, PKG)
    from train_step import cosine_annealing_lr
    p = torch.zeros(1, requires_grad=True)
    opt = torch.optim.AdamW([p], lr=1e-3)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=100, eta_min=1e-5)
    for epoch in range(0, 101):
        assert abs(opt.param_groups[0]["lr"] - cosine_annealing_lr(epoch, 1e-3, 100)) <= 1e-12
        opt.step()
        sched.step()


def test_shard_batch_rejects_uneven():
    sys.path.insert(0, PKG)
    from train_step import shard_batch
    feats, mask, labels = _global_batch()
    with pytest.raises(ValueError, match="not divisible"):
        shard_batch(feats, mask[:7], labels[:7], 0, 2)
    with pytest.raises(ValueError, match="bad rank"):
        shard_batch(feats, mask, labels, 2, 2)
    parts = [shard_batch(feats, mask, labels, r, 4) for r in range(4)]
    assert torch.equal(torch.cat([p[1] for p in parts]), mask)
    assert torch.equal(torch.cat([p[0][1] for p in parts]), feats[1])


# ---------------------------------------------------------------------- GPU
def _gpu_rank(rank: int, world: int, port: int, out: str, accumulate: int = 1) -> None:
    _setup(rank, world, port)
    try:
        from train_step import HybridTrainStep, shard_batch
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        feats, mask, labels = _global_batch()
        lf, lm, ll = shard_batch(feats, mask, labels, rank, world)
        model = _model().to(dev)
        seed0 = int(model._rng_state[0].item())
        step = HybridTrainStep(model, [f.to(dev) for f in lf], lm.to(dev), ll.to(dev),
                               process_group=dist.group.WORLD, accumulate=accumulate)
        assert not step.fuse_clip   # (the clip norm is taken after the exchange)
        # every rank starts from the same seed; the step folds the rank into the Philox key of
        # the module's dropout state (once) and advances that buffer itself
        assert int(step.rng[0].item()) == seed0 ^ (rank * 0x9E3779B1)
        assert step.rng.data_ptr() == model._rng_state.data_ptr()
        HybridTrainStep(model, [f.to(dev) for f in lf], lm.to(dev), ll.to(dev), process_group=dist.group.WORLD)
        assert int(model._rng_state[0].item()) == seed0 ^ (rank * 0x9E3779B1)   # not folded twice
        step.forward_backward()
        step.allreduce()
        torch.cuda.synchronize(dev)
        dp = (step.grad / world).cpu()
        # the overlapped exchange of step(): part 1 of the train step, the all-reduce of its bucket
        # (pairs, gates, classifier) issued while part 2 (dZ, dX, the projections' weight gradients)
        # runs, then the projections' bucket -- eager and as two captured graphs
        # overlap=False (one exchange of the whole flat gradient after the backward), eager and
        # captured: the graph holds forward + backward only, step() exchanges and updates after the
        # replay (the captured form once skipped both)
        bucketed, updates = [], []
        for overlap, graph in ((True, False), (True, True), (False, False), (False, True)):
            st = HybridTrainStep(_model().to(dev), [f.to(dev) for f in lf], lm.to(dev), ll.to(dev),
                                 process_group=dist.group.WORLD, accumulate=accumulate, overlap=overlap)
            assert st.overlap == overlap
            if overlap:
                assert st.bucket_spans[0][1] == st.grad.numel() and st.bucket_spans[1][0] == 0
            flat0 = st.flat.clone()
            if graph:
                st.capture()
                assert (st.graph2 is not None) == overlap
            st.step()
            torch.cuda.synchronize(dev)
            bucketed.append((st.grad / world).cpu())
            updates.append((st.flat - flat0).cpu())
            assert int(st.step_dev.item()) == 1
        if rank == 0:
            full_model = _model().to(dev)
            full = HybridTrainStep(full_model, [f.to(dev) for f in feats], mask.to(dev), labels.to(dev))
            full.forward_backward()
            torch.cuda.synchronize(dev)
            torch.save({"dp": dp, "full": full.grad.cpu(), "names": full.plan.names, "bucketed": bucketed,
                        "updates": updates, "oracle": _oracle_flat_grad(_model(), feats, mask, labels)}, out)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("accumulate", [1, 4])
def test_dp_two_ranks_gpu_matches_single_process(accumulate):
    """Two ranks on one card (gloo) through the HIP fused step: each rank's shard of the global batch,
    optionally as `accumulate` micro-batches summed on the device before the one exchange (the
    reference's gradient_accumulation, config/base.yaml:75), equals one process on the whole batch --
    with one all-reduce after the backward, and with step()'s two buckets overlapped with the
    backward; step() with and without the overlap, eager and captured, applies the same update."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "dp_gpu.pt")
        mp.spawn(_gpu_rank, args=(2, _free_port(), out, accumulate), nprocs=2, join=True)
        r = torch.load(out, weights_only=True)
    full, dp, ref = r["full"], r["dp"], r["oracle"]
    assert (dp - full).abs().max() <= 1e-4 * full.abs().max()
    for b in r["bucketed"]:   # (overlapped, whole-buffer) x (eager, captured)
        assert (b - full).abs().max() <= 1e-4 * full.abs().max()
    # every variant updated the weights (the first AdamW step moves a weight by ~lr), and the
    # captured form of each exchange mode applied exactly its eager update
    ups = r["updates"]
    for u in ups:
        assert u.abs().max() > 1e-4
    assert (ups[1] - ups[0]).abs().max() <= 1e-6    # overlapped: eager vs captured
    assert (ups[3] - ups[2]).abs().max() <= 1e-6    # one exchange after the backward: eager vs captured
    # and both agree with the oracle at the parity tolerance
    assert (full - ref).abs().max() <= 1e-3 * ref.abs().max()
