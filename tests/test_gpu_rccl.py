"""RCCL (torch.distributed backend "nccl") executing the fused step's exchange on the one-GPU box.

The driver's 8-GPU scaling run is the first place several MI355X ranks meet; this pool gives one
card per call, and RCCL refuses two ranks on one device.  What can run here is the real RCCL path
at world size 1: the process group over RCCL, HybridTrainStep's overlapped exchange
(``overlap=True``: part 1 of the train step, the async all-reduce of its bucket on RCCL's stream
while part 2 runs, then the projections' bucket, wait, clip + AdamW), eager and as two captured
graphs.  A one-rank all-reduce is the identity, so the step must give the single-process step's
gradient (to the split-K summation order the two parts change) and, after the update, its weights.
"""
from __future__ import annotations

import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_dp import B, C, D, HEADS, H, L, M, PKG, ROOT, _free_port, _global_batch, _model

pytestmark = pytest.mark.gpu


def _rank(rank: int, port: int, out: str) -> None:
    import sys
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=1, device_id=dev)
    try:
        from train_step import HybridTrainStep, allreduce_flat
        assert dist.get_backend() == "nccl"
        feats, mask, labels = _global_batch()
        # a bare RCCL all-reduce of one rank
        t = torch.arange(1000, dtype=torch.float32, device=dev)
        dist.all_reduce(t)
        torch.cuda.synchronize()
        assert torch.equal(t.cpu(), torch.arange(1000, dtype=torch.float32))
        ref = HybridTrainStep(_model().to(dev), [f.to(dev) for f in feats], mask.to(dev), labels.to(dev))
        ref.forward_backward()
        ref.optimizer_step()
        torch.cuda.synchronize()
        res = {"ref_grad": ref.grad.cpu(), "ref_flat": ref.flat.cpu()}
        for graph in (False, True):
            st = HybridTrainStep(_model().to(dev), [f.to(dev) for f in feats], mask.to(dev), labels.to(dev),
                                 process_group=dist.group.WORLD, overlap=True)
            assert st.overlap and not st.fuse_clip
            if graph:
                st.capture()
            st.step()
            torch.cuda.synchronize()
            res[f"grad_{graph}"] = st.grad.cpu()
            res[f"flat_{graph}"] = st.flat.cpu()
            allreduce_flat(st.grad, dist.group.WORLD, 2)   # (the helper's collective on RCCL)
            torch.cuda.synchronize()
        torch.save(res, out)
    finally:
        dist.destroy_process_group()


def test_rccl_overlapped_exchange_one_rank():
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "rccl.pt")
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        mp.spawn(_rank, args=(_free_port(), out), nprocs=1, join=True)
        r = torch.load(out, weights_only=True)
    g, f = r["ref_grad"], r["ref_flat"]
    # (AdamW's first step moves a weight by ~lr sign(g): where g is rounding noise -- key_proj.bias,
    # mathematically zero -- the two summation orders may flip its sign; the weights are compared
    # where the gradient is not noise)
    sig = g.abs() > 1e-4 * g.abs().max()
    for graph in (False, True):
        assert (r[f"grad_{graph}"] - g).abs().max() <= 1e-5 * g.abs().max(), graph
        fg = r[f"flat_{graph}"]
        assert torch.isfinite(fg).all()
        assert (fg - f)[sig].abs().max() <= 1e-5 * f.abs().max(), graph
