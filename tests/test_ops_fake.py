"""Fake (meta) kernels of the torch.library operators, on the CPU (mmf_ops.py).

torch.compile traces the drop-in modules with fake tensors: every operator's
``register_fake`` must give the shapes, dtypes and devices the HIP implementation
returns, without touching a device.  Under ``FakeTensorMode`` with fake "cuda" tensors
(no GPU needed) the modules' forwards run end to end through the fake kernels, and each
backward operator is called with the forward's fake outputs; the shapes are checked
against the reference's contract (src/fusion.py:331-427, src/attention.py:68-146,
src/encoders.py:135-166, 313-336).  The numbers these operators compute are covered by
the GPU tests (test_gpu_compile.py runs the same graphs compiled on the device).
"""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode


@pytest.fixture(scope="module")
def mods(pkg_on_path):
    import attention
    import encoders
    import fusion
    import mmf_ops
    return fusion, attention, encoders, mmf_ops


DIMS = {"imu_hand": 24, "imu_chest": 32, "heart_rate": 16}


@pytest.mark.parametrize("seq", [16, 1], ids=["seq16", "l1"])
@pytest.mark.parametrize("hidden,heads", [(32, 4), (256, 2)], ids=["h32", "hd128"])
def test_hybrid_fake_forward_and_backward_shapes(mods, seq, hidden, heads):
    fusion, _, _, mmf_ops = mods
    B, C = 4, 5
    with FakeTensorMode(), torch.device("cuda"):
        m = fusion.HybridFusion(dict(DIMS), hidden_dim=hidden, num_classes=C, num_heads=heads, dropout=0.1).train()
        shape = (lambda d: (B, seq, d)) if seq > 1 else (lambda d: (B, d))
        feats = {k: torch.randn(*shape(d), requires_grad=True) for k, d in DIMS.items()}
        mask = torch.ones(B, len(DIMS))
        logits, info = m(feats, mask, return_attention=True)
        assert logits.shape == (B, C) and logits.device.type == "cuda" and logits.dtype == torch.float32
        assert info["fusion_weights"].shape == (B, len(DIMS))
        names = list(DIMS)
        want = {f"{a}_to_{b}" for a in names for b in names if a != b}
        assert set(info["attention_maps"]) == want
        for v in info["attention_maps"].values():
            assert v.shape == (B, heads, seq, seq)
        # the backward operator on the forward's fake outputs
        params = [p for _, p in m.named_parameters()]
        offsets, nelem = mmf_ops.flat_offsets([p.numel() for p in params])
        assert all(o % mmf_ops.ALIGN == 0 for o in offsets) and nelem >= sum(p.numel() for p in params)
        pairs = [(q, k) for q in range(3) for k in range(3) if q != k]
        idesc = mmf_ops.hybrid_idesc(B, hidden, heads, C, [seq] * 3, list(DIMS.values()), pairs, True, False, 0)
        xs = [feats[k] for k in names]
        _, _, saved, rng_next, maps = torch.ops.mmfusion.hybrid_fwd(idesc, 0.1, m._rng_state, mask, xs, params)
        assert saved.dtype == torch.uint8 and saved.numel() > 0 and maps == []
        assert rng_next.shape == m._rng_state.shape and rng_next.dtype == torch.int64
        dxs, flat = torch.ops.mmfusion.hybrid_bwd(idesc, 0.1, mask, xs, params, saved, torch.randn(B, C),
                                                  [True, False, True], offsets, nelem)
        assert [tuple(t.shape) for t in dxs] == [tuple(xs[0].shape), (0,), tuple(xs[2].shape)]
        assert flat.shape == (nelem,)
        for v, p in zip(mmf_ops._views(flat, params, offsets), params):
            assert v.shape == p.shape


@pytest.mark.parametrize("lq,lk,mask_kind", [(8, 5, None), (1, 1, "1d"), (8, 12, "2d")])
def test_cma_fake_forward_and_backward_shapes(mods, lq, lk, mask_kind):
    _, attention, _, mmf_ops = mods
    B, dq, dk, H, h = 3, 24, 32, 64, 4
    with FakeTensorMode(), torch.device("cuda"):
        c = attention.CrossModalAttention(dq, dk, hidden_dim=H, num_heads=h, dropout=0.1).train()
        q = torch.randn(B, lq, dq, requires_grad=True)
        k = torch.randn(B, lk, dk, requires_grad=True)
        mask = None if mask_kind is None else (torch.ones(B) if mask_kind == "1d" else torch.ones(B, lk))
        att, w = c(q, k, k, mask)
        assert att.shape == (B, lq, H) and w.shape == (B, h, lq, lk)
        params = [p for _, p in c.named_parameters()]
        mode = {None: 0, "1d": 1, "2d": 2}[mask_kind]
        idesc = [B, lq, lk, dq, dk, H, h, mode, 1, 0]
        att2, w2, saved, rng_next = torch.ops.mmfusion.cma_fwd(idesc, 0.1, c._rng_state, q, k, k, mask, params)
        assert att2.shape == att.shape and w2.shape == w.shape and saved.dtype == torch.uint8
        offsets, nelem = mmf_ops.flat_offsets([p.numel() for p in params])
        dq_, dk_, dv_, flat = torch.ops.mmfusion.cma_bwd(idesc, 0.1, q, k, k, mask, params, saved,
                                                        torch.randn(B, lq, H), [True, True, False], offsets, nelem)
        assert dq_.shape == q.shape and dk_.shape == k.shape and dv_.numel() == 0 and flat.shape == (nelem,)


def test_encoder_and_weighting_fake_shapes(mods):
    fusion, _, encoders, _ = mods
    with FakeTensorMode(), torch.device("cuda"):
        seq = encoders.SequenceEncoder(17, hidden_dim=64, output_dim=32, num_layers=2, dropout=0.0)
        assert seq(torch.randn(3, 20, 17)).shape == (3, 32)
        hs, cs, gates, flag = torch.ops.mmfusion.lstm_layer_fwd([torch.randn(3, 20, 256)] * 2, [torch.randn(256, 64)] * 2)
        assert [t.shape for t in hs] == [(3, 20, 64)] * 2 and [t.shape for t in gates] == [(3, 20, 256)] * 2
        assert flag.dtype == torch.int32
        dg, flag = torch.ops.mmfusion.lstm_layer_bwd([torch.randn(256, 64)] * 2, cs, gates, hs)
        assert [t.shape for t in dg] == [(3, 20, 256)] * 2
        frame = encoders.FrameEncoder(48, hidden_dim=32, output_dim=16, dropout=0.0)
        assert frame(torch.randn(3, 9, 48), torch.ones(3, 9)).shape == (3, 16)
        pooled, wts = torch.ops.mmfusion.attention_pool_fwd(torch.randn(3, 9, 32), torch.randn(1, 32),
                                                            torch.randn(1), None)
        assert pooled.shape == (3, 32) and wts.shape == (3, 9)
        dx, dw, db = torch.ops.mmfusion.attention_pool_bwd(torch.randn(3, 9, 32), torch.randn(1, 32), wts, pooled)
        assert dx.shape == (3, 9, 32) and dw.shape == (32,) and db.shape == (1,)
        fused, w = torch.ops.mmfusion.late_weights_fwd(torch.randn(4, 3, 5), torch.randn(3), torch.ones(4, 3))
        assert fused.shape == (4, 5) and w.shape == (4, 3)
        ds, dwl = torch.ops.mmfusion.late_weights_bwd(torch.randn(4, 3, 5), torch.randn(3), torch.ones(4, 3), w, fused)
        assert ds.shape == (4, 3, 5) and dwl.shape == (3,)
        m = fusion.HybridFusion(dict(DIMS), hidden_dim=32, num_classes=5, num_heads=4)
        pooled = {k: torch.randn(4, 32) for k in DIMS}
        assert m.compute_adaptive_weights(pooled, torch.ones(4, 3)).shape == (4, 3)
