"""HIP masked-softmax weighting ops beside the fused path:
FrameEncoder.attention_pool (src/encoders.py:313-336) and the LateFusion
weighting (src/fusion.py:228-245), against fixtures produced by the reference
(tests/golden/gen_golden.py) and, at larger sizes, against the CPU oracle.
Tolerance: 1e-3 relative (BASELINE.json fp32 parity)."""
import numpy as np
import pytest
import torch

from _util import close, load_fixture, rel_err
from cases import (FRAMEPOOL_CASES, LATE_CASES, framepool_inputs, framepool_state, late_inputs,
                   late_state)

TOL = 1e-3


@pytest.fixture(scope="module")
def enc_mod(pkg_on_path):
    import encoders
    return encoders


@pytest.fixture(scope="module")
def fusion_mod(pkg_on_path):
    import fusion
    return fusion


def test_frame_encoder_surface_cpu(enc_mod):
    """Construction / validation errors of the reference (src/encoders.py:246-247, 275-278, 306-309, 330-331)."""
    with pytest.raises(ValueError, match="Unknown pooling"):
        enc_mod.FrameEncoder(16, 8, 4, temporal_pooling="median")
    e = enc_mod.FrameEncoder(16, 8, 4, temporal_pooling="average")
    with pytest.raises(ValueError, match="Expected 3D frame tensor"):
        e(torch.randn(16))
    with pytest.raises(RuntimeError, match="Attention layer not initialized"):
        e.attention_pool(torch.randn(2, 3, 8))
    e.temporal_pooling = "bogus"
    with pytest.raises(ValueError, match="Unknown pooling strategy"):
        e(torch.randn(2, 3, 16))
    a = enc_mod.FrameEncoder(16, 8, 4)
    assert sorted(a.state_dict()) == sorted(["frame_processor.0.weight", "frame_processor.0.bias",
                                            "attention.weight", "attention.bias", "projection.0.weight",
                                            "projection.0.bias", "projection.3.weight", "projection.3.bias"])
    with pytest.raises(RuntimeError, match="ROCm device"):
        a(torch.randn(2, 3, 16))


def test_late_fusion_requires_device_cpu(fusion_mod):
    late = fusion_mod.build_fusion_model("late", {"a": 4, "b": 4}, num_classes=2, num_heads=3)
    with pytest.raises(RuntimeError, match="ROCm device"):
        late({"a": torch.randn(2, 4), "b": torch.randn(2, 4)}, None)


def _load(model, sd, dev):
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    return model.to(dev).eval()


@pytest.mark.gpu
@pytest.mark.parametrize("case", FRAMEPOOL_CASES, ids=lambda c: c.name)
def test_frame_encoder_matches_reference(enc_mod, case):
    dev = torch.device("cuda", 0)
    fx = load_fixture(case.name)
    model = _load(enc_mod.FrameEncoder(case.frame_dim, case.hidden, case.out_dim, temporal_pooling="attention"),
                  framepool_state(case), dev)
    frames, mask, g_pool, g_out = framepool_inputs(case)
    m = torch.from_numpy(mask).to(dev) if mask is not None else None
    pin = torch.from_numpy(fx["pool_in"]).to(dev).requires_grad_(True)
    pooled = model.attention_pool(pin, m)
    (pooled * torch.from_numpy(g_pool).to(dev)).sum().backward()
    assert torch.isfinite(pooled).all()
    assert rel_err(pooled.detach(), fx["pooled"]) <= TOL
    assert rel_err(pin.grad, fx["dpool_in"]) <= TOL
    assert rel_err(model.attention.weight.grad, fx["pool_grad/attention.weight"]) <= TOL
    # mathematically zero (softmax is shift-invariant): rounding noise only
    assert close(model.attention.bias.grad, fx["pool_grad/attention.bias"], TOL, 1e-5)
    model.zero_grad(set_to_none=True)
    ft = torch.from_numpy(frames).to(dev).requires_grad_(True)
    enc = model(ft, m)
    (enc * torch.from_numpy(g_out).to(dev)).sum().backward()
    assert rel_err(enc.detach(), fx["encoding"]) <= TOL
    assert rel_err(ft.grad, fx["dframes"]) <= TOL
    for name, p in model.named_parameters():
        assert close(p.grad, fx[f"grad/{name}"], TOL, 1e-5), name


@pytest.mark.gpu
@pytest.mark.parametrize("B,T,D", [(64, 300, 256), (3, 1, 5), (17, 77, 130)])
def test_attention_pool_vs_oracle(enc_mod, B, T, D):
    """Sizes beyond the fixtures (C4-shaped 300-frame video), ragged and all-masked rows."""
    from oracle.softmax_pool_cpu import attention_pool as ref_pool
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(B * 1000 + T)
    x = torch.randn(B, T, D, generator=g)
    lin = torch.nn.Linear(D, 1)
    with torch.no_grad():
        lin.weight.copy_(torch.randn(1, D, generator=g) * 0.3)
        lin.bias.fill_(0.1)
    mask = (torch.rand(B, T, generator=g) > 0.3).float()
    mask[0] = 0.0
    if T > 1:
        mask[-1, 1:] = 0.0
    gp = torch.randn(B, D, generator=g)
    xr = x.clone().requires_grad_(True)
    lr = torch.nn.Linear(D, 1)
    lr.load_state_dict(lin.state_dict())
    ref = ref_pool(xr, lr.weight, lr.bias, mask)
    (ref * gp).sum().backward()
    lin = lin.to(dev)
    xd = x.to(dev).requires_grad_(True)
    out = enc_mod.attention_pool(xd, lin, mask.to(dev))
    (out * gp.to(dev)).sum().backward()
    assert rel_err(out.detach(), ref.detach()) <= TOL
    assert rel_err(xd.grad, xr.grad) <= TOL
    assert rel_err(lin.weight.grad, lr.weight.grad) <= TOL
    assert close(lin.bias.grad, lr.bias.grad, TOL, 1e-4)   # ~0: shift-invariant softmax
    assert float(out[0].detach().abs().max()) == 0.0          # all frames masked -> nan_to_num -> 0


@pytest.mark.gpu
@pytest.mark.parametrize("case", LATE_CASES, ids=lambda c: c.name)
def test_late_fusion_matches_reference(fusion_mod, case):
    dev = torch.device("cuda", 0)
    fx = load_fixture(case.name)
    model = _load(fusion_mod.LateFusion({m: case.dims[m] for m in case.names}, hidden_dim=case.hidden,
                                        num_classes=case.classes), late_state(case), dev)
    feats_np, mask_np, grad = late_inputs(case)
    feats = {m: torch.from_numpy(v).to(dev).requires_grad_(True) for m, v in feats_np.items()}
    fused, per = model(feats, torch.from_numpy(mask_np).to(dev))
    (fused * torch.from_numpy(grad).to(dev)).sum().backward()
    assert rel_err(fused.detach(), fx["fused"]) <= TOL
    for m in case.names:
        assert rel_err(per[m].detach(), fx[f"per/{m}"]) <= TOL
        assert rel_err(feats[m].grad, fx[f"dx/{m}"]) <= TOL
    for name, p in model.named_parameters():
        assert close(p.grad, fx[f"grad/{name}"], TOL, 1e-6), name


@pytest.mark.gpu
def test_late_fusion_missing_modality_fallback(fusion_mod):
    """tests/test_fusion.py:22-48 semantics (reference): one modality present -> its logits;
    none present -> the uniform 1/M average."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = fusion_mod.LateFusion({"video": 4, "imu": 4}, num_classes=3, hidden_dim=8, dropout=0.0).to(dev).eval()
    feats = {"video": torch.randn(2, 4, device=dev), "imu": torch.randn(2, 4, device=dev)}
    fused, per = model(feats, torch.tensor([[1.0, 0.0], [0.0, 0.0]], device=dev))
    assert torch.allclose(fused[0], per["video"][0], atol=1e-6)
    assert torch.allclose(fused[1], (per["video"][1] + per["imu"][1]) / 2, atol=1e-6)


@pytest.mark.gpu
def test_late_weights_vs_oracle_large(fusion_mod):
    from oracle.softmax_pool_cpu import late_weights
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    B, M, C = 1000, 8, 25
    st = torch.randn(B, M, C, generator=g)
    wl = torch.randn(M, generator=g)
    mask = (torch.rand(B, M, generator=g) > 0.5).float()
    mask[:10] = 0.0
    gf = torch.randn(B, C, generator=g)
    sr, wr = st.clone().requires_grad_(True), wl.clone().requires_grad_(True)
    (late_weights(sr, wr, mask) * gf).sum().backward()
    sd, wd = st.to(dev).requires_grad_(True), wl.to(dev).requires_grad_(True)
    out = fusion_mod._late_weights(sd, wd, mask.to(dev))
    (out * gf.to(dev)).sum().backward()
    assert rel_err(out.detach(), late_weights(st, wl, mask)) <= TOL
    assert rel_err(sd.grad, sr.grad) <= TOL
    assert rel_err(wd.grad, wr.grad) <= TOL
