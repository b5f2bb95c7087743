"""The rest of src/attention.py's import surface (tests/test_attention.py:22-27):
TemporalAttention, PairwiseModalityAttention, visualize_attention.

CPU tests cover structure, error behaviour and the pure-torch helpers; GPU tests
compare the HIP-backed forward/backward with fixtures produced by the reference
(tests/golden/gen_golden.py) at the parity tolerance (1e-3 relative).
"""
import numpy as np
import pytest
import torch

from _util import close, load_fixture
from cases import (PAIRWISE_CASES, TEMPORAL_CASES, cma_state, pairwise_inputs, pairwise_state,
                   temporal_inputs)

RTOL, ATOL = 1e-3, 1e-5


@pytest.fixture(scope="module")
def attn_mod(pkg_on_path):
    import attention
    return attention


def test_import_surface(attn_mod):
    for name in ("CrossModalAttention", "TemporalAttention", "PairwiseModalityAttention", "visualize_attention"):
        assert hasattr(attn_mod, name), name


@pytest.mark.parametrize("case", TEMPORAL_CASES, ids=lambda c: c.name)
def test_temporal_state_dict_keys(attn_mod, case):
    m = attn_mod.TemporalAttention(case.feature_dim, hidden_dim=case.hidden, num_heads=case.heads)
    fx = load_fixture(case.name)
    assert {f"grad/{k}" for k in m.state_dict()} == {k for k in fx if k.startswith("grad/")}
    assert (m.feature_dim, m.hidden_dim, m.num_heads, m.head_dim) == (
        case.feature_dim, case.hidden, case.heads, case.hidden // case.heads)
    assert abs(m.scale - (case.hidden // case.heads) ** -0.5) < 1e-12


def test_pool_sequence(attn_mod):
    torch.manual_seed(0)
    m = attn_mod.TemporalAttention(8, hidden_dim=16, num_heads=4)
    seq = torch.randn(3, 5, 16)
    w = torch.rand(3, 4, 5, 5)
    pooled = m.pool_sequence(seq, w)
    pw = w.mean(dim=1).mean(dim=1)
    pw = pw / (pw.sum(dim=1, keepdim=True) + 1e-8)
    assert pooled.shape == (3, 16)
    assert torch.allclose(pooled, torch.einsum("bl,bld->bd", pw, seq), atol=1e-6)
    with pytest.raises(ValueError):
        m.pool_sequence(seq, w.mean(dim=1))


def test_pairwise_structure_and_errors(attn_mod):
    case = PAIRWISE_CASES[0]
    m = attn_mod.PairwiseModalityAttention({k: case.dims[k] for k in case.names}, hidden_dim=case.hidden,
                                           num_heads=case.heads)
    for key in case.deleted:
        del m.attention_layers[key]
    assert set(m.state_dict()) == set(pairwise_state(case))
    with pytest.raises(ValueError, match="No modalities"):
        attn_mod.PairwiseModalityAttention({})({}, modality_mask=None)


def test_visualize_attention_saves(attn_mod, tmp_path):
    import matplotlib
    matplotlib.use("Agg")
    out = tmp_path / "sub" / "attn.png"
    attn_mod.visualize_attention(torch.rand(4, 3, 3), ["a", "b", "c"], save_path=str(out))
    assert out.exists() and out.stat().st_size > 0


# --------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("case", TEMPORAL_CASES, ids=lambda c: c.name)
def test_temporal_matches_reference(attn_mod, case):
    fx = load_fixture(case.name)
    m = attn_mod.TemporalAttention(case.feature_dim, hidden_dim=case.hidden, num_heads=case.heads, dropout=0.1)
    sd = cma_state(case.feature_dim, case.feature_dim, case.hidden, case.seed)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    m = m.cuda().eval()
    seq, mask, grad = temporal_inputs(case)
    st = torch.from_numpy(seq).cuda().requires_grad_(True)
    mt = torch.from_numpy(mask).cuda() if mask is not None else None
    att, w = m(st, mt)
    assert tuple(att.shape) == fx["attended"].shape
    (att * torch.from_numpy(grad).cuda()).sum().backward()
    torch.cuda.synchronize()
    assert close(att.detach().cpu(), fx["attended"], RTOL, ATOL)
    assert close(w.cpu(), fx["weights"], RTOL, ATOL)
    assert not torch.isnan(att).any()
    assert close(st.grad.cpu(), fx["dsequence"], RTOL, ATOL)
    for name, p in m.named_parameters():
        assert close(p.grad.cpu(), fx[f"grad/{name}"], RTOL, ATOL), name


@pytest.mark.gpu
@pytest.mark.parametrize("case", PAIRWISE_CASES, ids=lambda c: c.name)
def test_pairwise_matches_reference(attn_mod, case):
    fx = load_fixture(case.name)
    m = attn_mod.PairwiseModalityAttention({k: case.dims[k] for k in case.names}, hidden_dim=case.hidden,
                                           num_heads=case.heads, dropout=0.1)
    for key in case.deleted:
        del m.attention_layers[key]
    m.load_state_dict({k: torch.from_numpy(v) for k, v in pairwise_state(case).items()}, strict=True)
    m = m.cuda().eval()
    feats_np, mask_np, grads_np = pairwise_inputs(case)
    feats = {k: torch.from_numpy(v).cuda().requires_grad_(True) for k, v in feats_np.items()}
    attended, maps = m(feats, torch.from_numpy(mask_np).cuda())
    sum((attended[k] * torch.from_numpy(grads_np[k]).cuda()).sum() for k in case.names).backward()
    torch.cuda.synchronize()
    assert set(maps) == {k[5:] for k in fx if k.startswith("attn/")}
    for k in case.names:
        assert close(attended[k].detach().cpu(), fx[f"attended/{k}"], RTOL, ATOL), k
        assert close(feats[k].grad.cpu(), fx[f"dx/{k}"], RTOL, ATOL), k
    for k, w in maps.items():
        assert close(w.cpu(), fx[f"attn/{k}"], RTOL, ATOL), k
    for name, p in m.named_parameters():
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        assert close(g.cpu(), fx[f"grad/{name}"], RTOL, ATOL), name
