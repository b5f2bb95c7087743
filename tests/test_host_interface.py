"""CPU tests of the drop-in host mirror (no GPU needed).

The reference's own interface tests (tests/test_fusion.py:330-406,
tests/test_attention.py:30-110) pin: constructor surface, state_dict keys,
error types/messages raised before any compute, the deleted-pair skip, and the
factory.  Compute itself needs a ROCm device: on CPU tensors the product path
must raise (no CPU fallback).
"""
import numpy as np
import pytest
import torch

from _util import load_fixture
from cases import HYBRID_CASES, hybrid_state


@pytest.fixture(scope="module")
def mods(pkg_on_path):
    import attention
    import fusion
    return fusion, attention


def test_state_dict_keys_match_reference(mods):
    fusion, _ = mods
    for case in HYBRID_CASES:
        model = fusion.HybridFusion({m: case.dims[m] for m in case.names}, hidden_dim=case.hidden,
                                    num_classes=case.classes, num_heads=case.heads)
        for key in case.deleted:
            del model.attention_modules[key]
        ref_keys = list(hybrid_state(case.names, case.dims, case.hidden, case.classes, case.seed,
                                     case.deleted).keys())
        assert sorted(model.state_dict().keys()) == sorted(ref_keys)
        # shapes too
        sd = hybrid_state(case.names, case.dims, case.hidden, case.classes, case.seed, case.deleted)
        model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)


def test_fixture_param_names_are_reference_names(mods):
    """The fixtures store grads under the reference module's own named_parameters()."""
    fusion, _ = mods
    fx = load_fixture("tiny_l1")
    case = HYBRID_CASES[0]
    model = fusion.HybridFusion({m: case.dims[m] for m in case.names}, hidden_dim=case.hidden,
                                num_classes=case.classes, num_heads=case.heads)
    names = {k[len("grad/"):] for k in fx if k.startswith("grad/")}
    assert names == {n for n, _ in model.named_parameters()}


def test_same_init_as_reference_under_seed(mods):
    """Construction order mirrors src/fusion.py:291-328 so a seed gives the reference's init."""
    fusion, _ = mods
    torch.manual_seed(123)
    a = fusion.HybridFusion({"video": 8, "imu": 4}, hidden_dim=16, num_classes=3, num_heads=2)
    torch.manual_seed(123)
    b = fusion.HybridFusion({"video": 8, "imu": 4}, hidden_dim=16, num_classes=3, num_heads=2)
    for (ka, va), (kb, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert ka == kb and torch.equal(va, vb)


def test_reference_init_equivalence_if_available(mods):
    """Same seed => bitwise-identical parameters to the reference module (container only)."""
    import sys
    from pathlib import Path
    if not Path("/root/reference/src/fusion.py").exists():
        pytest.skip("reference not present (GPU box)")
    fusion, _ = mods
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_attention", "/root/reference/src/attention.py")
    ref_att = importlib.util.module_from_spec(spec)
    sys.modules["ref_attention"] = ref_att
    spec.loader.exec_module(ref_att)
    torch.manual_seed(7)
    ours = fusion.CrossModalAttention(12, 20, hidden_dim=16, num_heads=4)
    torch.manual_seed(7)
    theirs = ref_att.CrossModalAttention(12, 20, hidden_dim=16, num_heads=4)
    for (ka, va), (kb, vb) in zip(ours.state_dict().items(), theirs.state_dict().items()):
        assert ka == kb and torch.equal(va, vb)


def test_errors_before_launch(mods):
    fusion, _ = mods
    with pytest.raises(ValueError, match="No modalities configured"):
        fusion.HybridFusion({}, num_classes=3)({}, torch.ones(2, 0))
    model = fusion.HybridFusion({"video": 4, "imu": 4}, num_classes=3)
    with pytest.raises(KeyError, match="Missing features for modality"):
        model({"video": torch.randn(2, 4)}, torch.ones(2, 2))
    with pytest.raises(ValueError, match="modality_mask must be provided"):
        model.compute_adaptive_weights({m: torch.randn(2, 4) for m in ("video", "imu")}, None)
    agg = {"video": model.projections["video"](torch.randn(2, 4))}
    with pytest.raises(KeyError, match="Missing aggregated features"):
        model.compute_adaptive_weights(agg, torch.ones(2, 2))
    with pytest.raises(ValueError, match="Unknown fusion type"):
        fusion.build_fusion_model("ensemble", {"video": 4}, num_classes=3)
    with pytest.raises(AssertionError):
        fusion.CrossModalAttention(4, 4, hidden_dim=10, num_heads=4)


def test_mask_and_feature_shapes_checked_before_launch(mods):
    """A mask that is not (B, M) / (1, M) -- the shapes the reference's indexing and
    broadcasting accept (src/fusion.py:371-373,462-467) -- raises on the host, before
    its pointer could reach a kernel; so do wrongly shaped compute_adaptive_weights
    features (gating_layers[m](feat) then cat(dim=1), src/fusion.py:452-461)."""
    fusion, _ = mods
    model = fusion.HybridFusion({"video": 4, "imu": 4}, num_classes=3, hidden_dim=8, num_heads=2)
    feats = {"video": torch.randn(3, 4), "imu": torch.randn(3, 4)}
    for bad in (torch.ones(2), torch.ones(3), torch.ones(3, 1), torch.ones(3, 3), torch.ones(2, 2),
                torch.ones(4, 2), torch.ones(3, 2, 1)):
        with pytest.raises(RuntimeError, match="modality_mask must have shape"):
            model(feats, bad)
    late = fusion.LateFusion({"video": 4, "imu": 4}, num_classes=3, hidden_dim=8)
    for bad in (torch.ones(2), torch.ones(3, 1), torch.ones(5, 2)):
        with pytest.raises(RuntimeError, match="modality_mask must have shape"):
            late(feats, bad)
    agg = {"video": torch.randn(3, 8), "imu": torch.randn(3, 8)}
    with pytest.raises(RuntimeError, match="modality_mask must have shape"):
        model.compute_adaptive_weights(agg, torch.ones(3, 3))
    for bad_feats in ({"video": torch.randn(3, 8), "imu": torch.randn(2, 8)},
                      {"video": torch.randn(3, 8), "imu": torch.randn(3, 7)},
                      {"video": torch.randn(3, 1, 8), "imu": torch.randn(3, 8)}):
        with pytest.raises(RuntimeError, match="must have shape"):
            model.compute_adaptive_weights(bad_feats, torch.ones(3, 2))
    # a (1, M) mask broadcasts over the batch as in the reference: passes the checks
    # and reaches the device requirement
    with pytest.raises(RuntimeError, match="ROCm device"):
        model(feats, torch.ones(1, 2))


def test_cpu_tensors_raise_no_fallback(mods):
    fusion, attention = mods
    model = fusion.HybridFusion({"video": 4, "imu": 4}, num_classes=3, num_heads=1, hidden_dim=8)
    with pytest.raises(RuntimeError, match="ROCm device"):
        model({"video": torch.randn(2, 4), "imu": torch.randn(2, 4)}, torch.ones(2, 2))
    cma = attention.CrossModalAttention(8, 8, hidden_dim=8, num_heads=2)
    with pytest.raises(RuntimeError, match="ROCm device"):
        cma(torch.randn(2, 8), torch.randn(2, 8), torch.randn(2, 8))


def test_deleted_pair_and_pair_order(mods):
    fusion, _ = mods
    model = fusion.HybridFusion({"a": 4, "b": 4, "c": 4}, num_classes=3, hidden_dim=8, num_heads=2)
    del model.attention_modules["a_to_b"]
    keys = [k for _, _, k in model.present_pairs()]
    assert keys == ["a_to_c", "b_to_a", "b_to_c", "c_to_a", "c_to_b"]


def test_factory_signature(mods):
    fusion, _ = mods
    m = fusion.build_fusion_model("hybrid", {"a": 4, "b": 6}, num_classes=5, hidden_dim=8,
                                  num_heads=2, dropout=0.2)
    assert isinstance(m, fusion.HybridFusion)
    assert m.hidden_dim == 8 and m.num_modalities == 2 and m.dropout.p == 0.2
    e = fusion.build_fusion_model("early", {"a": 4}, num_classes=5, hidden_dim=8, num_heads=2)
    assert isinstance(e, fusion.EarlyFusion)
    late = fusion.build_fusion_model("late", {"a": 4, "b": 4}, num_classes=2, num_heads=3)
    assert isinstance(late, fusion.LateFusion) and late.weight_logits.shape == (2,)


def test_deepcopy_and_plan_descriptor(mods):
    import copy
    fusion, _ = mods
    model = fusion.HybridFusion({"a": 6, "b": 10}, num_classes=4, hidden_dim=32, num_heads=4)
    model2 = copy.deepcopy(model)
    assert model2.state_dict().keys() == model.state_dict().keys()
    plan = model._plan([torch.randn(3, 5, 6), torch.randn(3, 7, 10)], True)
    d = plan.desc
    assert (d.batch, d.num_modalities, d.hidden, d.num_heads, d.num_classes) == (3, 2, 32, 4, 4)
    assert list(d.seq_len)[:2] == [5, 7] and list(d.in_dim)[:2] == [6, 10]
    assert d.num_pairs == 2 and (d.pair_q[0], d.pair_k[0], d.pair_q[1], d.pair_k[1]) == (0, 1, 1, 0)
    params = plan.params(model)
    assert len(params) == len(list(model.parameters()))
    # flat buffers: every tensor on a 256-byte boundary, no overlap
    assert all(o % 64 == 0 for o in plan.offsets)
    ends = [o + p.numel() for o, p in zip(plan.offsets, params)]
    assert all(e <= o2 for e, o2 in zip(ends, plan.offsets[1:])) and ends[-1] <= plan.num_param_elems
    views = plan.grad_views(torch.zeros(plan.num_param_elems), params)
    assert [v.shape for v in views] == [p.shape for p in params]


def test_early_fusion_matches_reference(mods):
    """BASELINE config C1's fusion: EarlyFusion (src/fusion.py:17-123) is plain-torch plumbing
    (concat of masked features -> MLP, no HIP part) and runs on CPU as the reference's does;
    logits and every gradient equal the reference's on tests/golden/early_3mod.npz."""
    from cases import EARLY_CASES, early_state, late_inputs
    fusion, _ = mods
    torch.set_float32_matmul_precision("highest")
    for case in EARLY_CASES:
        fx = load_fixture(case.name)
        model = fusion.EarlyFusion({m: case.dims[m] for m in case.names}, hidden_dim=case.hidden,
                                   num_classes=case.classes, dropout=0.1)
        model.load_state_dict({k: torch.from_numpy(v) for k, v in early_state(case).items()}, strict=True)
        model.eval()
        feats_np, mask_np, grad = late_inputs(case)
        feats = {m: torch.from_numpy(v).requires_grad_(True) for m, v in feats_np.items()}
        logits = model(feats, torch.from_numpy(mask_np))
        (logits * torch.from_numpy(grad)).sum().backward()
        tol = dict(rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(logits.detach().numpy(), fx["logits"], **tol)
        for m in case.names:
            np.testing.assert_allclose(feats[m].grad.numpy(), fx[f"dx/{m}"], **tol)
        for name, p in model.named_parameters():
            np.testing.assert_allclose(p.grad.numpy(), fx[f"grad/{name}"], **tol, err_msg=name)
        with pytest.raises(ValueError, match="Expected 2D tensor"):
            model({m: torch.zeros(2, 3, case.dims[m]) for m in case.names})
