"""Single-key attention (Lk = 1, the reference's own 2-D inputs) on the GPU.

With one key, softmax over the key axis is the mask indicator (1, or 0 through
-inf -> NaN -> nan_to_num; src/attention.py:118-129), so the reference's autograd
gives query_proj / key_proj exactly zero gradient, and the standalone
CrossModalAttention exactly zero d(query) / d(key) (SURVEY §0.3, §8d "Q/K grads are
exactly 0 at L=1"; the reference fixtures hold 0.0 there).  The HIP path skips the
Q / K projections, QK^T and every Q / K gradient for such pairs (csrc/single_key.hip)
and writes those gradients as exact zeros: asserted bit-exactly here at every
matmul precision, in eval and train mode, alongside the usual tolerance on every
other output (tests/test_gpu_parity.py has the full fixture comparison).
"""
import numpy as np
import pytest
import torch

from _util import close, load_fixture
from cases import CMA_CASES, HYBRID_CASES, cma_inputs, cma_state, hybrid_inputs, hybrid_state

pytestmark = pytest.mark.gpu

L1_CASES = [c for c in HYBRID_CASES if not c.seq_mode]
L1_CMA = [c for c in CMA_CASES if c.lk == 0]


@pytest.fixture(scope="module")
def mods(pkg_on_path):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    import attention
    import fusion
    import mmf_native
    mmf_native.lib()
    return fusion, attention, mmf_native


@pytest.fixture(params=["highest", "high", "medium"])
def precision(request):
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision(request.param)
    yield request.param
    torch.set_float32_matmul_precision(prev)


def _build(fusion, case, train=False, p=0.1):
    model = fusion.HybridFusion({m: case.dims[m] for m in case.names}, hidden_dim=case.hidden,
                                num_classes=case.classes, num_heads=case.heads, dropout=p)
    for key in case.deleted:
        del model.attention_modules[key]
    sd = hybrid_state(case.names, case.dims, case.hidden, case.classes, case.seed, case.deleted)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    model = model.cuda()
    return model.train() if train else model.eval()


def _assert_qk_zero(model):
    n = 0
    for name, prm in model.named_parameters():
        if ".query_proj." in name or ".key_proj." in name:
            assert prm.grad is not None, name
            assert torch.all(prm.grad == 0), (name, float(prm.grad.abs().max()))
            n += 1
    return n


def _kernels(launches):
    return [k for _, k, *_ in launches]


@pytest.mark.parametrize("case", L1_CASES, ids=lambda c: c.name)
def test_hybrid_l1_qk_grads_exactly_zero(mods, case, precision):
    fusion, _, nat = mods
    model = _build(fusion, case)
    feats_np, mask_np, grad_np = hybrid_inputs(case)
    feats = {m: torch.from_numpy(v).cuda().requires_grad_(True) for m, v in feats_np.items()}
    nat.profile_begin()
    logits, info = model(feats, torch.from_numpy(mask_np).cuda(), return_attention=True)
    (logits * torch.from_numpy(grad_np).cuda()).sum().backward()
    torch.cuda.synchronize()
    _, launches = nat.profile_end()
    assert _assert_qk_zero(model) == 4 * len(model.attention_modules)
    names = _kernels(launches)
    # no attention kernel (QK^T / softmax / dQ / dK) ran: the single-key kernels replaced it --
    # the launch-lean step (csrc/l1.hip) where it applies ("highest", every pair present, D_m and
    # H <= 128 and % 4), the general single-key plan otherwise
    lean = precision == "highest" and not case.deleted and case.hidden <= 128 and case.hidden % 4 == 0 \
        and all(case.dims[m] % 4 == 0 and case.dims[m] <= 128 for m in case.names) and case.classes <= 16
    want = "l1_pair_fwd_kernel" if lean else "sk_fwd_kernel"
    assert any(k.startswith(want) for k in names), names
    assert not [k for k in names if k.startswith("attn_")], names
    # the attention maps are the mask indicator (eval mode): exactly {0, 1}
    fx = load_fixture(case.name)
    for key, amap in info["attention_maps"].items():
        if case.attn_slice:
            ref = fx[f"attnslice/{key}"]
            got = amap.cpu().reshape(-1)[::case.attn_slice]
        else:
            ref, got = fx[f"attn/{key}"], amap.cpu()
        assert torch.equal(got, torch.from_numpy(np.ascontiguousarray(ref))), key
    if precision == "medium":
        return   # the bf16 bounds of the other outputs: tests/test_gpu_bf16.py
    assert close(logits.detach().cpu(), fx["logits"], 1e-3, 1e-5)


def test_hybrid_l1_train_mode_qk_grads_exactly_zero(mods, precision):
    """Train mode (dropout 0.5 on the attention maps): maps are {0, 2} per (b, head) and the
    Q / K gradients are still exact zeros."""
    fusion, _, _ = mods
    case = next(c for c in HYBRID_CASES if c.name == "c2_l1")
    model = _build(fusion, case, train=True, p=0.5)
    feats_np, mask_np, grad_np = hybrid_inputs(case)
    feats = {m: torch.from_numpy(v).cuda().requires_grad_(True) for m, v in feats_np.items()}
    mask = torch.from_numpy(mask_np).cuda()
    logits, info = model(feats, mask, return_attention=True)
    (logits * torch.from_numpy(grad_np).cuda()).sum().backward()
    torch.cuda.synchronize()
    _assert_qk_zero(model)
    names = list(model.modality_names)
    for key, amap in info["attention_maps"].items():
        assert set(torch.unique(amap).cpu().tolist()) <= {0.0, 2.0}, key
        k = names.index(key.split("_to_")[1])
        masked = mask[:, k] == 0
        assert torch.all(amap[masked] == 0), key
        keep = float((amap[~masked] == 2.0).float().mean())
        assert 0.4 < keep < 0.6, (key, keep)
    for m in names:
        assert torch.isfinite(feats[m].grad).all()


@pytest.mark.parametrize("case", L1_CMA, ids=lambda c: c.name)
def test_cma_l1_query_key_grads_exactly_zero(mods, case, precision):
    _, attention, nat = mods
    fx = load_fixture(case.name)
    model = attention.CrossModalAttention(case.query_dim, case.key_dim, hidden_dim=case.hidden,
                                          num_heads=case.heads, dropout=0.1)
    sd = cma_state(case.query_dim, case.key_dim, case.hidden, case.seed)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    model = model.cuda().eval()
    q, k, v, mask, grad = cma_inputs(case)
    qt, kt, vt = (torch.from_numpy(a).cuda().requires_grad_(True) for a in (q, k, v))
    mt = torch.from_numpy(mask).cuda() if mask is not None else None
    nat.profile_begin()
    att, w = model(qt, kt, vt, mt)
    (att * torch.from_numpy(grad).cuda()).sum().backward()
    torch.cuda.synchronize()
    _, launches = nat.profile_end()
    names = _kernels(launches)
    assert "sk_out_kernel" in names and not [n for n in names if n.startswith("attn_")], names
    assert torch.all(qt.grad == 0) and torch.all(kt.grad == 0)
    for name in ("query_proj.weight", "query_proj.bias", "key_proj.weight", "key_proj.bias"):
        g = dict(model.named_parameters())[name].grad
        assert torch.all(g == 0), name
    assert torch.equal(w.cpu(), torch.from_numpy(fx["weights"]))
    if precision != "medium":
        assert close(att.detach().cpu(), fx["attended"], 1e-3, 1e-5)
        assert close(vt.grad.cpu(), fx["dvalue"], 1e-3, 1e-5)


@pytest.mark.parametrize("case_name", ["tiny_l1", "c2_l1"])
@pytest.mark.parametrize("train", [False, True])
def test_lean_l1_step_matches_general_plan(mods, case_name, train, monkeypatch):
    """The launch-lean single-key step (csrc/l1.hip) against the general single-key plan
    (MMF_NO_L1_LEAN=1) on the same weights, inputs and dropout stream: same logits, attention maps
    and fusion weights to 1e-5, every gradient to 1e-4 of its largest element (fp32 reassociation
    only), and the same exact zeros."""
    fusion, _, nat = mods
    case = next(c for c in HYBRID_CASES if c.name == case_name)
    feats_np, mask_np, grad_np = hybrid_inputs(case)
    runs = []
    for general in (False, True):
        if general:
            monkeypatch.setenv("MMF_NO_L1_LEAN", "1")
        model = _build(fusion, case, train=train, p=0.3)
        model._rng_state.copy_(torch.tensor([0x5EED, 3], dtype=torch.int64))
        feats = {m: torch.from_numpy(v).cuda().requires_grad_(True) for m, v in feats_np.items()}
        nat.profile_begin()
        logits, info = model(feats, torch.from_numpy(mask_np).cuda(), return_attention=True)
        (logits * torch.from_numpy(grad_np).cuda()).sum().backward()
        torch.cuda.synchronize()
        _, launches = nat.profile_end()
        names = _kernels(launches)
        want = "sk_fwd_kernel" if general else "l1_pair_fwd_kernel"
        assert any(k.startswith(want) for k in names), names
        runs.append((logits.detach().cpu(), {k: v.cpu() for k, v in info["attention_maps"].items()},
                     info["fusion_weights"].cpu(), [feats[m].grad.cpu() for m in case.names],
                     {n: p.grad.cpu() for n, p in model.named_parameters()}))
        monkeypatch.delenv("MMF_NO_L1_LEAN", raising=False)
    (l1, m1, w1, dx1, g1), (l2, m2, w2, dx2, g2) = runs
    assert close(l1, l2, 1e-5, 1e-6)
    assert close(w1, w2, 1e-5, 1e-7)
    for k in m1:
        assert torch.equal(m1[k], m2[k]), k
    for a, b in zip(dx1, dx2):
        assert close(a, b, 1e-4, 1e-8)
    for n in g1:
        if ".query_proj." in n or ".key_proj." in n:
            assert torch.all(g1[n] == 0) and torch.all(g2[n] == 0), n
        else:
            assert close(g1[n], g2[n], 1e-4, 1e-8), n
