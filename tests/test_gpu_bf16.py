"""GPU parity of the bf16 math mode (torch.set_float32_matmul_precision("medium")).

The reference trains with ``training.matmul_precision: medium``
(config/base.yaml:80, applied by src/train.py:53-68,448), which lets fp32
matmuls use bf16 operands with fp32 accumulation.  The drop-in modules read
``torch.get_float32_matmul_precision()`` and, at "medium", every MFMA of the
HIP path (projection / Q K V O GEMMs, QK^T, attn.V and their backward) takes
bf16 operands; storage, softmax, reductions and the head stay fp32.

Tolerances, written here, against the fp32 reference
(the reference-generated fixtures tests/golden/*.npz, or at the C5 per-sample
shape -- 6 modalities, L = 512, H = 256, key masks -- the CPU oracle on the same
seeded inputs):
  * logits: max|got - ref| <= 3e-2 * max|ref|, argmax agreement >= 99 %;
  * fusion weights, attention maps, input and parameter gradients:
    ||got - ref||_2 <= max(3e-2 ||ref||_2, 4 ||emu - ref||_2, 3e-3 S), where
    emu is the CPU oracle with every matmul (forward and backward) taking
    bf16-rounded operands (tests/_util.bf16_matmul_mode) -- the error bf16
    operands cost by themselves -- and S is the largest reference norm among
    the gradients compared in the same test.  Gradients behind a softmax
    backward with cancellation (dS = P (dP - D)) legitimately lose more than
    3e-2 in bf16 (seq_equal dx/m0: 9.5 % in the emulation); the path must stay
    within a small multiple of what bf16 operands alone cost.  The 3e-3 S
    floor covers tensors that are mathematically zero or cancelling sums:
    key_proj.bias grads (softmax shift invariance), dQ at L = 1 (where the
    flash-style D = rowsum(dO * O) and the bf16 dP = dO V^T differ by
    rounding, as in any reduced-precision attention backward), and the gating
    bias grads (a sum over the batch of per-sample terms of both signs).
Each test also checks that the bf16 instantiations ran (the precision argument of
the profiler kernel names is 1) and that the result differs from the fp32 path.
"""
import re

import numpy as np
import pytest
import torch

from _util import load_fixture, oracle_cma, oracle_hybrid
from cases import CMA_CASES, HYBRID_CASES, HybridCase, cma_inputs, cma_state, hybrid_inputs, hybrid_state

pytestmark = pytest.mark.gpu
LOGIT_RTOL = 3e-2
NORM_RTOL, NORM_ATOL, FLOOR_REL = 3e-2, 1e-6, 3e-3


@pytest.fixture(scope="module")
def mods(pkg_on_path):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    import attention
    import fusion
    import mmf_native
    mmf_native.lib()
    return fusion, attention, mmf_native


@pytest.fixture
def medium():
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("medium")
    yield
    torch.set_float32_matmul_precision(prev)


def _t(x):
    return torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x).double().cpu()


def logits_ok(got, ref):
    got, ref = _t(got), _t(ref)
    assert got.shape == ref.shape
    err = float((got - ref).abs().max()) / max(float(ref.abs().max()), 1e-6)
    agree = float((got.argmax(-1) == ref.argmax(-1)).double().mean())
    return err <= LOGIT_RTOL and agree >= 0.99, (err, agree)


def norm_ok(got, ref, emu, scale=0.0):
    got, ref, emu = _t(got), _t(ref), _t(emu)
    assert got.shape == ref.shape == emu.shape, (tuple(got.shape), tuple(ref.shape), tuple(emu.shape))
    d, de, rn = float((got - ref).norm()), float((emu - ref).norm()), float(ref.norm())
    bound = max(NORM_RTOL * rn, 4.0 * de, FLOOR_REL * scale) + NORM_ATOL
    return d <= bound, dict(err=d, bound=bound, ref_norm=rn, emu_err=de)


def group_scale(refs):
    return max(float(_t(r).norm()) for r in refs)


def _precision(kname):
    """The int precision argument of a library MFMA kernel name (bench.kernel_precision)."""
    m = re.search(r"[<, ]([012])(?:, (?:true|false)){0,3}>$", kname)
    return int(m.group(1)) if m else None


def _is_bf16(kname):
    return _precision(kname) == 1


def _bf16_kernels_ran(nat, launches):
    names = [k for _, k, *_ in launches]
    mfma = [k for k in names if k.startswith(("gemm_lds", "gemm_wsr", "attn_fwd", "attn_bwd_d", "attn_pool"))]
    return len(mfma) > 0 and all(_is_bf16(k) for k in mfma), mfma


def build_hybrid(fusion, case, dev="cuda"):
    model = fusion.HybridFusion({m: case.dims[m] for m in case.names}, hidden_dim=case.hidden,
                                num_classes=case.classes, num_heads=case.heads, dropout=0.1)
    for key in case.deleted:
        del model.attention_modules[key]
    sd = hybrid_state(case.names, case.dims, case.hidden, case.classes, case.seed, case.deleted)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    return model.to(dev).eval()


def run_hybrid(fusion, case):
    model = build_hybrid(fusion, case)
    feats_np, mask_np, grad_np = hybrid_inputs(case)
    feats = {m: torch.from_numpy(v).cuda().requires_grad_(True) for m, v in feats_np.items()}
    logits, info = model(feats, torch.from_numpy(mask_np).cuda(), return_attention=True)
    (logits * torch.from_numpy(grad_np).cuda()).sum().backward()
    torch.cuda.synchronize()
    return model, feats, logits.detach(), info


SEQ_CASES = [c for c in HYBRID_CASES if c.seq_mode] + [c for c in HYBRID_CASES if c.name == "c2_l1"]


@pytest.mark.parametrize("case", SEQ_CASES, ids=lambda c: c.name)
def test_hybrid_bf16_matches_reference(mods, medium, case):
    fusion, _, nat = mods
    fx = load_fixture(case.name)
    nat.profile_begin()
    model, feats, logits, info = run_hybrid(fusion, case)
    _, launches = nat.profile_end()
    ran, names = _bf16_kernels_ran(nat, launches)
    assert ran, names
    eo, eg, edx = oracle_hybrid(case, bf16_matmul=True)
    ok, e = logits_ok(logits.cpu(), fx["logits"])
    assert ok, e
    ok, e = norm_ok(info["fusion_weights"].cpu(), fx["fusion_weights"], eo["fusion_weights"])
    assert ok, e
    for key, amap in info["attention_maps"].items():
        if case.attn_slice:
            ok, e = norm_ok(amap.cpu().reshape(-1)[::case.attn_slice], fx[f"attnslice/{key}"],
                            eo[f"attn/{key}"].reshape(-1)[::case.attn_slice])
        else:
            ok, e = norm_ok(amap.cpu(), fx[f"attn/{key}"], eo[f"attn/{key}"])
        assert ok, (key, e)
    gpre = "grad/" if case.full else "gradslice/"
    S = group_scale([fx[f"dx/{m}"] for m in case.names] + [fx[gpre + n] for n, _ in model.named_parameters()])
    for m in case.names:
        ok, e = norm_ok(feats[m].grad.cpu(), fx[f"dx/{m}"], edx[m], S)
        assert ok, (m, e)
    for name, p in model.named_parameters():
        g = p.grad.detach().cpu()
        if case.full:
            ok, e = norm_ok(g, fx[f"grad/{name}"], eg[name], S)
        else:
            ok, e = norm_ok(g.reshape(-1)[::37], fx[f"gradslice/{name}"], eg[name].reshape(-1)[::37], S)
        assert ok, (name, e)


def test_bf16_differs_from_fp32(mods):
    """The mode switch is real: same inputs, "highest" vs "medium" give different bits,
    and "highest" runs only fp32 instantiations."""
    fusion, _, nat = mods
    case = next(c for c in HYBRID_CASES if c.name == "seq_c2_b3")
    prev = torch.get_float32_matmul_precision()
    try:
        torch.set_float32_matmul_precision("highest")
        nat.profile_begin()
        _, _, l32, _ = run_hybrid(fusion, case)
        _, launches = nat.profile_end()
        mfma = [k for _, k, *_ in launches if k.startswith(("gemm_lds", "gemm_wsr", "attn_"))]
        assert mfma and not any(_precision(k) in (1, 2) for k in mfma), mfma
        torch.set_float32_matmul_precision("medium")
        _, _, l16, _ = run_hybrid(fusion, case)
    finally:
        torch.set_float32_matmul_precision(prev)
    assert not torch.equal(l32, l16)
    ok, e = logits_ok(l16.cpu(), l32.cpu())
    assert ok, e


@pytest.mark.parametrize("case", CMA_CASES, ids=lambda c: c.name)
def test_cma_bf16_matches_reference(mods, medium, case):
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
    att, w = model(qt, kt, vt, mt)
    (att * torch.from_numpy(grad).cuda()).sum().backward()
    torch.cuda.synchronize()
    emu = oracle_cma(case, bf16_matmul=True)
    for got, key in ((att.detach(), "attended"), (w, "weights")):
        ok, e = norm_ok(got.cpu().reshape(fx[key].shape), fx[key], emu[key].reshape(fx[key].shape))
        assert ok, (key, e)
    S = group_scale([fx[k] for k in ("dquery", "dkey", "dvalue")] +
                    [fx[f"grad/{n}"] for n, _ in model.named_parameters()])
    for got, key in ((qt.grad, "dquery"), (kt.grad, "dkey"), (vt.grad, "dvalue")):
        ok, e = norm_ok(got.cpu().reshape(fx[key].shape), fx[key], emu[key].reshape(fx[key].shape), S)
        assert ok, (key, e)
    for name, p in model.named_parameters():
        ok, e = norm_ok(p.grad.cpu(), fx[f"grad/{name}"], emu[f"grad/{name}"], S)
        assert ok, (name, e)


# C5 per-sample shape (M = 6, T = 512, D = H = 256, 4 heads, key
# masks keep 0.9 with >= 1 kept) at B = 2: the general attention plan
# (Lk > 128) in bf16, checked against the CPU oracle on the same inputs.
C5_MINI = HybridCase("c5_mini", [f"m{i}" for i in range(6)], {f"m{i}": 256 for i in range(6)},
                     {f"m{i}": 512 for i in range(6)}, batch=2, hidden=256, heads=4, classes=5,
                     seed=51, mask=[[1, 1, 0, 1, 1, 1], [1, 0, 1, 1, 1, 0]], full=True)


@pytest.mark.parametrize("precision", ["highest", "high", "medium"])
def test_c5_shape_vs_oracle(mods, precision):
    """fp32 tolerance at "highest" and "high" (bf16x3; plus a 1e-4 S floor for the
    near-zero gradients whose cancelling terms carry the split-operand rounding), the
    bf16 bounds at "medium"."""
    fusion, _, nat = mods
    out, grads, dx = oracle_hybrid(C5_MINI)
    if precision == "medium":
        _, egrads, edx = oracle_hybrid(C5_MINI, bf16_matmul=True)
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision(precision)
    try:
        model, feats, logits, info = run_hybrid(fusion, C5_MINI)
    finally:
        torch.set_float32_matmul_precision(prev)
    fp32 = precision in ("highest", "high")
    if fp32:
        err = float((_t(logits) - _t(out["logits"])).abs().max() / _t(out["logits"]).abs().max())
        assert err <= 1e-3, err
    else:
        ok, e = logits_ok(logits.cpu(), out["logits"])
        assert ok, e
    S = group_scale([dx[m] for m in C5_MINI.names] + list(grads.values()))
    floor = 1e-6 if precision == "highest" else 1e-4 * S
    for m in C5_MINI.names:
        if fp32:
            d = _t(feats[m].grad) - _t(dx[m])
            assert float(d.norm()) <= 1e-3 * float(_t(dx[m]).norm()) + floor, m
        else:
            ok, e = norm_ok(feats[m].grad, dx[m], edx[m], S)
            assert ok, (m, e)
    for name, p in model.named_parameters():
        if fp32:
            d = _t(p.grad) - _t(grads[name])
            assert float(d.norm()) <= 1e-3 * float(_t(grads[name]).norm()) + floor, name
        else:
            ok, e = norm_ok(p.grad, grads[name], egrads[name], S)
            assert ok, (name, e)


# One-pass long-key forward and backward (csrc/attn_long.hip, "medium" only) against the
# two-kernel paths they replace (MMF_NO_LONG_FUSED=1: attn_poolL_lse/colsum_kernel,
# attn_poolL_dq_kernel + attn_pool_bwd_dk_kernel) on the same inputs, in TRAIN mode (both
# draw the same Philox keep words), with
# partial query blocks (a: 500 queries), 256- and 512-key pairs, a masked key modality in
# one sample and the pairs whose keys are not whole 32-key tiles removed (they would send
# the call to the two-kernel path).  Both are bf16 computations of the same math; they
# differ by the rounding of P' (bf16 terms of the column sums) and dS (fma vs two ops) and
# the summation order, so the bounds are the bf16 ones (LOGIT_RTOL, NORM_RTOL) relative to
# the two-kernel result.
LONG_TRAIN = HybridCase("long_train", ["a", "b", "c"], {"a": 48, "b": 64, "c": 32}, {"a": 500, "b": 512, "c": 256},
                        batch=3, hidden=128, heads=2, classes=5, seed=77,
                        mask=[[1, 1, 1], [1, 1, 0], [1, 0, 1]], deleted=["b_to_a", "c_to_a"])


def test_long_key_one_pass_backward_matches_two_kernel_path(mods, medium, monkeypatch):
    fusion, _, nat = mods
    case = LONG_TRAIN
    feats_np, mask_np, grad_np = hybrid_inputs(case)
    mask = torch.from_numpy(mask_np).cuda()
    g = torch.from_numpy(grad_np).cuda()

    def run(two_kernel):
        if two_kernel:
            monkeypatch.setenv("MMF_NO_LONG_FUSED", "1")
        else:
            monkeypatch.delenv("MMF_NO_LONG_FUSED", raising=False)
        model = build_hybrid(fusion, case).train()
        model._rng_state.copy_(torch.tensor([1234, 5], dtype=torch.int64))
        feats = {m: torch.from_numpy(v).cuda().requires_grad_(True) for m, v in feats_np.items()}
        nat.profile_begin()
        logits = model(feats, mask)
        (logits * g).sum().backward()
        torch.cuda.synchronize()
        _, launches = nat.profile_end()
        names = [k for _, k, *_ in launches]
        return logits.detach(), {m: f.grad for m, f in feats.items()}, \
            {n: p.grad.clone() for n, p in model.named_parameters()}, names

    l1, dx1, dw1, n1 = run(False)
    l2, dx2, dw2, n2 = run(True)
    monkeypatch.delenv("MMF_NO_LONG_FUSED", raising=False)
    assert any(k.startswith("attn_poolL_bwd_fused_bf16<true, ") for k in n1), n1
    assert any(k.startswith("attn_poolL_fwd_fused_bf16<true") for k in n1), n1
    assert not any(k.startswith(("attn_poolL_dq", "attn_poolL_lse", "attn_poolL_colsum")) for k in n1), n1
    assert any(k.startswith("attn_poolL_dq") for k in n2), n2
    ok, e = logits_ok(l1.cpu(), l2.cpu())
    assert ok, e
    S = group_scale([_t(v) for v in dx2.values()] + [_t(v) for v in dw2.values()])
    for m in case.names:
        ok, e = norm_ok(dx1[m], dx2[m], dx2[m], S)
        assert ok, (m, e)
    for n in dw2:
        ok, e = norm_ok(dw1[n], dw2[n], dw2[n], S)
        assert ok, (n, e)


def test_long_key_one_pass_train_vs_oracle_medium(mods, medium):
    """The one-pass long-key kernels in TRAIN mode against the CPU oracle: the device's Philox
    keep masks replayed on the CPU (tests/_philox.py), the oracle run in fp32 and with
    bf16-rounded matmul operands (the error a bf16 path must show), the bf16 bounds."""
    from _philox import mask_provider
    from _util import bf16_matmul_mode
    from oracle.hybrid_cpu import hybrid_forward
    fusion, _, nat = mods
    case = LONG_TRAIN
    seed, offset, p = 0x2468_ACE0_1357, 3, 0.1
    sd = hybrid_state(case.names, case.dims, case.hidden, case.classes, case.seed, case.deleted)
    model = build_hybrid(fusion, case).train()
    model._rng_state.copy_(torch.tensor([seed, offset], dtype=torch.int64))
    feats_np, mask_np, grad_np = hybrid_inputs(case)
    feats = {m: torch.from_numpy(v).cuda().requires_grad_(True) for m, v in feats_np.items()}
    nat.profile_begin()
    logits = model(feats, torch.from_numpy(mask_np).cuda())
    (logits * torch.from_numpy(grad_np).cuda()).sum().backward()
    torch.cuda.synchronize()
    _, launches = nat.profile_end()
    names = [k for _, k, *_ in launches]
    assert any(k.startswith("attn_poolL_fwd_fused_bf16<true") for k in names), names
    assert any(k.startswith("attn_poolL_bwd_fused_bf16<true, ") for k in names), names
    # the Q / K projections on bf16 copies of P_m and of the weights (qk_gemm_b16)
    assert "gemm_lds_kernel<0, 0, 32, 3, 1, 1>" in names and "cvt_bf16_kernel" in names, names

    def oracle(bf16):
        params = {k: torch.from_numpy(v).requires_grad_(True) for k, v in sd.items()}
        xs = {m: torch.from_numpy(v).requires_grad_(True) for m, v in feats_np.items()}

        def run():
            ref, _ = hybrid_forward(params, case.names, xs, torch.from_numpy(mask_np), case.heads, p=p,
                                    train=True, gen=mask_provider(seed, offset, p))
            (ref * torch.from_numpy(grad_np)).sum().backward()
            return ref.detach()
        if bf16:
            with bf16_matmul_mode():
                ref = run()
        else:
            ref = run()
        return ref, {m: xs[m].grad for m in case.names}, {n: params[n].grad for n in sd}

    ref, rdx, rdw = oracle(False)
    emu, edx, edw = oracle(True)
    ok, e = logits_ok(logits.detach().cpu(), ref)
    assert ok, e
    S = group_scale(list(rdx.values()) + list(rdw.values()))
    for m in case.names:
        ok, e = norm_ok(feats[m].grad, rdx[m], edx[m], S)
        assert ok, (m, e)
    for n, prm in model.named_parameters():
        ok, e = norm_ok(prm.grad, rdw[n], edw[n], S)
        assert ok, (n, e)
