"""Pin the CPU oracle against outputs of the reference itself (golden fixtures).

CPU-only.  The fixtures were produced by tests/golden/gen_golden.py running the
reference HybridFusion / CrossModalAttention (src/fusion.py:331-479,
src/attention.py:68-146) in eval mode.  The oracle is an independent
restatement, so agreement here is at fp32 reassociation level (<=1e-5 rel).
"""
import numpy as np
import pytest
import torch

from _util import close, load_fixture, oracle_cma, oracle_hybrid, rel_err
from cases import CMA_CASES, HYBRID_CASES, TEMPORAL_CASES, cma_state, temporal_inputs

TOL = 1e-5


@pytest.mark.parametrize("case", HYBRID_CASES, ids=lambda c: c.name)
def test_oracle_hybrid_matches_reference(case):
    fx = load_fixture(case.name)
    out, grads, dx = oracle_hybrid(case)
    assert rel_err(out["logits"], fx["logits"]) <= TOL
    assert rel_err(out["fusion_weights"], fx["fusion_weights"]) <= TOL
    assert rel_err(out["pooled"], fx["pooled"]) <= TOL
    for k in fx:
        if k.startswith("attn/"):
            assert rel_err(out[k], fx[k]) <= TOL, k
        elif k.startswith("attnslice/"):
            got = out["attn/" + k[len("attnslice/"):]].reshape(-1)[::case.attn_slice]
            assert rel_err(got, fx[k]) <= TOL, k
    for m in case.names:
        assert rel_err(dx[m], fx[f"dx/{m}"]) <= TOL, m
    for k, g in grads.items():
        if case.full:
            assert close(g, fx[f"grad/{k}"], TOL, 1e-6), k
        else:
            n = float(np.linalg.norm(g.double().numpy().reshape(-1)))
            assert abs(n - float(fx[f"gradnorm/{k}"][0])) <= TOL * max(n, 1e-6) + 1e-6, k
            assert close(g.reshape(-1)[::37], fx[f"gradslice/{k}"], TOL, 1e-6), k


@pytest.mark.parametrize("case", CMA_CASES, ids=lambda c: c.name)
def test_oracle_cma_matches_reference(case):
    fx = load_fixture(case.name)
    out = oracle_cma(case)
    for k in fx:
        assert close(out[k], fx[k], TOL, 1e-6), k


def test_known_answer_weights():
    """tests/test_fusion.py:50-80 semantics: [1,1] sums to 1, [1,0] -> [1,0], [0,0] -> [.5,.5]."""
    fx = load_fixture("known_answer_2mod")
    w = torch.from_numpy(fx["fusion_weights"])
    assert torch.allclose(w[0].sum(), torch.tensor(1.0), atol=1e-6)
    assert torch.allclose(w[1], torch.tensor([1.0, 0.0]), atol=1e-6)
    assert torch.allclose(w[2], torch.full((2,), 0.5), atol=1e-6)


def test_l1_zero_qk_grads():
    """At L=1 the softmax over one key is constant: q/k projection grads are exactly 0."""
    fx = load_fixture("tiny_l1")
    for k, v in fx.items():
        if k.startswith("grad/attention_modules") and ("query_proj" in k or "key_proj" in k):
            assert np.all(v == 0.0), k


@pytest.mark.parametrize("case", TEMPORAL_CASES, ids=lambda c: c.name)
def test_oracle_temporal_matches_reference(case):
    """TemporalAttention = the CMA restatement with q = k = v and a per-key mask,
    then the reference's post-mask broadcast (src/attention.py:233-248)."""
    from oracle.hybrid_cpu import cma_forward
    fx = load_fixture(case.name)
    sd = cma_state(case.feature_dim, case.feature_dim, case.hidden, case.seed)
    params = {k: torch.from_numpy(v) for k, v in sd.items()}
    seq, mask, _ = temporal_inputs(case)
    st = torch.from_numpy(seq)
    km = None
    if mask is not None:
        m = torch.from_numpy(mask)
        m = m.unsqueeze(0) if m.dim() == 1 else m
        km = m.expand(case.batch, case.seq).contiguous()
    att, w = cma_forward(params, "", st, st, st, case.heads, mask=km)
    if mask is not None:
        att = att * m.unsqueeze(1).unsqueeze(2).unsqueeze(-1)
    assert rel_err(att, fx["attended"]) <= TOL
    assert rel_err(w, fx["weights"]) <= TOL


# --------------------------------------------------------------------------
# §8(f) masked-softmax weighting ops: FrameEncoder attention pooling, LateFusion
# --------------------------------------------------------------------------
from cases import (FRAMEPOOL_CASES, LATE_CASES, framepool_inputs, framepool_state,  # noqa: E402
                   late_inputs, late_state)


@pytest.mark.parametrize("case", FRAMEPOOL_CASES, ids=lambda c: c.name)
def test_oracle_framepool_matches_reference(case):
    from oracle.softmax_pool_cpu import attention_pool, frame_encoder
    fx = load_fixture(case.name)
    params = {k: torch.from_numpy(v).requires_grad_(True) for k, v in framepool_state(case).items()}
    frames, mask, g_pool, g_out = framepool_inputs(case)
    m = torch.from_numpy(mask) if mask is not None else None
    pin = torch.from_numpy(fx["pool_in"]).requires_grad_(True)
    pooled = attention_pool(pin, params["attention.weight"], params["attention.bias"], m)
    (pooled * torch.from_numpy(g_pool)).sum().backward()
    assert rel_err(pooled.detach(), fx["pooled"]) <= TOL
    assert rel_err(pin.grad, fx["dpool_in"]) <= TOL
    assert rel_err(params["attention.weight"].grad, fx["pool_grad/attention.weight"]) <= TOL
    assert close(params["attention.bias"].grad, fx["pool_grad/attention.bias"], TOL, 1e-6)
    assert torch.isfinite(pooled).all()
    for p in params.values():
        p.grad = None
    ft = torch.from_numpy(frames).requires_grad_(True)
    enc = frame_encoder(params, ft, m)
    (enc * torch.from_numpy(g_out)).sum().backward()
    assert rel_err(enc.detach(), fx["encoding"]) <= TOL
    assert rel_err(ft.grad, fx["dframes"]) <= TOL
    for k, p in params.items():
        assert close(p.grad, fx[f"grad/{k}"], TOL, 1e-7), k


@pytest.mark.parametrize("case", LATE_CASES, ids=lambda c: c.name)
def test_oracle_late_matches_reference(case):
    from oracle.softmax_pool_cpu import late_fusion
    fx = load_fixture(case.name)
    params = {k: torch.from_numpy(v).requires_grad_(True) for k, v in late_state(case).items()}
    feats_np, mask_np, grad = late_inputs(case)
    feats = {m: torch.from_numpy(v).requires_grad_(True) for m, v in feats_np.items()}
    fused, per = late_fusion(params, case.names, feats, torch.from_numpy(mask_np))
    (fused * torch.from_numpy(grad)).sum().backward()
    assert rel_err(fused.detach(), fx["fused"]) <= TOL
    for m in case.names:
        assert rel_err(per[m].detach(), fx[f"per/{m}"]) <= TOL
        assert rel_err(feats[m].grad, fx[f"dx/{m}"]) <= TOL
    for k, p in params.items():
        assert close(p.grad, fx[f"grad/{k}"], TOL, 1e-7), k


# --------------------------------------------------------------------------
# §8(f) SequenceEncoder (LSTM)
# --------------------------------------------------------------------------
from cases import SEQENC_CASES, seqenc_inputs, seqenc_state  # noqa: E402


@pytest.mark.parametrize("case", SEQENC_CASES, ids=lambda c: c.name)
def test_oracle_seqenc_matches_reference(case):
    from oracle.lstm_cpu import sequence_encoder
    fx = load_fixture(case.name)
    params = seqenc_state(case)
    seq, lengths, g_out = seqenc_inputs(case)
    enc, outputs, dseq, grads = sequence_encoder(params, case.layers, seq, lengths, g_out)
    assert rel_err(torch.from_numpy(enc), fx["encoding"]) <= TOL
    assert rel_err(torch.from_numpy(outputs), fx["outputs"]) <= TOL
    assert rel_err(torch.from_numpy(dseq), fx["dsequence"]) <= TOL
    for k, g in grads.items():
        assert close(torch.from_numpy(g), fx[f"grad/{k}"], TOL, 1e-7), k


def test_oracle_relu_gate_hook():
    """hybrid_forward(relu_gate=...) (the device's ReLU' decision at pre-activations within rounding
    of 0, used by the GPU parity tests): an empty selection is the plain oracle bit for bit; a
    selected element takes the given slope; tests/_util.device_relu_gates refuses a device that
    passed a pre-activation the oracle puts clearly below 0."""
    from _util import device_relu_gates, hybrid_inputs, hybrid_state
    from oracle.hybrid_cpu import hybrid_forward
    case = HYBRID_CASES[0]
    sd = hybrid_state(case.names, case.dims, case.hidden, case.classes, case.seed, case.deleted)
    feats_np, mask_np, grad_np = hybrid_inputs(case)

    def run(taps=None, gate=None):
        params = {k: torch.from_numpy(v).requires_grad_(True) for k, v in sd.items()}
        feats = {m: torch.from_numpy(v).requires_grad_(True) for m, v in feats_np.items()}
        logits, _ = hybrid_forward(params, case.names, feats, torch.from_numpy(mask_np), case.heads,
                                   taps=taps, relu_gate=gate)
        (logits * torch.from_numpy(grad_np)).sum().backward()
        return logits.detach(), {k: p.grad for k, p in params.items()}

    taps = {}
    base, gbase = run(taps)
    m = case.names[0]
    z = taps[f"z/{m}"]
    none = {m: (torch.zeros_like(z, dtype=torch.bool), torch.zeros_like(z, dtype=torch.bool))}
    same, gsame = run(gate=none)
    assert torch.equal(same, base) and all(torch.equal(gsame[k], gbase[k]) for k in gbase if gbase[k] is not None)
    # one clearly positive pre-activation given slope 0: that activation (only) is 0
    flat = int((z.reshape(-1) > 0).nonzero()[0])
    sel = torch.zeros(z.numel(), dtype=torch.bool)
    sel[flat] = True
    taps2 = {}
    cut, _ = run(taps2, gate={m: (sel.reshape(z.shape), torch.zeros_like(z, dtype=torch.bool))})
    a0, a1 = taps[f"a/{m}"].detach().reshape(-1), taps2[f"a/{m}"].detach().reshape(-1)
    assert float(a0[flat]) > 0 and float(a1[flat]) == 0.0
    keep = torch.ones_like(a0, dtype=torch.bool)
    keep[flat] = False
    assert torch.equal(a0[keep], a1[keep]) and not torch.equal(cut, base)
    # device_relu_gates: the oracle's own activations pass; a clearly positive z the "device" passed
    # as 0 is allowed (dropout), a clearly negative z it passed as > 0 is refused
    wts = {mm: torch.from_numpy(sd[f"projections.{mm}.0.weight"]) for mm in case.names}
    acts = {mm: torch.relu(taps[f"z/{mm}"]) for mm in case.names}
    gates, band = device_relu_gates(taps, wts, acts)
    assert set(gates) == set(case.names) and all(v >= 0 for v in band.values())
    neg = int((z.reshape(-1) < -1e-3).nonzero()[0])
    bad = acts[m].clone().reshape(-1)
    bad[neg] = 1.0
    acts[m] = bad.reshape(z.shape)
    with pytest.raises(AssertionError):
        device_relu_gates(taps, wts, acts)
