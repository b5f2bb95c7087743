"""Generate golden parity fixtures by running the REFERENCE implementation.

Container-only tool: it imports ``/root/reference/src`` (read-only, never copied)
and writes small ``.npz`` fixtures next to this file.  The GPU box never runs
it; tests there rebuild the inputs from the seeds in ``cases.py`` and compare
against the stored outputs.

What is recorded (eval mode, ``torch.set_float32_matmul_precision("highest")``):
  * HybridFusion, 2-D inputs (reference semantics, L=1): the reference module's
    own ``forward(..., return_attention=True)`` (src/fusion.py:331-427).
  * HybridFusion, 3-D inputs (sequence mode): the composed oracle of SURVEY §8c,
    built only from the reference module's own sub-modules: ``projections``,
    ``attention_modules`` called on 3-D tensors (src/attention.py:92-146),
    mean over the per-modality list, x mask, mean-pool over L,
    ``compute_adaptive_weights`` (src/fusion.py:429-479), ``classifier``.
  * standalone CrossModalAttention (src/attention.py:68-146), TemporalAttention
    (src/attention.py:149-281) and PairwiseModalityAttention (:284-424).
  * FrameEncoder attention pooling (src/encoders.py:210-336) and LateFusion
    (src/fusion.py:126-245), the §8(f) masked-softmax weighting ops; EarlyFusion
    (src/fusion.py:17-123), config C1's fusion.
  * for a fixed upstream gradient G: d(sum(out * G)) w.r.t. inputs and params.

Run:  python tests/golden/gen_golden.py [case1,case2,...]
"""

from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
REF_SRC = Path("/root/reference/src")

from cases import (CMA_CASES, EARLY_CASES, FRAMEPOOL_CASES, HYBRID_CASES, LATE_CASES, PAIRWISE_CASES, SEQENC_CASES,  # noqa: E402
                   TEMPORAL_CASES, cma_inputs, cma_state, early_state, framepool_inputs, framepool_state,
                   hybrid_inputs, hybrid_state, late_inputs, late_state, pair_names,
                   pairwise_inputs, pairwise_state, temporal_inputs, seqenc_inputs, seqenc_state)


def _load_reference():
    sys.path.insert(0, str(REF_SRC))
    import attention as ref_attention  # noqa: F401
    import encoders as ref_encoders
    import fusion as ref_fusion
    return ref_fusion, ref_attention, ref_encoders


def composed_seq_forward(model, feats, mask):
    """SURVEY §8c composed oracle: reference sub-modules only, pooled over L."""
    names = model.modality_names
    P = {}
    for i, m in enumerate(names):
        x = feats[m]
        mk = mask[:, i].reshape(-1, *([1] * (x.dim() - 1)))
        P[m] = model.projections[m](model.dropout(x * mk))
    lists = {m: [P[m]] for m in names}
    maps = {}
    for q in names:
        for k in names:
            if q == k:
                continue
            key = f"{q}_to_{k}"
            if key not in model.attention_modules:
                continue
            ki = names.index(k)
            att, w = model.attention_modules[key](P[q], P[k], P[k], mask=mask[:, ki])
            lists[q].append(att)
            maps[key] = w
    pooled = {}
    for i, m in enumerate(names):
        agg = torch.stack(lists[m], dim=0).mean(dim=0)
        mk = mask[:, i].reshape(-1, *([1] * (agg.dim() - 1)))
        agg = agg * mk
        pooled[m] = agg.mean(dim=1) if agg.dim() == 3 else agg
    weights = model.compute_adaptive_weights(pooled, mask)
    stacked = torch.stack([pooled[m] for m in names], dim=1)
    fused = (stacked * weights.unsqueeze(-1)).sum(dim=1)
    logits = model.classifier(fused)
    return logits, {"attention_maps": maps, "fusion_weights": weights, "pooled": stacked}


def gen_hybrid(ref_fusion, case):
    dims = {m: case.dims[m] for m in case.names}
    model = ref_fusion.HybridFusion(dims, hidden_dim=case.hidden, num_classes=case.classes,
                                    num_heads=case.heads, dropout=0.1)
    for key in case.deleted:
        del model.attention_modules[key]
    sd = hybrid_state(case.names, case.dims, case.hidden, case.classes, case.seed, case.deleted)
    missing, unexpected = model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()},
                                                strict=True)
    assert not missing and not unexpected
    model.eval()
    feats_np, mask_np, grad_np = hybrid_inputs(case)
    feats = {m: torch.from_numpy(v).requires_grad_(True) for m, v in feats_np.items()}
    mask = torch.from_numpy(mask_np)

    pooled_hook = {}
    if case.seq_mode:
        logits, info = composed_seq_forward(model, feats, mask)
        pooled = info["pooled"]
    else:
        # capture the aggregated (B,M,H) tensor the reference feeds to the weighting
        orig = model.compute_adaptive_weights

        def hook(features, m):
            pooled_hook["pooled"] = torch.stack([features[n] for n in model.modality_names], 1)
            return orig(features, m)
        model.compute_adaptive_weights = hook
        logits, info = model(feats, mask, return_attention=True)
        pooled = pooled_hook["pooled"]
        # reference-vs-composed self check at L=1 (bit-identical)
        del model.compute_adaptive_weights
        logits2, _ = composed_seq_forward(model, {m: t.detach() for m, t in feats.items()}, mask)
        assert torch.equal(logits.detach(), logits2.detach()), "composed oracle != reference at L=1"

    (logits * torch.from_numpy(grad_np)).sum().backward()
    out = {
        "logits": logits.detach().numpy(),
        "fusion_weights": info["fusion_weights"].detach().numpy(),
        "pooled": pooled.detach().numpy(),
        "mask": mask_np,
    }
    for key in pair_names(case.names, case.deleted):
        amap = info["attention_maps"][key].detach().numpy()
        if case.attn_slice:
            out[f"attnslice/{key}"] = amap.reshape(-1)[::case.attn_slice].copy()
        else:
            out[f"attn/{key}"] = amap
    for m in case.names:
        g = feats[m].grad.numpy()
        out[f"dx/{m}"] = g
    for k, p in model.named_parameters():
        g = p.grad.numpy() if p.grad is not None else np.zeros_like(p.detach().numpy())
        if case.full:
            out[f"grad/{k}"] = g
        else:
            flat = g.reshape(-1)
            out[f"gradnorm/{k}"] = np.asarray([np.linalg.norm(flat.astype(np.float64))])
            out[f"gradslice/{k}"] = flat[::37].copy()
    return out


def gen_cma(ref_attention, case):
    model = ref_attention.CrossModalAttention(case.query_dim, case.key_dim, hidden_dim=case.hidden,
                                              num_heads=case.heads, dropout=0.1)
    sd = cma_state(case.query_dim, case.key_dim, case.hidden, case.seed)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    model.eval()
    q, k, v, mask, grad = cma_inputs(case)
    qt = torch.from_numpy(q).requires_grad_(True)
    kt = torch.from_numpy(k).requires_grad_(True)
    vt = torch.from_numpy(v).requires_grad_(True)
    mt = torch.from_numpy(mask) if mask is not None else None
    att, w = model(qt, kt, vt, mt)
    (att * torch.from_numpy(grad)).sum().backward()
    out = {"attended": att.detach().numpy(), "weights": w.detach().numpy(),
           "dquery": qt.grad.numpy(), "dkey": kt.grad.numpy(), "dvalue": vt.grad.numpy()}
    for name, p in model.named_parameters():
        out[f"grad/{name}"] = p.grad.numpy()
    return out


def gen_temporal(ref_attention, case):
    model = ref_attention.TemporalAttention(case.feature_dim, hidden_dim=case.hidden, num_heads=case.heads,
                                            dropout=0.1)
    sd = cma_state(case.feature_dim, case.feature_dim, case.hidden, case.seed)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    model.eval()
    seq, mask, grad = temporal_inputs(case)
    st = torch.from_numpy(seq).requires_grad_(True)
    mt = torch.from_numpy(mask) if mask is not None else None
    att, w = model(st, mt)
    assert tuple(att.shape) == grad.shape, (tuple(att.shape), grad.shape)
    (att * torch.from_numpy(grad)).sum().backward()
    out = {"attended": att.detach().numpy(), "weights": w.detach().numpy(), "dsequence": st.grad.numpy()}
    for name, p in model.named_parameters():
        out[f"grad/{name}"] = p.grad.numpy()
    return out


def gen_pairwise(ref_attention, case):
    model = ref_attention.PairwiseModalityAttention({m: case.dims[m] for m in case.names},
                                                    hidden_dim=case.hidden, num_heads=case.heads, dropout=0.1)
    for key in case.deleted:
        del model.attention_layers[key]
    model.load_state_dict({k: torch.from_numpy(v) for k, v in pairwise_state(case).items()}, strict=True)
    model.eval()
    feats_np, mask_np, grads_np = pairwise_inputs(case)
    feats = {m: torch.from_numpy(v).requires_grad_(True) for m, v in feats_np.items()}
    attended, maps = model(feats, torch.from_numpy(mask_np))
    sum(((attended[m] * torch.from_numpy(grads_np[m])).sum() for m in case.names)).backward()
    out = {}
    for m in case.names:
        out[f"attended/{m}"] = attended[m].detach().numpy()
        out[f"dx/{m}"] = feats[m].grad.numpy()
    for k, w in maps.items():
        out[f"attn/{k}"] = w.detach().numpy()
    for name, p in model.named_parameters():
        out[f"grad/{name}"] = p.grad.numpy() if p.grad is not None else np.zeros_like(p.detach().numpy())
    return out


def gen_framepool(ref_encoders, case):
    """FrameEncoder(temporal_pooling="attention") (src/encoders.py:210-336): attention_pool
    on a fixed (B, T, hidden) input, and the whole encoder, each with its gradients."""
    model = ref_encoders.FrameEncoder(case.frame_dim, hidden_dim=case.hidden, output_dim=case.out_dim,
                                      temporal_pooling="attention", dropout=0.1)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in framepool_state(case).items()}, strict=True)
    model.eval()
    frames_np, mask_np, g_pool, g_out = framepool_inputs(case)
    mask = torch.from_numpy(mask_np) if mask_np is not None else None
    out = {}
    with torch.no_grad():
        pool_in = model.frame_processor(torch.from_numpy(frames_np))
    pin = pool_in.clone().requires_grad_(True)
    pooled = model.attention_pool(pin, mask)
    (pooled * torch.from_numpy(g_pool)).sum().backward()
    out.update({"pool_in": pool_in.numpy(), "pooled": pooled.detach().numpy(), "dpool_in": pin.grad.numpy(),
                "pool_grad/attention.weight": model.attention.weight.grad.numpy(),
                "pool_grad/attention.bias": model.attention.bias.grad.numpy()})
    model.zero_grad(set_to_none=True)
    ft = torch.from_numpy(frames_np).requires_grad_(True)
    enc = model(ft, mask)
    (enc * torch.from_numpy(g_out)).sum().backward()
    out.update({"encoding": enc.detach().numpy(), "dframes": ft.grad.numpy()})
    for name, p in model.named_parameters():
        out[f"grad/{name}"] = p.grad.numpy()
    return out


def gen_late(ref_fusion, case):
    """LateFusion (src/fusion.py:126-245): fused and per-modality logits, gradients."""
    model = ref_fusion.LateFusion({m: case.dims[m] for m in case.names}, hidden_dim=case.hidden,
                                  num_classes=case.classes, dropout=0.1)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in late_state(case).items()}, strict=True)
    model.eval()
    feats_np, mask_np, grad = late_inputs(case)
    feats = {m: torch.from_numpy(v).requires_grad_(True) for m, v in feats_np.items()}
    fused, per = model(feats, torch.from_numpy(mask_np))
    (fused * torch.from_numpy(grad)).sum().backward()
    out = {"fused": fused.detach().numpy()}
    for m in case.names:
        out[f"per/{m}"] = per[m].detach().numpy()
        out[f"dx/{m}"] = feats[m].grad.numpy()
    for name, p in model.named_parameters():
        out[f"grad/{name}"] = p.grad.numpy()
    return out


def gen_early(ref_fusion, case):
    """EarlyFusion (src/fusion.py:17-123): logits and gradients of sum(logits * G)."""
    model = ref_fusion.EarlyFusion({m: case.dims[m] for m in case.names}, hidden_dim=case.hidden,
                                   num_classes=case.classes, dropout=0.1)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in early_state(case).items()}, strict=True)
    model.eval()
    feats_np, mask_np, grad = late_inputs(case)
    feats = {m: torch.from_numpy(v).requires_grad_(True) for m, v in feats_np.items()}
    logits = model(feats, torch.from_numpy(mask_np))
    (logits * torch.from_numpy(grad)).sum().backward()
    out = {"logits": logits.detach().numpy()}
    for m in case.names:
        out[f"dx/{m}"] = feats[m].grad.numpy()
    for name, p in model.named_parameters():
        out[f"grad/{name}"] = p.grad.numpy()
    return out


def gen_seqenc(ref_encoders, case):
    """SequenceEncoder(encoder_type="lstm") (src/encoders.py:34-166): encoding, top-layer output
    sequence, and gradients of sum(encoding * g) w.r.t. the sequence and every parameter."""
    model = ref_encoders.SequenceEncoder(case.input_dim, hidden_dim=case.hidden, output_dim=case.out_dim,
                                         num_layers=case.layers, encoder_type="lstm", dropout=0.1)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in seqenc_state(case).items()}, strict=True)
    model.eval()
    seq_np, len_np, g_out = seqenc_inputs(case)
    seq = torch.from_numpy(seq_np).requires_grad_(True)
    lengths = torch.from_numpy(len_np) if len_np is not None else None
    enc = model(seq, lengths)
    (enc * torch.from_numpy(g_out)).sum().backward()
    with torch.no_grad():
        outputs, _ = model.rnn(torch.from_numpy(seq_np))
    out = {"encoding": enc.detach().numpy(), "dsequence": seq.grad.numpy(), "outputs": outputs.numpy()}
    for name, p in model.named_parameters():
        out[f"grad/{name}"] = p.grad.numpy()
    return out


def main():
    only = set(sys.argv[1].split(",")) if len(sys.argv) > 1 else None   # e.g. seq_c2_b3,seq_lean_hd64
    torch.set_float32_matmul_precision("highest")
    torch.set_num_threads(4)
    ref_fusion, ref_attention, ref_encoders = _load_reference()
    for case in HYBRID_CASES:
        if only and case.name not in only:
            continue
        out = gen_hybrid(ref_fusion, case)
        np.savez_compressed(HERE / f"{case.name}.npz", **out)
        print(f"wrote {case.name}.npz ({sum(a.nbytes for a in out.values())} B raw)")
    for cases, gen, mod in ((CMA_CASES, gen_cma, ref_attention), (TEMPORAL_CASES, gen_temporal, ref_attention),
                            (PAIRWISE_CASES, gen_pairwise, ref_attention),
                            (FRAMEPOOL_CASES, gen_framepool, ref_encoders), (LATE_CASES, gen_late, ref_fusion),
                            (EARLY_CASES, gen_early, ref_fusion),
                            (SEQENC_CASES, gen_seqenc, ref_encoders)):
        for case in cases:
            if only and case.name not in only:
                continue
            out = gen(mod, case)
            np.savez_compressed(HERE / f"{case.name}.npz", **out)
            print(f"wrote {case.name}.npz ({sum(a.nbytes for a in out.values())} B raw)")


if __name__ == "__main__":
    main()
