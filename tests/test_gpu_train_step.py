"""The optimizer side of HybridTrainStep on the device:

* global-norm gradient clipping (torch.nn.utils.clip_grad_norm_, max_norm =
  config/base.yaml:74 gradient_clip_norm; Lightning applies it every step,
  src/train.py:416-430) and AdamW (src/train.py:374-381) against torch's own
  clip_grad_norm_ + torch.optim.AdamW on the same gradient;
* the flat gradient's norm against the oracle's gradients;
* a captured hipGraph step follows set_lr() (scheduler) and load_batch() (new
  data) without re-capture: bit-identical to the same sequence run eagerly.
"""
from __future__ import annotations

import math

import pytest
import torch

pytestmark = pytest.mark.gpu

M, B, L, D, H, HEADS, C = 3, 8, 6, 16, 16, 2, 5


@pytest.fixture(scope="module")
def mods(pkg_on_path):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    import fusion
    import train_step
    return fusion, train_step


def _batch(seed):
    g = torch.Generator().manual_seed(seed)
    feats = [torch.randn(B, L, D, generator=g) for _ in range(M)]
    mask = torch.ones(B, M)
    mask[1, 0] = 0.0
    mask[5, 2] = 0.5
    labels = torch.randint(0, C, (B,), generator=g)
    return feats, mask, labels


def _model(fusion, dropout):
    torch.manual_seed(3)
    return fusion.HybridFusion({f"m{i}": D for i in range(M)}, hidden_dim=H, num_classes=C, num_heads=HEADS,
                               dropout=dropout)


@pytest.mark.parametrize("max_norm", [0.05, 1.0, 0.0])
def test_clip_and_adamw_match_torch(mods, max_norm):
    fusion, train_step = mods
    from oracle.hybrid_cpu import hybrid_train_step
    feats, mask, labels = _batch(1)
    model = _model(fusion, 0.0).cuda()
    step = train_step.HybridTrainStep(model, [f.cuda() for f in feats], mask.cuda(), labels.cuda(), lr=3e-3,
                                      weight_decay=1e-4, gradient_clip_norm=max_norm)
    p0 = step.flat.clone().cpu()
    step.forward_backward()
    g = step.grad.clone().cpu()
    step.optimizer_step()
    torch.cuda.synchronize()
    # torch on the same gradient: clip_grad_norm_ then AdamW
    p = p0.clone().requires_grad_(True)
    p.grad = g.clone()
    norm = torch.nn.utils.clip_grad_norm_([p], max_norm if max_norm > 0 else float("inf"))
    opt = torch.optim.AdamW([p], lr=3e-3, weight_decay=1e-4)
    opt.step()
    assert abs(float(step.grad_norm.item()) - float(norm)) <= 1e-5 * float(norm)
    coef = float(step.clip_coef.item())
    want = min(1.0, max_norm / (float(norm) + 1e-6)) if max_norm > 0 else 1.0
    assert abs(coef - want) <= 1e-6 * want
    if max_norm == 0.05:
        assert coef < 1.0   # clipping is active in this case
    torch.testing.assert_close(step.flat.cpu(), p.detach(), rtol=1e-6, atol=1e-7)
    # and the gradient itself is the reference's (parity tolerance)
    names = model.modality_names
    params = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in model.state_dict().items()}
    for n, o in zip(step.plan.names, step.plan.offsets):   # pre-update weights
        params[n] = p0[o:o + params[n].numel()].view_as(params[n]).clone().requires_grad_(True)
    hybrid_train_step(params, names, {n: f.clone() for n, f in zip(names, feats)}, mask, labels, HEADS, 0.0)
    ref_norm = torch.sqrt(sum((params[n].grad.double() ** 2).sum() for n in step.plan.names
                              if params[n].grad is not None))
    assert abs(float(step.grad_norm.item()) - float(ref_norm)) <= 1e-3 * float(ref_norm)


def test_graph_follows_lr_and_new_batches(mods):
    fusion, train_step = mods
    a, b = _batch(2), _batch(3)

    def run(graph: bool):
        model = _model(fusion, 0.1).cuda()
        model._rng_state.copy_(torch.tensor([1234, 0], dtype=torch.int64))
        st = train_step.HybridTrainStep(model, [f.cuda() for f in a[0]], a[1].cuda(), a[2].cuda(), lr=1e-3)
        if graph:
            st.capture()
            # capture() ran one warm-up forward/backward: realign the step's own dropout state
            # (a copy of the module's buffer taken at construction) with the eager run
            st.rng.copy_(torch.tensor([1234, 0], dtype=torch.int64))
        st.step()
        st.set_lr(train_step.cosine_annealing_lr(50, 1e-3, 100))
        st.load_batch([f.cuda() for f in b[0]], b[1].cuda(), b[2].cuda())
        st.step()
        torch.cuda.synchronize()
        return st.flat.cpu(), float(st.loss.item()), st.lr

    pg, lg, lrg = run(True)
    pe, le, lre = run(False)
    assert lrg == lre == pytest.approx(train_step.cosine_annealing_lr(50, 1e-3, 100))
    assert le == lg
    assert torch.equal(pg, pe)


def test_load_batch_rejects_new_shapes(mods):
    fusion, train_step = mods
    feats, mask, labels = _batch(4)
    st = train_step.HybridTrainStep(_model(fusion, 0.0).cuda(), [f.cuda() for f in feats], mask.cuda(),
                                    labels.cuda())
    with pytest.raises(ValueError, match="load_batch"):
        st.load_batch([f[:4].cuda() for f in feats], mask[:4].cuda(), labels[:4].cuda())
    with pytest.raises(ValueError, match="load_batch"):
        st.load_batch([f.cuda() for f in feats[:2]], mask.cuda(), labels.cuda())


@pytest.mark.parametrize("max_norm", [0.05, 1e9])
def test_fused_clip_adamw_matches_two_call_path(mods, max_norm):
    """mmf_clip_adamw_step_dev (2 launches) == mmf_grad_clip_coef + mmf_adamw_step_dev (4), bit for bit."""
    import mmf_native as nat
    L = nat.lib()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    n = 70001                                   # not a multiple of 4: the scalar tail of the sum of squares
    grad = torch.randn(n, generator=g).to(dev)
    base = [torch.randn(n, generator=g).to(dev) for _ in range(3)]
    base[2] = base[2].abs()
    runs = []
    for fused in (False, True):
        p, m, v = (t.clone() for t in base)
        step = torch.full((1,), 4, dtype=torch.int64, device=dev)
        lr = torch.full((1,), 3e-3, dtype=torch.float32, device=dev)
        norm = torch.zeros(1, device=dev)
        coef = torch.zeros(1, device=dev)
        ws = torch.empty(L.mmf_grad_clip_workspace_bytes(), dtype=torch.uint8, device=dev)
        st = nat.stream_ptr(dev)
        for _ in range(2):
            if fused:
                rc = L.mmf_clip_adamw_step_dev(n, p.data_ptr(), grad.data_ptr(), m.data_ptr(), v.data_ptr(),
                                               step.data_ptr(), lr.data_ptr(), max_norm, norm.data_ptr(),
                                               coef.data_ptr(), ws.data_ptr(), 0.9, 0.999, 1e-8, 1e-4, 0.5, st)
                nat.check(rc, "fused")
            else:
                nat.check(L.mmf_grad_clip_coef(n, grad.data_ptr(), 0.5, max_norm, norm.data_ptr(), coef.data_ptr(),
                                               ws.data_ptr(), st), "clip")
                nat.check(L.mmf_adamw_step_dev(n, p.data_ptr(), grad.data_ptr(), m.data_ptr(), v.data_ptr(),
                                               step.data_ptr(), lr.data_ptr(), coef.data_ptr(), 0.9, 0.999, 1e-8,
                                               1e-4, 0.5, st), "adamw")
        torch.cuda.synchronize()
        runs.append((p, m, v, step, norm, coef))
    for a, b in zip(*runs):
        assert torch.equal(a, b)
    assert int(runs[1][3].item()) == 6
    if max_norm < 1.0:
        assert float(runs[1][5].item()) < 1.0


@pytest.mark.parametrize("accumulate", [2, 4])
@pytest.mark.parametrize("seq", [True, False])
def test_gradient_accumulation_equals_full_batch(mods, accumulate, seq):
    """accumulate = k (config/base.yaml:75 gradient_accumulation, Lightning's accumulate_grad_batches):
    k micro-batches of B/k samples, each loss scaled by 1/k, gradients summed on the device -- the
    gradient of the whole batch's mean loss (no dropout, so both runs see the same function), the
    same mean loss, the same input gradients; sequence mode and the 2-D single-key step."""
    fusion, train_step = mods
    feats, mask, labels = _batch(7)
    if not seq:
        feats = [f[:, 0] for f in feats]
    runs = []
    for acc in (1, accumulate):
        model = _model(fusion, 0.0).cuda()
        st = train_step.HybridTrainStep(model, [f.cuda() for f in feats], mask.cuda(), labels.cuda(), accumulate=acc)
        st.forward_backward()
        torch.cuda.synchronize()
        runs.append((st.grad.cpu(), float(st.loss.item()), [t.cpu() for t in st.dx], st.logits.cpu()))
    (g1, l1, dx1, lg1), (g2, l2, dx2, lg2) = runs
    assert torch.allclose(lg1, lg2, rtol=1e-5, atol=1e-6)
    assert abs(l1 - l2) <= 1e-5 * abs(l1)
    assert (g1 - g2).abs().max() <= 1e-5 * g1.abs().max()
    for a, b in zip(dx1, dx2):
        assert (a - b).abs().max() <= 1e-5 * a.abs().max()


def test_accumulate_rejects_uneven_micro_batches(mods):
    fusion, train_step = mods
    feats, mask, labels = _batch(8)
    with pytest.raises(ValueError, match="equal micro-batches"):
        train_step.HybridTrainStep(_model(fusion, 0.0).cuda(), [f.cuda() for f in feats], mask.cuda(), labels.cuda(),
                                   accumulate=3)


def _three_calls(st, nat):
    """The split path the one-call step replaces: mmf_hybrid_forward -> mmf_cross_entropy_ls ->
    mmf_hybrid_backward on the step's own buffers (accumulate = 1)."""
    import ctypes
    L = nat.lib()
    d = st.plan.desc
    s = nat.stream_ptr(st.dev)
    rc = L.mmf_hybrid_forward(ctypes.byref(d), ctypes.byref(st.pstruct), ctypes.cast(st.xarr[0], ctypes.c_void_p),
                              st.mask.data_ptr(), st.rng.data_ptr(), st.saved.data_ptr(), st.logits.data_ptr(),
                              st.fw.data_ptr(), None, s)
    nat.check(rc, "forward")
    rc = L.mmf_cross_entropy_ls(st.mask.size(0), d.num_classes, st.logits.data_ptr(), st.labels.data_ptr(),
                                st.smoothing, 1.0, st.losses.data_ptr(), st.dlogits.data_ptr(), s)
    nat.check(rc, "cross-entropy")
    rc = L.mmf_hybrid_backward(ctypes.byref(d), ctypes.byref(st.pstruct), ctypes.cast(st.xarr[0], ctypes.c_void_p),
                               st.mask.data_ptr(), st.saved.data_ptr(), st.dlogits.data_ptr(), st.ws.data_ptr(),
                               ctypes.byref(st.gstruct), ctypes.cast(st.dxarr[0], ctypes.c_void_p), s)
    nat.check(rc, "backward")


@pytest.mark.parametrize("seq", [False, True])
def test_one_call_train_step_matches_three_calls(mods, seq):
    """mmf_hybrid_train_step (HybridTrainStep's forward + CE + backward: on the 2-D single-key plan
    one launch for the forward, the loss, the head backward and the key-modality backward -- a
    per-tile arrival count hands each tile to the last of its pair workgroups, which runs the head
    while the others wait on its done word, then per-(tile, key) counts pick the workgroup that
    forms dZ / dX -- and one for the weight gradients) against forward -> cross-entropy -> backward
    as three calls, train mode with dropout, two consecutive steps: the same logits, loss, dlogits,
    fusion weights, parameter and input gradients bit for bit, the dropout stream advanced once
    per step, and every sync word (counts, done / seen words, the poll-timeout error word) at zero."""
    import mmf_native as nat
    fusion, train_step = mods
    feats, mask, labels = _batch(11)
    if not seq:
        feats = [f[:, 0] for f in feats]
    runs = []
    for split in (False, True):
        model = _model(fusion, 0.3).cuda()
        model._rng_state.copy_(torch.tensor([0xC0FFEE, 5], dtype=torch.int64))
        st = train_step.HybridTrainStep(model, [f.cuda() for f in feats], mask.cuda(), labels.cuda())
        nat.profile_begin()
        outs = []
        for _ in range(2):
            _three_calls(st, nat) if split else st.forward_backward()
            torch.cuda.synchronize()
            outs.append([t.detach().cpu().clone() for t in (st.logits, st.losses, st.dlogits, st.fw, st.grad,
                                                            *st.dx, model._rng_state)])
        _, launches = nat.profile_end()
        names = [k for _, k, *_ in launches]
        if not split and not seq:
            assert any(k.startswith("l1_fwd_loss_kernel") for k in names), names
            assert not any(k.startswith(("cross_entropy_kernel", "l1_head", "l1_key_bwd")) for k in names), names
            assert int(st.sync.count_nonzero()) == 0
        runs.append(outs)
    for step_a, step_b in zip(*runs):
        for a, b in zip(step_a, step_b):
            assert torch.equal(a, b)
    assert int(runs[0][1][-1][1]) == 7   # offset 5 -> 7 after two steps


@pytest.mark.parametrize("seq", [False, True])
def test_clip_partials_from_the_train_step(mods, seq):
    """fuse_clip (one process, one micro-batch): the train step writes the clip norm's squared-norm
    partials itself (the L = 1 plan in its weight-gradient launch, one partial per output tile; other
    plans with grad_sumsq_kernel) and advances the step counter, the optimizer runs the update launch
    only -- against fuse_clip=False (mmf_clip_adamw_step_dev's own reduction pass) over two clipped
    steps: the same gradient, the norm to 1e-6, the weights to 1e-6, the same step count."""
    fusion, train_step = mods
    feats, mask, labels = _batch(13)
    if not seq:
        feats = [f[:, 0] for f in feats]
    runs = []
    for fuse in (True, False):
        model = _model(fusion, 0.0).cuda()
        st = train_step.HybridTrainStep(model, [f.cuda() for f in feats], mask.cuda(), labels.cuda(), lr=3e-3,
                                        gradient_clip_norm=0.05, fuse_clip=fuse)
        assert st.fuse_clip == fuse
        out = []
        for _ in range(2):
            st.step()
            torch.cuda.synchronize()
            out.append((st.grad.cpu().clone(), float(st.grad_norm.item()), st.flat.cpu().clone(),
                        int(st.step_dev.item()), float(st.clip_coef.item())))
        runs.append(out)
        # gradients only (no optimizer step) leaves the optimizer's step counter alone, fused or not
        st.forward_backward()
        st.forward_backward()
        torch.cuda.synchronize()
        assert int(st.step_dev.item()) == 2
    for k, ((g1, n1, p1, s1, c1), (g2, n2, p2, s2, c2)) in enumerate(zip(*runs)):
        if k == 0:
            assert torch.equal(g1, g2)   # (the second step's gradient sees weights 1e-7 apart)
        assert abs(n1 - n2) <= 1e-6 * n2 and c1 < 1.0
        assert s1 == s2
        torch.testing.assert_close(p1, p2, rtol=1e-6, atol=1e-7)


def _seq_batch(seed, B=40, L=128, D=32, C=5):
    g = torch.Generator().manual_seed(seed)
    feats = [torch.randn(B, L, D, generator=g) for _ in range(M)]
    mask = (torch.rand(B, M, generator=g) < 0.8).float()
    mask[3] = 0.0
    mask[7, 1] = 0.5
    labels = torch.randint(0, C, (B,), generator=g)
    return feats, mask, labels


@pytest.mark.parametrize("hidden", [64, 128])
def test_tile_head_train_step(mods, hidden, monkeypatch):
    """The pooled tail plan's training step on the 16-sample tile head (csrc/l1.hip seq_head_kernel:
    the head forward, the cross-entropy, dlogits and the head backward in one launch, the batch-mean
    loss by the last tile to count) against (a) forward -> cross-entropy -> backward as three calls
    (the tile head's forward and backward launches): bit for bit over two steps, the sync word back
    at zero; (b) the per-sample head kernels (MMF_TAIL_HEAD_GEMV=1, tail.hip): the same values to
    fp32 reassociation.  L = 128 (the projection GEMM's column sums feed the pooling), B = 40 (a
    ragged last tile), dropout 0.3, a fully masked sample and a fractional mask."""
    import mmf_native as nat
    fusion, train_step = mods
    feats, mask, labels = _seq_batch(17)
    runs = {}
    for mode in ("one", "three", "gemv"):
        if mode == "gemv":
            monkeypatch.setenv("MMF_TAIL_HEAD_GEMV", "1")
        torch.manual_seed(3)
        model = fusion.HybridFusion({f"m{i}": 32 for i in range(M)}, hidden_dim=hidden, num_classes=5, num_heads=4,
                                    dropout=0.3).cuda()
        model._rng_state.copy_(torch.tensor([0xBEEF, 9], dtype=torch.int64))
        st = train_step.HybridTrainStep(model, [f.cuda() for f in feats], mask.cuda(), labels.cuda())
        nat.profile_begin()
        outs = []
        for _ in range(2):
            _three_calls(st, nat) if mode == "three" else st.forward_backward()
            torch.cuda.synchronize()
            outs.append([t.detach().cpu().clone() for t in (st.logits, st.losses, st.dlogits, st.fw, st.grad,
                                                            *st.dx, model._rng_state)])
        _, launches = nat.profile_end()
        names = [k for _, k, *_ in launches]
        if mode == "one":
            assert any(k.startswith("seq_head_kernel") and k.endswith(", 1>") for k in names), names
            assert not any(k.startswith(("cross_entropy_kernel", "tail_head", "l1_head_bwd")) for k in names), names
            assert int(st.sync.count_nonzero()) == 0
        elif mode == "three":
            assert any(k.startswith("seq_head_kernel") and k.endswith(", 0>") for k in names), names
            assert any(k.startswith("l1_head_bwd_kernel") for k in names), names
        else:
            assert any(k.startswith("tail_head_fwd_kernel") for k in names), names
            assert not any(k.startswith("seq_head_kernel") for k in names), names
        runs[mode] = outs
        monkeypatch.delenv("MMF_TAIL_HEAD_GEMV", raising=False)
    for step_a, step_b in zip(runs["one"], runs["three"]):
        for a, b in zip(step_a, step_b):
            assert torch.equal(a, b)
    for step_a, step_b in zip(runs["one"], runs["gemv"]):
        for a, b in zip(step_a, step_b):
            if a.dtype == torch.int64:
                assert torch.equal(a, b)
                continue
            tol = 1e-4 * max(float(b.abs().max()), 1e-6)
            assert float((a - b).abs().max()) <= tol, float((a - b).abs().max())


@pytest.mark.parametrize("M_,H_,C_,B_", [(4, 32, 7, 20), (2, 128, 3, 17)])
def test_tile_head_module_path_matches_per_sample_head(mods, M_, H_, C_, B_, monkeypatch):
    """The module path (HybridFusion.forward + autograd) with the 16-sample tile head against the
    per-sample head kernels (MMF_TAIL_HEAD_GEMV=1) on the same weights, inputs and dropout
    stream: four modalities (twelve pairs, the tile head's maxima) at H = 32 and two at H = 128,
    ragged tiles, train mode -- logits and every gradient to 1e-5 of the largest element + 1e-8
    (fp32 reassociation only)."""
    fusion, _ = mods
    g = torch.Generator().manual_seed(M_ * 7 + H_)
    feats = [torch.randn(B_, 128, 16, generator=g) for _ in range(M_)]
    mask = (torch.rand(B_, M_, generator=g) < 0.8).float()
    mask[2] = 0.0
    runs = []
    for gemv in (False, True):
        if gemv:
            monkeypatch.setenv("MMF_TAIL_HEAD_GEMV", "1")
        torch.manual_seed(5)
        model = fusion.HybridFusion({f"m{i}": 16 for i in range(M_)}, hidden_dim=H_, num_classes=C_, num_heads=4,
                                    dropout=0.2).cuda().train()
        model._rng_state.copy_(torch.tensor([0xABC, 1], dtype=torch.int64))
        xs = {f"m{i}": f.cuda().requires_grad_(True) for i, f in enumerate(feats)}
        logits = model(xs, mask.cuda())
        (logits * torch.linspace(-1, 1, C_, device="cuda")).sum().backward()
        torch.cuda.synchronize()
        runs.append([logits.detach().cpu()] + [xs[k].grad.cpu() for k in sorted(xs)] +
                    [p.grad.cpu() for _, p in sorted(model.named_parameters())])
        monkeypatch.delenv("MMF_TAIL_HEAD_GEMV", raising=False)
    for a, b in zip(*runs):
        # (+1e-8: gradients that cancel to ~1e-10 -- the gating biases, whose softmax-backward
        # terms sum to zero over the modalities -- carry only rounding noise)
        tol = 1e-5 * float(b.abs().max()) + 1e-8
        assert float((a - b).abs().max()) <= tol, (float((a - b).abs().max()), tol)


def test_l1_poll_timeout_surfaces_and_recovers(mods, monkeypatch):
    """The launch-lean L = 1 step's bounded waits: with the poll
    bound at 0 (MMF_L1_POLL_BOUND, read per launch) every pair workgroup that waits for its tile's
    head gives up at once.  The step must (a) not hang, (b) report it: the loss reads NaN and
    check_status() / reading .loss raise RuntimeError, (c) leave the sync buffer clean (the
    weight-gradient launch resets the tile words, check_status clears the error word), and (d) with
    the default bound again, the next call on the same buffers equals a fresh step object's call bit
    for bit (logits, loss, dlogits, weights, every gradient, dX, the dropout stream).  A fused step
    (step(): clip partials from the train step) with the timeout reports an infinite norm and a zero
    clip coefficient (the update applied a zero gradient), with clipping on and off."""
    import mmf_native as nat
    fusion, train_step = mods
    feats, mask, labels = _batch(19)
    feats = [f[:, 0] for f in feats]

    def build(clip=1.0):
        model = _model(fusion, 0.3).cuda()
        model._rng_state.copy_(torch.tensor([0x5EED, 3], dtype=torch.int64))
        return train_step.HybridTrainStep(model, [f.cuda() for f in feats], mask.cuda(), labels.cuda(),
                                          gradient_clip_norm=clip)

    def outs(st):
        return [t.detach().cpu().clone() for t in (st.logits, st.losses, st.dlogits, st.fw, st.grad, *st.dx,
                                                    st.rng)]

    st = build()
    monkeypatch.setenv("MMF_L1_POLL_BOUND", "0")
    nat.profile_begin()
    st.forward_backward()
    torch.cuda.synchronize()
    _, launches = nat.profile_end()
    assert any(k.startswith("l1_fwd_loss_kernel") for _, k, *_ in launches)
    assert math.isnan(float(st.losses[0].item()))
    words = st.sync.view(torch.int32)
    assert int(words.count_nonzero()) == 1 and int(words[7].item()) == 1   # the error word (1 tile x 7
    # tile words before it) alone: the weight-gradient launch reset the tile words
    with pytest.raises(RuntimeError, match="gave up waiting"):
        st.check_status()
    assert int(st.sync.count_nonzero()) == 0
    st.check_status()   # cleared
    monkeypatch.delenv("MMF_L1_POLL_BOUND")
    st.rng.copy_(torch.tensor([0x5EED, 3], dtype=torch.int64))
    st.forward_backward()
    torch.cuda.synchronize()
    ref = build()
    ref.forward_backward()
    torch.cuda.synchronize()
    for a, b in zip(outs(st), outs(ref)):
        assert torch.equal(a, b)
    assert math.isfinite(float(st.loss.item()))   # (.loss checks the status: nothing pending)
    # the fused step under a timeout: norm inf, coefficient 0, reported on .loss
    monkeypatch.setenv("MMF_L1_POLL_BOUND", "0")
    st.step()
    torch.cuda.synchronize()
    assert math.isinf(float(st.grad_norm.item())) and float(st.clip_coef.item()) == 0.0
    with pytest.raises(RuntimeError, match="gave up waiting"):
        st.loss
    monkeypatch.delenv("MMF_L1_POLL_BOUND")
    st.step()
    torch.cuda.synchronize()
    assert math.isfinite(float(st.loss.item())) and int(st.sync.count_nonzero()) == 0
    # clipping off (gradient_clip_norm = 0): the incomplete gradient still stays out of
    # the update -- coefficient 0, and the first AdamW step with a zero gradient moves the weights by
    # the decoupled weight decay alone
    st0 = build(clip=0.0)
    flat0 = st0.flat.clone()
    monkeypatch.setenv("MMF_L1_POLL_BOUND", "0")
    st0.step()
    torch.cuda.synchronize()
    monkeypatch.delenv("MMF_L1_POLL_BOUND")
    assert math.isinf(float(st0.grad_norm.item())) and float(st0.clip_coef.item()) == 0.0
    torch.testing.assert_close(st0.flat, flat0 * (1 - 1e-3 * 1e-4), rtol=0, atol=1e-6)   # (a gradient step: ~1e-3)
    with pytest.raises(RuntimeError, match="gave up waiting"):
        st0.loss


@pytest.mark.parametrize("seq", [False, True])
def test_plan_switch_after_sizing_is_refused(mods, seq, monkeypatch):
    """The buffer contract: HybridTrainStep sizes `saved` / `workspace` once.
    A plan switch set afterwards (MMF_PSTORE=1, whose stored probabilities need a larger `saved` --
    the round-5 illegal-address fault class) makes step() raise RuntimeError before any launch; a
    shortened declared capacity does too; with the switch gone the step runs and matches a fresh
    step's gradient bit for bit."""
    fusion, train_step = mods
    monkeypatch.delenv("MMF_PSTORE", raising=False)
    feats, mask, labels = _batch(5)
    if not seq:
        feats = [f[:, 0] for f in feats]
    model = _model(fusion, 0.1).cuda()
    st = train_step.HybridTrainStep(model, [f.cuda() for f in feats], mask.cuda(), labels.cuda())
    rng0 = model._rng_state.clone()
    monkeypatch.setenv("MMF_PSTORE", "1")
    with pytest.raises(RuntimeError, match="plan switches"):
        st.step()
    monkeypatch.delenv("MMF_PSTORE")
    d = st.plan.desc
    d.saved_capacity -= 4096
    with pytest.raises(RuntimeError, match="saved buffer too small"):
        st.step()
    d.saved_capacity += 4096
    cap = d.workspace_capacity
    d.workspace_capacity = 256
    with pytest.raises(RuntimeError, match="workspace too small"):
        st.step()
    d.workspace_capacity = cap
    torch.cuda.synchronize()
    assert torch.equal(model._rng_state, rng0)          # nothing ran
    st.forward_backward()
    ref_model = _model(fusion, 0.1).cuda()
    ref = train_step.HybridTrainStep(ref_model, [f.cuda() for f in feats], mask.cuda(), labels.cuda())
    ref_model._rng_state.copy_(rng0)
    ref.forward_backward()
    torch.cuda.synchronize()
    assert torch.equal(st.grad, ref.grad)


@pytest.mark.parametrize("seq", [True])
def test_dx_chained_into_dz_is_bit_exact(mods, seq, monkeypatch):
    """MMF_DX_CHAIN=1 (opt-in): dX_m computed by the dZ launch's workgroups right after
    their dZ_m row tiles (gemm_lds_chain_kernel) -- the same tiles, k order and epilogue as the
    separate dX launch, so logits, every parameter gradient and dX agree bit for bit."""
    import mmf_native as nat
    fusion, train_step = mods
    feats, mask, labels = _batch(23)
    runs = []
    for chain in (False, True):
        if chain:
            monkeypatch.setenv("MMF_DX_CHAIN", "1")
        model = _model(fusion, 0.3).cuda()
        model._rng_state.copy_(torch.tensor([0x5EED, 9], dtype=torch.int64))
        st = train_step.HybridTrainStep(model, [f.cuda() for f in feats], mask.cuda(), labels.cuda())
        nat.profile_begin()
        st.forward_backward()
        torch.cuda.synchronize()
        _, launches = nat.profile_end()
        names = [k for _, k, *_ in launches]
        assert any(k.startswith("gemm_lds_chain_kernel") for k in names) == chain, names
        runs.append([t.detach().cpu().clone() for t in (st.logits, st.grad, *st.dx)])
        monkeypatch.delenv("MMF_DX_CHAIN", raising=False)
    for a, b in zip(*runs):
        assert torch.equal(a, b)
