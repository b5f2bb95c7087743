"""torch.compile of the drop-in modules (SURVEY §8b "C-ABI to export").

The reference wraps its fusion model and encoders in
torch.compile(backend="inductor", mode="reduce-overhead") (src/train.py:193-231,
config/base.yaml:76-79).  The library's entry points are torch custom operators with
fake kernels and autograd formulas (mmf_ops.py), so TorchDynamo traces each module
into ONE graph (fullgraph=True: a graph break would raise), AOTAutograd sees the
forward and backward operators, and "reduce-overhead" replays the step as a HIP graph.
The compiled forward + backward must equal eager bit for bit (the same kernels run),
in eval and in train mode (the device dropout state advances identically), and the
compiled module's state dict round-trips with the `_orig_mod.` prefix.
"""
import pytest
import torch

from cases import CMA_CASES, HYBRID_CASES, cma_inputs, cma_state, hybrid_inputs, hybrid_state

pytestmark = pytest.mark.gpu
STEPS = 3   # cudagraph trees record on the first replays: compare every step


@pytest.fixture(scope="module")
def mods(pkg_on_path):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    import attention
    import encoders
    import fusion
    import harness
    return fusion, attention, encoders, harness


def _hybrid(fusion, case, p=0.1):
    sd = hybrid_state(case.names, case.dims, case.hidden, case.classes, case.seed)
    model = fusion.HybridFusion({m: case.dims[m] for m in case.names}, hidden_dim=case.hidden,
                                num_classes=case.classes, num_heads=case.heads, dropout=p)
    model.traceable = True   # the fully traceable form (custom operators; the default is opaque)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return model.cuda()


def _run_steps(m, owner, feats_np, mask, g, rng0):
    """STEPS fwd+bwd calls from the same device dropout state; clones of every output / grad."""
    owner._rng_state.copy_(rng0)
    outs = []
    for _ in range(STEPS):
        feats = {k: torch.from_numpy(v).cuda().requires_grad_(True) for k, v in feats_np.items()}
        for prm in owner.parameters():
            prm.grad = None
        out = m(feats, mask)
        (out * g).sum().backward()
        torch.cuda.synchronize()
        outs.append((out.detach().clone(), {k: f.grad.clone() for k, f in feats.items()},
                     {n: prm.grad.clone() for n, prm in owner.named_parameters()}, owner._rng_state.clone()))
    return outs


@pytest.mark.parametrize("train", [False, True], ids=["eval", "train"])
@pytest.mark.parametrize("case_name", ["seq_c2_b3", "tiny_l1"])
def test_hybrid_compile_reduce_overhead_fullgraph_bit_identical(mods, case_name, train):
    fusion = mods[0]
    case = next(c for c in HYBRID_CASES if c.name == case_name)
    model = _hybrid(fusion, case)
    model.train(train)
    feats_np, mask_np, grad_np = hybrid_inputs(case)
    mask, g = torch.from_numpy(mask_np).cuda(), torch.from_numpy(grad_np).cuda()
    rng0 = torch.tensor([0x5EED, 11], dtype=torch.int64)
    ref = _run_steps(model, model, feats_np, mask, g, rng0)
    torch._dynamo.reset()
    from torch._dynamo.utils import counters
    counters.clear()
    compiled = torch.compile(model, mode="reduce-overhead", fullgraph=True)
    got = _run_steps(compiled, model, feats_np, mask, g, rng0)
    # the HIP graphs are really used: inductor skipped cudagraphs for no graph (a skip -- e.g. a
    # mutated non-static input -- would leave the custom operators' host code running every call)
    assert not counters["inductor"].get("cudagraph_skips"), dict(counters["inductor"])
    for step, ((ro, rdx, rdw, rr), (co, cdx, cdw, cr)) in enumerate(zip(ref, got)):
        assert torch.equal(co, ro), step
        assert torch.equal(cr, rr), step            # the dropout state advanced the same way
        for k in rdx:
            assert torch.equal(cdx[k], rdx[k]), (step, k)
        for n in rdw:
            assert torch.equal(cdw[n], rdw[n]), (step, n)
    if train:
        assert not torch.equal(ref[0][0], ref[1][0])   # dropout masks differ between steps
    keys = list(compiled.state_dict().keys())
    assert all(k.startswith("_orig_mod.") for k in keys)
    plain = _hybrid(fusion, case)
    plain.load_state_dict({k[len("_orig_mod."):]: v for k, v in compiled.state_dict().items()})
    torch._dynamo.reset()


def test_hybrid_compile_return_attention_and_adaptive_weights(mods):
    """return_attention (maps + fusion weights) and the public compute_adaptive_weights trace too."""
    fusion = mods[0]
    case = next(c for c in HYBRID_CASES if c.name == "seq_equal")
    model = _hybrid(fusion, case).eval()
    feats_np, mask_np, _ = hybrid_inputs(case)
    feats = {k: torch.from_numpy(v).cuda() for k, v in feats_np.items()}
    mask = torch.from_numpy(mask_np).cuda()
    ref_l, ref_i = model(feats, mask, return_attention=True)
    torch._dynamo.reset()
    fn = torch.compile(lambda f, m: model(f, m, return_attention=True), fullgraph=True)
    l, info = fn(feats, mask)
    assert torch.equal(l, ref_l) and torch.equal(info["fusion_weights"], ref_i["fusion_weights"])
    for k in ref_i["attention_maps"]:
        assert torch.equal(info["attention_maps"][k], ref_i["attention_maps"][k]), k
    pooled = {m: torch.randn(case.batch, case.hidden, device="cuda", requires_grad=True) for m in case.names}
    aw_ref = model.compute_adaptive_weights(pooled, mask)
    aw_ref.sum().backward()
    ref_g = {m: t.grad.clone() for m, t in pooled.items()}
    for t in pooled.values():
        t.grad = None
    torch._dynamo.reset()
    aw = torch.compile(model.compute_adaptive_weights, fullgraph=True)(pooled, mask)
    aw.sum().backward()
    assert torch.equal(aw, aw_ref)
    for m in case.names:
        assert torch.equal(pooled[m].grad, ref_g[m]), m
    torch._dynamo.reset()


@pytest.mark.parametrize("case_name", ["cma_3d_mask2d", "cma_2d_mask1d", "cma_3d_wide_hd128"])
def test_cma_compile_fullgraph_bit_identical(mods, case_name):
    attention = mods[1]
    case = next(c for c in CMA_CASES if c.name == case_name)
    model = attention.CrossModalAttention(case.query_dim, case.key_dim, hidden_dim=case.hidden,
                                          num_heads=case.heads, dropout=0.1)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in cma_state(case.query_dim, case.key_dim, case.hidden,
                                                                        case.seed).items()})
    model = model.cuda().train()
    q, k, v, mask, grad = cma_inputs(case)
    mt = torch.from_numpy(mask).cuda() if mask is not None else None
    gt = torch.from_numpy(grad).cuda()

    def run(m):
        model._rng_state.copy_(torch.tensor([77, 3], dtype=torch.int64))
        res = []
        for _ in range(STEPS):
            qt, kt, vt = (torch.from_numpy(a).cuda().requires_grad_(True) for a in (q, k, v))
            for prm in model.parameters():
                prm.grad = None
            att, w = m(qt, kt, vt, mt)
            (att * gt).sum().backward()
            torch.cuda.synchronize()
            res.append([att.detach().clone(), w.clone(), qt.grad.clone(), kt.grad.clone(), vt.grad.clone()]
                       + [prm.grad.clone() for prm in model.parameters()])
        return res

    ref = run(model)
    torch._dynamo.reset()
    got = run(torch.compile(model, mode="reduce-overhead", fullgraph=True))
    for a, b in zip(ref, got):
        for x, y in zip(a, b):
            assert torch.equal(x, y)
    torch._dynamo.reset()


def test_encoders_and_full_model_compile_fullgraph(mods):
    """The reference compiles each encoder too (src/train.py:203-214): SequenceEncoder (HIP LSTM
    recurrence), FrameEncoder (HIP attention pooling), and the whole encoders -> LayerNorm ->
    HybridFusion model, fullgraph, equal to eager."""
    _, _, encoders, harness = mods
    torch.manual_seed(4)
    seq = encoders.SequenceEncoder(17, hidden_dim=64, output_dim=32, num_layers=2, dropout=0.0).cuda()
    frame = encoders.FrameEncoder(48, hidden_dim=32, output_dim=32, dropout=0.0).cuda()
    x = torch.randn(3, 20, 17, device="cuda", requires_grad=True)
    fr = torch.randn(3, 9, 48, device="cuda", requires_grad=True)
    fmask = torch.ones(3, 9, device="cuda")
    fmask[1, 4:] = 0
    for mod, args in ((seq, (x,)), (frame, (fr, fmask))):
        ref = mod(*args)
        ref.square().sum().backward()
        ref_g = [a.grad.clone() for a in args if a.requires_grad] + [p.grad.clone() for p in mod.parameters()]
        for a in args:
            a.grad = None
        for p in mod.parameters():
            p.grad = None
        torch._dynamo.reset()
        out = torch.compile(mod, fullgraph=True)(*args)
        out.square().sum().backward()
        got_g = [a.grad.clone() for a in args if a.requires_grad] + [p.grad.clone() for p in mod.parameters()]
        # the encoders' torch ops around the HIP operators (input projections, the bias sum
        # b_ih + b_hh, the output Linear) become inductor kernels whose reduction order is not
        # eager's: equal to fp32 rounding, not bit for bit (the HIP operators are the same launches)
        torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-6, msg=type(mod).__name__)
        for a, b in zip(got_g, ref_g):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6, msg=type(mod).__name__)
    # encoders -> LayerNorm -> HybridFusion (config/base.yaml's PAMAP2 model, smaller hidden)
    enc = {m: {"type": "sequence", "input_dim": 17 if m != "heart_rate" else 1, "encoder_type": "lstm",
               "num_layers": 1} for m in ("imu_hand", "imu_chest", "heart_rate")}
    cfg = {"dataset": {"modalities": list(enc), "num_classes": 25},
           "model": {"fusion_type": "hybrid", "hidden_dim": 64, "output_dim": 32, "num_heads": 4,
                     "dropout": 0.0, "layer_norm": True, "encoders": enc}}
    model = harness.MultimodalFusionModel.from_config(cfg).cuda().eval()
    model.fusion_model.traceable = True   # (fullgraph: the traceable form of HybridFusion)
    feats = {m: torch.randn(2, 30, enc[m]["input_dim"], device="cuda") for m in enc}
    mask = torch.tensor([[1.0, 1.0, 1.0], [1.0, 0.0, 1.0]], device="cuda")
    ref = model(feats, mask)
    torch._dynamo.reset()
    got = torch.compile(model, fullgraph=True)(feats, mask)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
    torch._dynamo.reset()


@pytest.mark.parametrize("case_name", ["seq_c2_b3", "tiny_l1"])
def test_hybrid_compile_default_is_opaque_and_bit_identical(mods, case_name):
    """The default (HybridFusion.traceable = False) under the reference's own call,
    torch.compile(model, mode="reduce-overhead") without fullgraph (src/train.py:101-122): TorchDynamo
    runs the module as one opaque native step -- no graph is compiled for it -- and forward +
    backward (the grad-sink path) equal eager bit for bit over several steps, train mode."""
    fusion = mods[0]
    case = next(c for c in HYBRID_CASES if c.name == case_name)
    model = _hybrid(fusion, case)
    model.traceable = False
    model.train()
    feats_np, mask_np, grad_np = hybrid_inputs(case)
    mask, g = torch.from_numpy(mask_np).cuda(), torch.from_numpy(grad_np).cuda()
    rng0 = torch.tensor([0x5EED, 11], dtype=torch.int64)
    ref = _run_steps(model, model, feats_np, mask, g, rng0)
    torch._dynamo.reset()
    from torch._dynamo.utils import counters
    counters.clear()
    compiled = torch.compile(model, mode="reduce-overhead")
    got = _run_steps(compiled, model, feats_np, mask, g, rng0)
    for step, ((ro, rdx, rdw, rr), (co, cdx, cdw, cr)) in enumerate(zip(ref, got)):
        assert torch.equal(co, ro) and torch.equal(cr, rr), step
        for k in rdx:
            assert torch.equal(cdx[k], rdx[k]), (step, k)
        for n in rdw:
            assert torch.equal(cdw[n], rdw[n]), (step, n)
    assert not counters["inductor"].get("cudagraph_recorded_non_static_inputs"), dict(counters["inductor"])
    torch._dynamo.reset()
