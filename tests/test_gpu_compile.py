"""torch.compile wrapping of the drop-in module: the reference's
trainer may wrap the fusion model with torch.compile (config compile_mode);
the module must keep working under it, give the eager results, and its state
dict must round-trip with the `_orig_mod.` prefix compile adds.

backend="eager" exercises TorchDynamo's capture of the module (graph breaks
at the HIP library calls) without needing a code generator."""
import pytest
import torch

from cases import HYBRID_CASES, hybrid_inputs, hybrid_state

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fusion_mod(pkg_on_path):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    import fusion
    return fusion


def test_compiled_module_matches_eager(fusion_mod):
    case = next(c for c in HYBRID_CASES if c.name == "seq_c2_b3")
    sd = hybrid_state(case.names, case.dims, case.hidden, case.classes, case.seed)
    model = fusion_mod.HybridFusion({m: case.dims[m] for m in case.names}, hidden_dim=case.hidden,
                                    num_classes=case.classes, num_heads=case.heads, dropout=0.1)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model = model.cuda().eval()
    feats_np, mask_np, grad_np = hybrid_inputs(case)
    mask = torch.from_numpy(mask_np).cuda()
    g = torch.from_numpy(grad_np).cuda()

    def run(m):
        feats = {k: torch.from_numpy(v).cuda().requires_grad_(True) for k, v in feats_np.items()}
        for p in m.parameters():
            p.grad = None
        out = m(feats, mask)
        (out * g).sum().backward()
        torch.cuda.synchronize()
        return out.detach().clone(), {k: f.grad.clone() for k, f in feats.items()}, \
            {n.replace("_orig_mod.", ""): p.grad.clone() for n, p in m.named_parameters()}

    ref_out, ref_dx, ref_dw = run(model)
    torch._dynamo.reset()
    compiled = torch.compile(model, backend="eager")
    out, dx, dw = run(compiled)
    assert torch.equal(out, ref_out)
    for k in ref_dx:
        assert torch.equal(dx[k], ref_dx[k]), k
    for n in ref_dw:
        assert torch.equal(dw[n], ref_dw[n]), n
    keys = list(compiled.state_dict().keys())
    assert all(k.startswith("_orig_mod.") for k in keys)
    plain = fusion_mod.HybridFusion({m: case.dims[m] for m in case.names}, hidden_dim=case.hidden,
                                    num_classes=case.classes, num_heads=case.heads, dropout=0.1).cuda()
    plain.load_state_dict({k[len("_orig_mod."):]: v for k, v in compiled.state_dict().items()})
    torch._dynamo.reset()
