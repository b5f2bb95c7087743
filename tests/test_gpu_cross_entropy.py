"""mmf_ops.cross_entropy (head.hip cross_entropy_kernel behind torch's functional signature; the
module path's loss in bench.py) against torch.nn.functional.cross_entropy(label_smoothing) with
reduction "mean" (src/train.py:185-186, 310): loss and d loss / d logits to fp32 rounding, with
a non-unit upstream gradient, at the C2 shape and a ragged one."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops(pkg_on_path):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    import mmf_native
    import mmf_ops
    mmf_native.lib()
    return mmf_ops


@pytest.mark.parametrize("B,C,eps", [(256, 5, 0.05), (37, 11, 0.0), (3, 25, 0.2)])
def test_cross_entropy_matches_torch(ops, B, C, eps):
    g = torch.Generator().manual_seed(B * 131 + C)
    logits = (3 * torch.randn(B, C, generator=g)).cuda()
    labels = torch.randint(0, C, (B,), generator=g).cuda()
    a = logits.clone().requires_grad_(True)
    b = logits.clone().requires_grad_(True)
    la = ops.cross_entropy(a, labels, label_smoothing=eps)
    lb = torch.nn.functional.cross_entropy(b, labels, label_smoothing=eps)
    (la * 1.7).backward()
    (lb * 1.7).backward()
    torch.cuda.synchronize()
    assert la.shape == lb.shape == ()
    torch.testing.assert_close(la, lb, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(a.grad, b.grad, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("eps", [0.05, 0.0])
def test_ignore_index_rows_match_torch(ops, eps):
    """Rows labelled -100 (torch's default ignore_index): no loss, zero gradient, the mean over the
    remaining rows -- as torch.nn.functional.cross_entropy(label_smoothing) computes it."""
    g = torch.Generator().manual_seed(99)
    B, C = 50, 7
    logits = (2 * torch.randn(B, C, generator=g)).cuda()
    labels = torch.randint(0, C, (B,), generator=g)
    labels[[0, 7, 8, 31]] = -100
    labels = labels.cuda()
    a = logits.clone().requires_grad_(True)
    b = logits.clone().requires_grad_(True)
    la = ops.cross_entropy(a, labels, label_smoothing=eps)
    lb = torch.nn.functional.cross_entropy(b, labels, label_smoothing=eps)
    la.backward()
    lb.backward()
    torch.cuda.synchronize()
    torch.testing.assert_close(la, lb, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(a.grad, b.grad, rtol=1e-5, atol=1e-7)
    assert float(a.grad[7].abs().max()) == 0.0


def test_out_of_range_label_gives_nan_not_a_stray_read(ops):
    """A label outside [0, C) that is not ignored (torch raises) makes the loss NaN; the kernel never
    indexes the logits with it."""
    logits = torch.randn(6, 4).cuda()
    for bad in (4, 1 << 40, -3):
        labels = torch.tensor([0, 1, bad, 3, 2, 1]).cuda()
        loss = ops.cross_entropy(logits, labels, label_smoothing=0.05)
        torch.cuda.synchronize()
        assert torch.isnan(loss).item()
