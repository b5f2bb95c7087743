"""The exact benchmark workload, at full size, against the oracle (src/fusion.py:331-427).

bench.py times C2 (BASELINE.json configs[1]): B = 256, three modalities of L = 128, D = H = 128,
4 heads, dropout 0.1 in train mode, fp32 ("highest"), one hipGraph replay of
train_step.HybridTrainStep per step (fwd -> CE(label_smoothing 0.05) -> bwd -> clip -> AdamW),
with the attention keep words drawn by the input-mask kernel.  This builds that step exactly as
bench.py does (its WORKLOADS / make_inputs, torch.manual_seed(0) weights), checks from the
library's launch records that the benchmarked instantiations ran, replays the captured graph
once and compares logits, the loss, every input gradient and every parameter gradient with the
CPU oracle under the replayed Philox masks (tests/_philox.py) at 1e-3 of each tensor's largest
element.  c2_l1 (the reference's own 2-D inputs, B = 256, train mode) the same way on the
single-key plan, whose query / key projection gradients must be exact zeros.
"""
import os
import sys

import pytest
import torch

from _philox import mask_provider
from _util import close

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def env(pkg_on_path):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    import fusion
    import mmf_native
    import train_step
    return bench, fusion, mmf_native, train_step


EXPECT = {   # the benchmarked kernel instantiations (bench.py's kernel table names them)
    "c2": ["mask_dropout_rows_kernel", "attn_pool_fwd_lean<32, 0, true, false, true>",
           "attn_pool_bwd_fused_lean<32, 0, false>", "gemm_wsr_kernel<0>"],
    # the launch-lean single-key step (csrc/l1.hip): forward + loss + head backward in one launch
    # (and the key-modality backward: two launches per step before the optimizer)
    "c2_l1": ["l1_fwd_loss_kernel<128>", "l1_wgrad_kernel"],
}


@pytest.mark.parametrize("workload", ["c2", "c2_l1"])
def test_benchmark_step_matches_oracle(env, workload):
    bench, fusion, mmf_native, train_step = env
    from oracle.hybrid_cpu import cross_entropy_ls, hybrid_forward
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("highest")
    try:
        w = bench.WORKLOADS[workload]
        dev = torch.device("cuda", 0)
        torch.manual_seed(0)
        names = [f"m{i}" for i in range(w["M"])]
        model = fusion.HybridFusion({n: w["D"] for n in names}, hidden_dim=w["H"], num_classes=w["C"],
                                    num_heads=w["heads"], dropout=0.1).to(dev)
        feats, mask, labels = bench.make_inputs(w, w["B"], 42, dev)
        step = train_step.HybridTrainStep(model, feats, mask, labels)

        # the benchmarked instantiations (eager profile step, as bench.py's kernel table)
        mmf_native.profile_begin()
        step.forward_backward()
        torch.cuda.synchronize()
        _, launches = mmf_native.profile_end()
        ran = {k for _, k, *_ in launches}
        for k in EXPECT[workload]:
            assert any(r == k or r.startswith(k) for r in ran), (k, sorted(ran))
        assert "attn_keep_words_kernel" not in ran, sorted(ran)   # the fold, not the side stream

        step.capture()                       # (its warm-up call advances the stream once more)
        seed, offset = (int(v) for v in step.rng.tolist())
        params_cpu = {n: p.detach().cpu().clone() for n, p in model.named_parameters()}
        step.graph.replay()                  # one benchmarked step: grads at the pre-update weights
        torch.cuda.synchronize()
        assert int(step.rng[1].item()) == offset + 1
    finally:
        torch.set_float32_matmul_precision(prev)

    params = {k: v.clone().requires_grad_(True) for k, v in params_cpu.items()}
    xs = {n: f.detach().cpu().clone().requires_grad_(True) for n, f in zip(names, feats)}
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    logits, _ = hybrid_forward(params, names, xs, mask.cpu(), w["heads"], p=0.1, train=True,
                               gen=mask_provider(seed, offset, 0.1))
    loss = cross_entropy_ls(logits, labels.cpu())
    loss.backward()

    assert close(step.logits.cpu(), logits.detach(), 1e-3, 1e-6 * float(logits.detach().abs().max()))
    assert abs(float(step.loss.item()) - float(loss.detach())) <= 1e-5 * max(1.0, abs(float(loss.detach())))
    grads = dict(step.named_grads())
    scale = max([float(p.grad.abs().max()) for p in params.values()] +
                [float(x.grad.abs().max()) for x in xs.values()])
    for i, n in enumerate(names):
        assert close(step.dx[i].cpu(), xs[n].grad, 1e-3, 1e-5 * scale), f"dx/{n}"
    for n, p in params.items():
        g = grads[n].cpu()
        if max(w["L"]) == 0 and (".query_proj." in n or ".key_proj." in n):
            assert torch.all(g == 0), n      # softmax over one key: exact zeros (src/attention.py:118-129)
            continue
        assert close(g, p.grad, 1e-3, 1e-5 * scale), n
