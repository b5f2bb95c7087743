"""C5's benchmarked path against the oracle (VERDICT r04 "next" #3).

bench.py --workload c5 --precision medium times BASELINE.json configs[4]: six modalities of
L = 512, D = H = 256, 4 heads (head_dim 64), 30 ordered pairs, dropout 0.1 in train mode, modality
masks (keep 0.9, >= 1 kept per row, 1 % all-masked rows: src/data.py:326-341 semantics, SURVEY
§8d), matmul precision "medium" (config/base.yaml:80), one hipGraph replay of
train_step.HybridTrainStep per step.  This builds that step exactly as bench.py does (its WORKLOADS /
make_inputs, torch.manual_seed(0) weights) at a batch the CPU oracle runs in seconds (B = 4: one
all-masked row), checks from the library's launch records that the benchmarked kernel set ran --
the one-pass long-key attention kernels, the Q / K projection GEMM on bf16 operand copies, the
keep-word kernel (more than 16 pairs: drawn on the side stream) -- replays the captured graph once
and compares logits, the loss, every input gradient and every parameter gradient with the oracle
under the replayed Philox masks (tests/_philox.py), with the bf16 bounds of tests/test_gpu_bf16.py:
logits within 3e-2 of the largest logit with argmax agreement, every gradient
||got - ref|| <= max(3e-2 ||ref||, 4 ||emu - ref||, 3e-3 S) where emu is the oracle with bf16-rounded
matmul operands (forward and backward) and S the largest reference gradient norm.
"""
import os
import sys

import pytest
import torch

from _philox import mask_provider
from _util import bf16_matmul_mode
from test_gpu_bf16 import group_scale, logits_ok, norm_ok

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

EXPECT = ["attn_poolL_fwd_fused_bf16<true", "attn_poolL_bwd_fused_bf16<true, ", "gemm_wsr_b16_kernel",
          "gemm_lds_kernel<1, 1, 32, 3, 1, 2, 1>", "gemm_lds_kernel<0, 1, 32, 3, 1, 3>",
          "gemm_lds_kernel<0, 0, 32, 3, 1, 1>", "gemm_lds_kernel<0, 1, 32, 3, 1, 3, 1>", "pool_e_mfma_kernel",
          "pool_u_mfma_kernel", "pool_dpbar_mfma_kernel", "cvt_bf16_kernel", "attn_keep_words_kernel"]


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


def test_c5_benchmark_step_matches_oracle(env):
    bench, fusion, nat, train_step = env
    from oracle.hybrid_cpu import cross_entropy_ls, hybrid_forward
    w = bench.WORKLOADS["c5"]
    B = 4
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("medium")
    try:
        dev = torch.device("cuda", 0)
        torch.manual_seed(0)
        names = [f"m{i}" for i in range(w["M"])]
        model = fusion.HybridFusion({n: w["D"] for n in names}, hidden_dim=w["H"], num_classes=w["C"],
                                    num_heads=w["heads"], dropout=0.1).to(dev)
        feats, mask, labels = bench.make_inputs(w, B, 42, dev)
        m_cpu = mask.cpu()
        assert bool((m_cpu.sum(1) == 0).any()) and bool((m_cpu == 0).any())   # an all-masked row, masked keys
        step = train_step.HybridTrainStep(model, feats, mask, labels)
        nat.profile_begin()
        step.forward_backward()
        torch.cuda.synchronize()
        _, launches = nat.profile_end()
        ran = [k for _, k, *_ in launches]
        for k in EXPECT:
            assert any(r.startswith(k) for r in ran), (k, sorted(set(ran)))
        assert not any(r.startswith(("attn_poolL_dq", "attn_poolL_lse", "attn_poolL_colsum")) for r in ran), ran

        step.capture()
        seed, offset = (int(v) for v in step.rng.tolist())
        params_cpu = {n: p.detach().cpu().clone() for n, p in model.named_parameters()}
        step.graph.replay()                 # one benchmarked step: gradients at the pre-update weights
        torch.cuda.synchronize()
        assert int(step.rng[1].item()) == offset + 1
    finally:
        torch.set_float32_matmul_precision(prev)

    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))

    def oracle(bf16):
        params = {k: v.clone().requires_grad_(True) for k, v in params_cpu.items()}
        xs = {n: f.detach().cpu().clone().requires_grad_(True) for n, f in zip(names, feats)}

        def run():
            logits, _ = hybrid_forward(params, names, xs, m_cpu, w["heads"], p=0.1, train=True,
                                       gen=mask_provider(seed, offset, 0.1))
            loss = cross_entropy_ls(logits, labels.cpu())
            loss.backward()
            return logits.detach(), loss.detach()
        if bf16:
            with bf16_matmul_mode():
                lg, ls = run()
        else:
            lg, ls = run()
        return lg, ls, {n: xs[n].grad for n in names}, {n: params[n].grad for n in params}

    ref, rloss, rdx, rdw = oracle(False)
    _, _, edx, edw = oracle(True)
    ok, e = logits_ok(step.logits.cpu(), ref)
    assert ok, e
    assert abs(float(step.loss.item()) - float(rloss)) <= 3e-2 * max(1.0, abs(float(rloss)))
    S = group_scale(list(rdx.values()) + [g for g in rdw.values() if g is not None])
    for i, n in enumerate(names):
        ok, e = norm_ok(step.dx[i].cpu(), rdx[n], edx[n], S)
        assert ok, (n, e)
    grads = dict(step.named_grads())
    for n, g in grads.items():
        ref_g = rdw[n] if rdw[n] is not None else torch.zeros_like(params_cpu[n])
        emu_g = edw[n] if edw[n] is not None else torch.zeros_like(params_cpu[n])
        ok, e = norm_ok(g.cpu(), ref_g, emu_g, S)
        assert ok, (n, e)
