#!/usr/bin/env python3
"""C2 benchmark step against the CPU oracle over several dropout seeds (diagnostic).

The module's Philox seed depends on how many modules the process constructed before it
(attention._new_rng_state), so test order changes the dropout masks a test sees.  This runs the
test_gpu_headline comparison for `--seeds` consecutive constructions and prints, per seed, the
worst |got - ref| / bound over logits, dX and every parameter gradient (bound = 1e-3 max|ref| +
1e-5 scale, as the test), and the tensors over 1: against the plain oracle and against the oracle
given the device's ReLU' decisions for pre-activations within rounding of 0
(tests/_util.device_relu_gates, as the test), with the number of such elements per layer.
usage (box): python scripts/seed_sweep.py [--seeds 8] [--workload c2]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "multimodal-sensor-fusion-with-attention-rajeevatla_amd")
for p in (PKG, ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

import bench  # noqa: E402
import fusion  # noqa: E402
import train_step  # noqa: E402
from _philox import mask_provider  # noqa: E402
from _util import device_relu_gates  # noqa: E402
from oracle.hybrid_cpu import cross_entropy_ls, hybrid_forward  # noqa: E402


def ratio(got, ref, atol):
    """worst |got - ref| / bound and the count over"""
    got, ref = got.double().cpu(), ref.double().cpu()
    bound = 1e-3 * float(ref.abs().max()) + atol
    d = (got - ref).abs()
    return float(d.max()) / bound, int((d > bound).sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=8)
    ap.add_argument("--workload", default="c2")
    a = ap.parse_args()
    torch.set_float32_matmul_precision("highest")
    torch.set_num_threads(16)
    w = bench.WORKLOADS[a.workload]
    dev = torch.device("cuda", 0)
    names = [f"m{i}" for i in range(w["M"])]
    for k in range(a.seeds):
        torch.manual_seed(0)
        model = fusion.HybridFusion({n: w["D"] for n in names}, hidden_dim=w["H"], num_classes=w["C"],
                                    num_heads=w["heads"], dropout=0.1).to(dev)
        feats, mask, labels = bench.make_inputs(w, w["B"], 42, dev)
        step = train_step.HybridTrainStep(model, feats, mask, labels)
        seed, offset = (int(v) for v in step.rng.tolist())
        params_cpu = {n: p.detach().cpu().clone() for n, p in model.named_parameters()}
        step.forward_backward()
        torch.cuda.synchronize()
        dev_acts = {m: step.saved_activation("proj", i).cpu() for i, m in enumerate(names)}
        dev_acts["cls"] = step.saved_activation("cls_hidden").cpu()

        def oracle(taps=None, relu_gate=None):
            params = {n: v.clone().requires_grad_(True) for n, v in params_cpu.items()}
            xs = {n: f.detach().cpu().clone().requires_grad_(True) for n, f in zip(names, feats)}
            logits, _ = hybrid_forward(params, names, xs, mask.cpu(), w["heads"], p=0.1, train=True,
                                       gen=mask_provider(seed, offset, 0.1), taps=taps, relu_gate=relu_gate)
            cross_entropy_ls(logits, labels.cpu()).backward()
            return logits.detach(), params, xs

        def compare(logits, params, xs):
            scale = max([float(p.grad.abs().max()) for p in params.values()] +
                        [float(x.grad.abs().max()) for x in xs.values()])
            res = {"logits": ratio(step.logits, logits, 1e-6 * float(logits.abs().max()))}
            for i, n in enumerate(names):
                res[f"dx/{n}"] = ratio(step.dx[i], xs[n].grad, 1e-5 * scale)
            grads = dict(step.named_grads())
            for n, p in params.items():
                res[n] = ratio(grads[n], p.grad, 1e-5 * scale)
            worst = max(res.items(), key=lambda kv: kv[1][0])
            over = {n: [round(r[0], 3), r[1]] for n, r in res.items() if r[0] > 1}
            return [worst[0], round(worst[1][0], 4)], over

        taps = {}
        plain = compare(*oracle(taps=taps))
        wts = {m: params_cpu[f"projections.{m}.0.weight"] for m in names}
        wts["cls"] = params_cpu["classifier.0.weight"]
        gates, band = device_relu_gates(taps, wts, dev_acts)
        gated = compare(*oracle(relu_gate=gates))
        print(json.dumps({"k": k, "seed": seed, "offset": offset, "plain": {"worst": plain[0], "over": plain[1]},
                          "device_relu_gates": {"worst": gated[0], "over": gated[1]}, "band": band}), flush=True)


if __name__ == "__main__":
    main()
