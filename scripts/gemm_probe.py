#!/usr/bin/env python3
"""What the platform GEMM (torch.matmul -> hipBLASLt on ROCm) reaches on C5's GEMM shapes, as the
yardstick for the library's own LDS-DMA kernels.  bf16 operands, fp32 accumulate.
usage: python scripts/gemm_probe.py [--out file.json]"""

import argparse
import json

import torch


def bench(fn, iters=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = "cuda"
    R, H = 128 * 512, 256
    res = {}
    # (name, M, N, K, layout): Y = X W^T (+ bias) forward projections, dX = dY W, dW = dY^T X
    shapes = [("qk_one_pair", R, H, H), ("qk_per_query_modality_5pairs", R, 5 * H, H),
              ("qk_per_modality_q_and_k_10", R, 10 * H, H), ("dP_sum_10_sources", R, H, 10 * H),
              ("wgrad_one", H, H, R), ("wgrad_10_stacked", 10 * H, H, R)]
    for name, M, N, K in shapes:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        bias = torch.randn(N, device=dev, dtype=torch.bfloat16)
        if name.startswith("wgrad"):
            xt = torch.randn(K, M, device=dev, dtype=torch.bfloat16)   # dY (R x M) read transposed
            wt = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
            ms = bench(lambda: xt.t() @ wt)
        else:
            ms = bench(lambda: torch.nn.functional.linear(x, w, bias))
        fl = 2.0 * M * N * K
        byt = 2.0 * (M * K + N * K + M * N)
        res[name] = {"M": M, "N": N, "K": K, "ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1),
                     "frac_bf16_dense_2500": round(fl / ms / 1e9 / 2500, 3), "GBps": round(byt / ms / 1e6, 1)}
        print(name, json.dumps(res[name]), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
