"""Library fp32 GEMM ceiling on the box: hipBLASLt / rocBLAS (torch.mm at matmul precision
"highest") on the C2 step's GEMM shapes, beside our kernels' rates from the bench line.

usage (GPU box): python scripts/lib_gemm_ceiling.py > gpurun_out/<run>/lib_gemm.json
"""
import json
import time

import torch

torch.backends.cuda.matmul.allow_tf32 = False
torch.set_float32_matmul_precision("highest")
dev = torch.device("cuda:0")
B, L, H = 256, 128, 128
R = B * L   # rows per modality

# (name, A shape, B shape, batch) -- C = A @ B
SHAPES = [
    ("proj: 3 x (32768x128)@(128x128)", (3, R, 128), (3, 128, H)),
    ("qk: 12 x (32768x128)@(128x128)", (12, R, H), (12, H, H)),
    ("dZ: 3 x (32768x512)@(512x128)", (3, R, 4 * H), (3, 4 * H, H)),
    ("dX: 3 x (32768x128)@(128x128)", (3, R, H), (3, H, 128)),
    ("dW: 15 x (128x32768)@(32768x128)", (15, H, R), (15, R, H)),
    ("square 8192^3", (1, 8192, 8192), (1, 8192, 8192)),
]


def bench(a, b, iters=20):
    for _ in range(3):
        torch.bmm(a, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        torch.bmm(a, b)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


out = []
for name, sa, sb in SHAPES:
    a = torch.randn(*sa, device=dev)
    b = torch.randn(*sb, device=dev)
    ms = bench(a, b)
    fl = 2.0 * sa[0] * sa[1] * sa[2] * sb[2]
    out.append({"gemm": name, "ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1),
                "frac_of_157.3": round(fl / ms / 1e9 / 157.3, 3)})
    print(json.dumps(out[-1]), flush=True)
    del a, b
