"""ctypes binding of libmmfusion.so (the C-ABI declared in include/mmfusion.h).

This is the only way the host mirror reaches the compute path.  There is no
CPU or PyTorch fallback: if the library is missing or a tensor is not on a
ROCm device, every entry point raises.
"""

from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int32, c_int64, c_size_t, c_void_p, POINTER
from typing import Optional

import torch

MAX_MODALITIES = 8
MAX_PAIRS = MAX_MODALITIES * (MAX_MODALITIES - 1)
MAX_HEAD_DIM = 64
PRECISION_HIGHEST = 0   # MMF_PRECISION_HIGHEST: fp32 MFMA
PRECISION_MEDIUM = 1    # MMF_PRECISION_MEDIUM: bf16 MFMA operands, fp32 accumulate
PRECISION_HIGH = 2      # MMF_PRECISION_HIGH: bf16x3 (operands split into bf16 hi + lo), fp32 accumulate


def matmul_precision() -> int:
    """The caller's torch.get_float32_matmul_precision() as the C-ABI enum.

    The reference sets it from ``training.matmul_precision`` (config/base.yaml:80,
    "medium") through ``_configure_matmul_precision`` (src/train.py:53-68,448);
    the reference's own tests set "high" (tests/test_train.py:45).  "medium" lets
    fp32 matmuls use bf16 operands with fp32 accumulation.  "high" lets them use
    TF32 or treat "each float32 number as the sum of two bfloat16 numbers"
    (torch.set_float32_matmul_precision); gfx950 has no TF32, so "high" runs the
    bf16x3 form: every MFMA operand split into bf16 hi + lo, three bf16 MFMAs
    (lo*hi + hi*lo + hi*hi) into the fp32 accumulator (csrc/mmf_device.h mfma_k16).
    """
    mode = torch.get_float32_matmul_precision()
    return {"medium": PRECISION_MEDIUM, "high": PRECISION_HIGH}.get(mode, PRECISION_HIGHEST)

_HERE = os.path.dirname(os.path.abspath(__file__))
# MMF_LIB_PATH selects another in-tree build (e.g. csrc/libmmfusion_stamps.so, the
# diagnostic phase-stamp build of scripts/attn_stamps.py)
LIB_PATH = os.environ.get("MMF_LIB_PATH") or os.path.join(_HERE, "csrc", "libmmfusion.so")

EXPORTED_SYMBOLS = (
    "mmf_hybrid_saved_bytes", "mmf_hybrid_workspace_bytes", "mmf_hybrid_forward",
    "mmf_hybrid_backward", "mmf_hybrid_train_sync_bytes", "mmf_hybrid_train_status", "mmf_hybrid_train_step",
    "mmf_hybrid_train_step_part", "mmf_hybrid_plan_flags", "mmf_hybrid_saved_region",
    "mmf_adaptive_weights_workspace_bytes", "mmf_adaptive_weights",
    "mmf_adaptive_weights_backward",
    "mmf_cma_saved_bytes", "mmf_cma_workspace_bytes", "mmf_cma_forward", "mmf_cma_backward",
    "mmf_cross_entropy_ls", "mmf_adamw_step", "mmf_adamw_step_dev", "mmf_grad_clip_workspace_bytes",
    "mmf_grad_clip_coef", "mmf_clip_adamw_step_dev", "mmf_clip_adamw_apply_dev", "mmf_grad_accumulate", "mmf_gemm_bf16_workspace_bytes", "mmf_gemm_bf16", "mmf_hybrid_lean_l1", "mmf_profile_begin", "mmf_profile_end",
    "mmf_last_error", "mmf_version",
    "mmf_attention_pool_workspace_bytes", "mmf_attention_pool_forward", "mmf_attention_pool_backward",
    "mmf_late_fusion_workspace_bytes", "mmf_late_fusion_forward", "mmf_late_fusion_backward",
    "mmf_gather_chunks",
    "mmf_lstm_sync_bytes", "mmf_lstm_forward", "mmf_lstm_backward",
)


class Linear(ctypes.Structure):
    _fields_ = [("w", c_void_p), ("b", c_void_p)]


class HybridDesc(ctypes.Structure):
    _fields_ = [
        ("batch", c_int32), ("num_modalities", c_int32), ("hidden", c_int32),
        ("num_heads", c_int32), ("num_classes", c_int32),
        ("seq_len", c_int32 * MAX_MODALITIES), ("in_dim", c_int32 * MAX_MODALITIES),
        ("num_pairs", c_int32),
        ("pair_q", c_int32 * MAX_PAIRS), ("pair_k", c_int32 * MAX_PAIRS),
        ("dropout", c_float), ("training", c_int32), ("return_attention", c_int32),
        ("matmul_precision", c_int32),
        # the buffer contract (include/mmfusion.h): the plan-switch fingerprint the buffers were
        # sized under, and their capacities in bytes
        ("plan_flags", ctypes.c_uint32), ("saved_capacity", ctypes.c_uint64),
        ("workspace_capacity", ctypes.c_uint64),
    ]


class HybridParams(ctypes.Structure):
    _fields_ = [
        ("proj", Linear * MAX_MODALITIES),
        ("q", Linear * MAX_PAIRS), ("k", Linear * MAX_PAIRS),
        ("v", Linear * MAX_PAIRS), ("o", Linear * MAX_PAIRS),
        ("gate", Linear * MAX_MODALITIES),
        ("cls1", Linear), ("cls2", Linear),
    ]


HybridGrads = HybridParams  # identical layout (mmf_linear_grad has the same two pointers)


class CmaDesc(ctypes.Structure):
    _fields_ = [
        ("batch", c_int32), ("lq", c_int32), ("lk", c_int32), ("query_dim", c_int32),
        ("key_dim", c_int32), ("hidden", c_int32), ("num_heads", c_int32),
        ("mask_mode", c_int32), ("dropout", c_float), ("training", c_int32),
        ("matmul_precision", c_int32),
    ]


class CmaParams(ctypes.Structure):
    _fields_ = [("q", Linear), ("k", Linear), ("v", Linear), ("o", Linear)]


CmaGrads = CmaParams

_LIB: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    """Load libmmfusion.so (built in-tree by `make -C csrc` / __graft_entry__.build())."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"mmfusion: HIP library not found at {LIB_PATH}. Build it with "
            f"`make -C {os.path.join(_HERE, 'csrc')}` (hipcc --offload-arch=gfx950). "
            "There is no CPU fallback.")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz = c_void_p, c_size_t
    L.mmf_hybrid_saved_bytes.argtypes = [POINTER(HybridDesc)]
    L.mmf_hybrid_saved_bytes.restype = sz
    L.mmf_hybrid_workspace_bytes.argtypes = [POINTER(HybridDesc)]
    L.mmf_hybrid_workspace_bytes.restype = sz
    L.mmf_hybrid_plan_flags.argtypes = []
    L.mmf_hybrid_plan_flags.restype = ctypes.c_uint32
    L.mmf_hybrid_saved_region.argtypes = [POINTER(HybridDesc), c_int32, c_int32, POINTER(ctypes.c_uint64),
                                          POINTER(ctypes.c_uint64)]
    L.mmf_hybrid_saved_region.restype = c_int32
    L.mmf_hybrid_forward.argtypes = [POINTER(HybridDesc), POINTER(HybridParams), vp, vp, vp, vp,
                                     vp, vp, vp, vp]
    L.mmf_hybrid_forward.restype = c_int32
    L.mmf_hybrid_backward.argtypes = [POINTER(HybridDesc), POINTER(HybridParams), vp, vp, vp, vp,
                                      vp, POINTER(HybridGrads), vp, vp]
    L.mmf_hybrid_backward.restype = c_int32
    L.mmf_hybrid_train_sync_bytes.argtypes = [POINTER(HybridDesc)]
    L.mmf_hybrid_train_sync_bytes.restype = sz
    L.mmf_hybrid_lean_l1.argtypes = [POINTER(HybridDesc)]
    L.mmf_hybrid_lean_l1.restype = c_int32
    L.mmf_hybrid_train_status.argtypes = [POINTER(HybridDesc), vp, c_int32, vp]
    L.mmf_hybrid_train_status.restype = c_int32
    L.mmf_hybrid_train_step.argtypes = [POINTER(HybridDesc), POINTER(HybridParams), vp, vp, vp, c_float, c_float,
                                        vp, vp, vp, vp, vp, vp, vp, vp, POINTER(HybridGrads), vp, vp, vp, vp,
                                        c_int64, vp]
    L.mmf_hybrid_train_step.restype = c_int32
    L.mmf_hybrid_train_step_part.argtypes = [c_int32] + L.mmf_hybrid_train_step.argtypes
    L.mmf_hybrid_train_step_part.restype = c_int32
    L.mmf_adaptive_weights_workspace_bytes.argtypes = [c_int32, c_int32, c_int32]
    L.mmf_adaptive_weights_workspace_bytes.restype = sz
    L.mmf_adaptive_weights.argtypes = [c_int32, c_int32, c_int32, vp, vp, vp, vp, vp, vp]
    L.mmf_adaptive_weights.restype = c_int32
    L.mmf_adaptive_weights_backward.argtypes = [c_int32, c_int32, c_int32, vp, vp, vp, vp, vp, vp, vp, vp]
    L.mmf_adaptive_weights_backward.restype = c_int32
    L.mmf_cma_saved_bytes.argtypes = [POINTER(CmaDesc)]
    L.mmf_cma_saved_bytes.restype = sz
    L.mmf_cma_workspace_bytes.argtypes = [POINTER(CmaDesc)]
    L.mmf_cma_workspace_bytes.restype = sz
    L.mmf_cma_forward.argtypes = [POINTER(CmaDesc), POINTER(CmaParams), vp, vp, vp, vp, vp, vp,
                                  vp, vp, vp]
    L.mmf_cma_forward.restype = c_int32
    L.mmf_cma_backward.argtypes = [POINTER(CmaDesc), POINTER(CmaParams), vp, vp, vp, vp, vp, vp,
                                   vp, POINTER(CmaGrads), vp, vp, vp, vp]
    L.mmf_cma_backward.restype = c_int32
    L.mmf_cross_entropy_ls.argtypes = [c_int32, c_int32, vp, vp, c_float, c_float, vp, vp, vp]
    L.mmf_cross_entropy_ls.restype = c_int32
    L.mmf_adamw_step.argtypes = [c_int64, vp, vp, vp, vp, vp, c_float, c_float, c_float, c_float,
                                 c_float, c_float, vp]
    L.mmf_adamw_step.restype = c_int32
    L.mmf_adamw_step_dev.argtypes = [c_int64, vp, vp, vp, vp, vp, vp, vp, c_float, c_float, c_float, c_float,
                                     c_float, vp]
    L.mmf_adamw_step_dev.restype = c_int32
    L.mmf_grad_clip_workspace_bytes.argtypes = []
    L.mmf_grad_clip_workspace_bytes.restype = c_size_t
    L.mmf_grad_clip_coef.argtypes = [c_int64, vp, c_float, c_float, vp, vp, vp, vp]
    L.mmf_grad_clip_coef.restype = c_int32
    L.mmf_clip_adamw_step_dev.argtypes = [c_int64, vp, vp, vp, vp, vp, vp, c_float, vp, vp, vp, c_float, c_float,
                                          c_float, c_float, c_float, vp]
    L.mmf_clip_adamw_step_dev.restype = c_int32
    L.mmf_clip_adamw_apply_dev.argtypes = [c_int64, vp, vp, vp, vp, vp, vp, c_float, vp, vp, vp, c_float, c_float,
                                           c_float, c_float, c_float, vp]
    L.mmf_clip_adamw_apply_dev.restype = c_int32
    L.mmf_grad_accumulate.argtypes = [c_int64, vp, vp, vp]
    L.mmf_grad_accumulate.restype = c_int32
    L.mmf_gemm_bf16_workspace_bytes.argtypes = [c_int32, c_int32, c_int32, c_int32]
    L.mmf_gemm_bf16_workspace_bytes.restype = sz
    L.mmf_gemm_bf16.argtypes = [c_int32, c_int32, c_int32, vp, c_int32, c_int32, vp, c_int32, c_int32, vp, vp,
                                c_int32, c_int32, vp, c_int32, vp, vp]
    L.mmf_gemm_bf16.restype = c_int32
    L.mmf_profile_begin.argtypes = []
    L.mmf_profile_begin.restype = None
    L.mmf_profile_end.argtypes = [ctypes.c_char_p, c_size_t]
    L.mmf_profile_end.restype = c_size_t
    L.mmf_attention_pool_workspace_bytes.argtypes = [c_int32, c_int32]
    L.mmf_attention_pool_workspace_bytes.restype = sz
    L.mmf_attention_pool_forward.argtypes = [c_int32, c_int32, c_int32, vp, vp, vp, vp, vp, vp, vp]
    L.mmf_attention_pool_forward.restype = c_int32
    L.mmf_attention_pool_backward.argtypes = [c_int32, c_int32, c_int32, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.mmf_attention_pool_backward.restype = c_int32
    L.mmf_late_fusion_workspace_bytes.argtypes = [c_int32, c_int32]
    L.mmf_late_fusion_workspace_bytes.restype = sz
    L.mmf_late_fusion_forward.argtypes = [c_int32, c_int32, c_int32, vp, vp, vp, vp, vp, vp]
    L.mmf_late_fusion_forward.restype = c_int32
    L.mmf_late_fusion_backward.argtypes = [c_int32, c_int32, c_int32, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.mmf_late_fusion_backward.restype = c_int32
    L.mmf_gather_chunks.argtypes = [vp, c_int64, c_int32, vp, vp, c_int32, c_int32, c_int32, vp, vp, vp, c_int32,
                                     vp, vp, vp]
    L.mmf_gather_chunks.restype = c_int32
    L.mmf_lstm_sync_bytes.argtypes = [c_int32, c_int32]
    L.mmf_lstm_sync_bytes.restype = c_size_t
    L.mmf_lstm_forward.argtypes = [c_int32, c_int32, c_int32, c_int32, vp, vp, vp, vp, vp, vp, vp, vp]
    L.mmf_lstm_forward.restype = c_int32
    L.mmf_lstm_backward.argtypes = [c_int32, c_int32, c_int32, c_int32, vp, vp, vp, vp, vp, vp, vp, vp]
    L.mmf_lstm_backward.restype = c_int32
    L.mmf_last_error.argtypes = []
    L.mmf_last_error.restype = ctypes.c_char_p
    L.mmf_version.argtypes = []
    L.mmf_version.restype = ctypes.c_char_p
    _LIB = L
    return L


def profile_begin() -> None:
    lib().mmf_profile_begin()


def profile_end() -> tuple:
    """(stages, launches) recorded since profile_begin(), in launch order.

    stages:   [(stage_name, ms), ...], one per launch group;
    launches: [(stage_name, kernel_name, ms, flops, bytes), ...], one per kernel
              launch, with the launch's algorithmic FLOPs and HBM bytes.
    """
    L = lib()
    buf = ctypes.create_string_buffer(1 << 22)
    L.mmf_profile_end(buf, len(buf))
    stages, launches = [], []
    for line in buf.value.decode().splitlines():
        f = line.split("\t")
        if f[0] == "S":
            stages.append((f[1], float(f[2])))
        elif f[0] == "L":
            launches.append((f[1], f[2], float(f[3]), float(f[4]), float(f[5])))
    return stages, launches


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().mmf_last_error().decode(errors="replace")
        raise RuntimeError(f"mmfusion {what} failed (code {rc}): {msg}")


def require_device(t: torch.Tensor, what: str) -> None:
    if t.device.type != "cuda":
        raise RuntimeError(
            f"mmfusion: {what} is on {t.device}; the cross-modal fusion hot path runs only as HIP "
            "kernels on a ROCm device (MI355X). Move the module and inputs to 'cuda'.")


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device: torch.device) -> int:
    """The current HIP stream of `device` (torch's raw-handle accessor: no Stream object per call)."""
    if _RAW_STREAM is not None and device.index is not None:
        return _RAW_STREAM(device.index)
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def ptr_array(ptrs) -> ctypes.Array:
    arr = (c_void_p * max(1, len(ptrs)))()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return arr


def f32c(t: torch.Tensor) -> torch.Tensor:
    """fp32 + contiguous view/copy of an input activation."""
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()
