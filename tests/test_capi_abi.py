"""C-ABI checks without a GPU: the library loads, exports every function
include/mmfusion.h declares, the ctypes mirrors match the C struct layouts,
and host-side validation (size queries, error codes) behaves."""
import ctypes
import re
import subprocess
import tempfile
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "mmfusion.h"


@pytest.fixture(scope="module")
def nat(pkg_on_path):
    import mmf_native
    try:
        mmf_native.lib()
    except RuntimeError as e:
        pytest.fail(f"libmmfusion.so not built: {e}")
    return mmf_native


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mmf_[a-z0-9_]+)\s*\(", text)))


def test_exports_every_declared_symbol(nat):
    L = nat.lib()
    names = declared_functions()
    assert len(names) >= 12
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert set(names) == set(nat.EXPORTED_SYMBOLS)


def test_struct_layouts_match_header(nat, tmp_path):
    src = tmp_path / "sizes.c"
    src.write_text(f"""
#include <stdio.h>
#include <stddef.h>
#include "{HEADER}"
int main(void) {{
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %d %d\\n", sizeof(mmf_hybrid_desc), sizeof(mmf_hybrid_params),
         sizeof(mmf_hybrid_grads), sizeof(mmf_cma_desc), sizeof(mmf_cma_params),
         offsetof(mmf_hybrid_desc, dropout), offsetof(mmf_hybrid_params, cls2),
         offsetof(mmf_hybrid_desc, matmul_precision), offsetof(mmf_cma_desc, matmul_precision),
         (int)MMF_PRECISION_MEDIUM, (int)MMF_PRECISION_HIGH);
  return 0;
}}
""")
    exe = tmp_path / "sizes"
    subprocess.run(["gcc", str(src), "-o", str(exe)], check=True)
    out = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    py = [ctypes.sizeof(nat.HybridDesc), ctypes.sizeof(nat.HybridParams),
          ctypes.sizeof(nat.HybridGrads), ctypes.sizeof(nat.CmaDesc), ctypes.sizeof(nat.CmaParams),
          nat.HybridDesc.dropout.offset, nat.HybridParams.cls2.offset,
          nat.HybridDesc.matmul_precision.offset, nat.CmaDesc.matmul_precision.offset, nat.PRECISION_MEDIUM,
          nat.PRECISION_HIGH]
    assert out == py


def _desc(nat, **kw):
    d = nat.HybridDesc()
    d.batch, d.num_modalities, d.hidden, d.num_heads, d.num_classes = 4, 3, 32, 4, 5
    for m in range(3):
        d.seq_len[m] = 0
        d.in_dim[m] = 16
    pairs = [(q, k) for q in range(3) for k in range(3) if q != k]
    d.num_pairs = len(pairs)
    for g, (q, k) in enumerate(pairs):
        d.pair_q[g], d.pair_k[g] = q, k
    d.dropout, d.training, d.return_attention = 0.1, 1, 0
    for k, v in kw.items():
        setattr(d, k, v)
    return d


def test_size_queries_and_validation(nat):
    L = nat.lib()
    d = _desc(nat)
    assert L.mmf_hybrid_saved_bytes(ctypes.byref(d)) > 0
    assert L.mmf_hybrid_workspace_bytes(ctypes.byref(d)) > 0
    bad = _desc(nat, num_heads=3)            # 32 % 3 != 0
    assert L.mmf_hybrid_saved_bytes(ctypes.byref(bad)) == 0
    assert b"divisible" in L.mmf_last_error()
    wide = _desc(nat, hidden=256, num_heads=2)  # head_dim 128 > 64: single-key / materialised-score plans
    assert L.mmf_hybrid_saved_bytes(ctypes.byref(wide)) > 0
    big = _desc(nat, hidden=256, num_heads=1)   # head_dim 256 at L = 50000: the score tensor's int32 strides
    for m in range(3):
        big.seq_len[m] = 50000
    assert L.mmf_hybrid_saved_bytes(ctypes.byref(big)) == 0
    assert b"head_dim" in L.mmf_last_error() and b"too large" in L.mmf_last_error()
    # forward refuses a bad descriptor before touching the device
    rc = L.mmf_hybrid_forward(ctypes.byref(bad), None, None, None, None, None, None, None, None, None)
    assert rc != 0
    odd = _desc(nat, matmul_precision=7)     # none of HIGHEST, MEDIUM, HIGH
    assert L.mmf_hybrid_saved_bytes(ctypes.byref(odd)) == 0
    assert b"matmul_precision" in L.mmf_last_error()
    assert L.mmf_hybrid_saved_bytes(ctypes.byref(_desc(nat, matmul_precision=nat.PRECISION_MEDIUM))) > 0
    assert L.mmf_hybrid_saved_bytes(ctypes.byref(_desc(nat, matmul_precision=nat.PRECISION_HIGH))) > 0
    c = nat.CmaDesc(2, 5, 7, 8, 8, 16, 4, 2, 0.0, 0)
    assert L.mmf_cma_saved_bytes(ctypes.byref(c)) > 0
    c.matmul_precision = 3
    assert L.mmf_cma_saved_bytes(ctypes.byref(c)) == 0
    c.matmul_precision = nat.PRECISION_MEDIUM
    assert L.mmf_cma_saved_bytes(ctypes.byref(c)) > 0
    c.matmul_precision = nat.PRECISION_HIGH
    assert L.mmf_cma_saved_bytes(ctypes.byref(c)) > 0
    c.mask_mode = 5
    assert L.mmf_cma_saved_bytes(ctypes.byref(c)) == 0
    assert L.mmf_version().startswith(b"mmfusion")


def test_workspace_scales_with_sequence(nat):
    L = nat.lib()
    d1 = _desc(nat)
    d2 = _desc(nat)
    for m in range(3):
        d2.seq_len[m] = 128
    assert L.mmf_hybrid_saved_bytes(ctypes.byref(d2)) > 10 * L.mmf_hybrid_saved_bytes(ctypes.byref(d1))
    assert L.mmf_hybrid_workspace_bytes(ctypes.byref(d2)) > 5 * L.mmf_hybrid_workspace_bytes(ctypes.byref(d1))


def test_matmul_precision_follows_torch(nat):
    """The modules read torch.get_float32_matmul_precision() (src/train.py:53-68
    applies config/base.yaml:80 training.matmul_precision through it)."""
    import torch
    prev = torch.get_float32_matmul_precision()
    try:
        for mode, want in (("highest", nat.PRECISION_HIGHEST), ("high", nat.PRECISION_HIGH),
                           ("medium", nat.PRECISION_MEDIUM)):
            torch.set_float32_matmul_precision(mode)
            assert nat.matmul_precision() == want, mode
    finally:
        torch.set_float32_matmul_precision(prev)


def test_lean_l1_query(nat):
    """mmf_hybrid_lean_l1: the launch-lean L = 1 plan serves 2-D inputs at fp32 "highest" with every
    ordered pair present (bench.py then launches its step eagerly, HybridTrainStep.replay_pays)."""
    L = nat.lib()
    d = _desc(nat)
    assert L.mmf_hybrid_lean_l1(ctypes.byref(d)) == 1
    for m in range(3):
        d.seq_len[m] = 128
    assert L.mmf_hybrid_lean_l1(ctypes.byref(d)) == 0
    assert L.mmf_hybrid_lean_l1(ctypes.byref(_desc(nat, matmul_precision=nat.PRECISION_MEDIUM))) == 0
    assert L.mmf_hybrid_lean_l1(ctypes.byref(_desc(nat, num_heads=3))) == 0   # invalid descriptor
