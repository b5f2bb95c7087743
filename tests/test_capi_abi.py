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
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %d %d %zu %zu %zu\\n", sizeof(mmf_hybrid_desc), sizeof(mmf_hybrid_params),
         sizeof(mmf_hybrid_grads), sizeof(mmf_cma_desc), sizeof(mmf_cma_params),
         offsetof(mmf_hybrid_desc, dropout), offsetof(mmf_hybrid_params, cls2),
         offsetof(mmf_hybrid_desc, matmul_precision), offsetof(mmf_cma_desc, matmul_precision),
         (int)MMF_PRECISION_MEDIUM, (int)MMF_PRECISION_HIGH, offsetof(mmf_hybrid_desc, plan_flags),
         offsetof(mmf_hybrid_desc, saved_capacity), offsetof(mmf_hybrid_desc, workspace_capacity));
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
          nat.PRECISION_HIGH, nat.HybridDesc.plan_flags.offset, nat.HybridDesc.saved_capacity.offset,
          nat.HybridDesc.workspace_capacity.offset]
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


PLAN_KNOBS = ("MMF_PSTORE", "MMF_NO_LONG_FUSED", "MMF_NO_FUSED_BWD", "MMF_NO_BF16_QK", "MMF_NO_GEMM_B16",
              "MMF_QK_CAT", "MMF_NO_DQK_B16", "MMF_NO_PROJ_B16", "MMF_NO_PCOL", "MMF_NO_POOLE", "MMF_POOLE_FLAT",
              "MMF_NO_L1_LEAN", "MMF_WGRAD_SPLIT_CAP", "MMF_NO_SIDE_STREAM", "MMF_SIDE_STREAM", "MMF_KW_SERIAL",
              "MMF_KW_FUSED", "MMF_NO_KW_FUSED", "MMF_NO_GATE_B16", "MMF_POOL_PER_PAIR", "MMF_TAIL_S")


def test_plan_flags_fingerprint_the_plan_switches(nat, monkeypatch):
    """mmf_hybrid_plan_flags: 0 with no plan switch set, a different value per switch and value,
    independent of the order the variables were set in; other MMF_* variables do not count."""
    L = nat.lib()
    for k in PLAN_KNOBS:
        monkeypatch.delenv(k, raising=False)
    assert L.mmf_hybrid_plan_flags() == 0
    monkeypatch.setenv("MMF_L1_POLL_BOUND", "100")      # (not a layout switch)
    assert L.mmf_hybrid_plan_flags() == 0
    monkeypatch.setenv("MMF_PSTORE", "1")
    a = L.mmf_hybrid_plan_flags()
    monkeypatch.setenv("MMF_PSTORE", "2")
    b = L.mmf_hybrid_plan_flags()
    assert a != 0 and b != 0 and a != b
    monkeypatch.setenv("MMF_NO_PCOL", "1")
    ab = L.mmf_hybrid_plan_flags()
    monkeypatch.delenv("MMF_PSTORE")
    monkeypatch.setenv("MMF_PSTORE", "2")              # (now after MMF_NO_PCOL in environ)
    assert L.mmf_hybrid_plan_flags() == ab != b
    monkeypatch.delenv("MMF_PSTORE")
    monkeypatch.delenv("MMF_NO_PCOL")
    assert L.mmf_hybrid_plan_flags() == 0


def test_buffer_contract_refused_before_launch(nat, monkeypatch):
    """The buffer contract (include/mmfusion.h): forward / backward / train step
    refuse a call whose plan switches differ from the descriptor's plan_flags, or whose layout
    needs more than the declared saved / workspace capacity -- MMF_EINVAL before any launch (host
    buffers here: nothing is dereferenced; no GPU needed)."""
    for k in PLAN_KNOBS:
        monkeypatch.delenv(k, raising=False)
    L = nat.lib()
    d = _desc(nat)
    d.plan_flags = L.mmf_hybrid_plan_flags()
    n_saved = L.mmf_hybrid_saved_bytes(ctypes.byref(d))
    n_ws = L.mmf_hybrid_workspace_bytes(ctypes.byref(d))
    params, grads = nat.HybridParams(), nat.HybridGrads()
    buf = (ctypes.c_float * 4096)()
    host = ctypes.addressof(buf)
    xs = nat.ptr_array([host] * 3)
    rng = (ctypes.c_uint64 * 2)()

    def fwd():
        return L.mmf_hybrid_forward(ctypes.byref(d), ctypes.byref(params), ctypes.cast(xs, ctypes.c_void_p), host,
                                    ctypes.addressof(rng), host, host, host, None, None)

    def bwd():
        return L.mmf_hybrid_backward(ctypes.byref(d), ctypes.byref(params), ctypes.cast(xs, ctypes.c_void_p), host,
                                     host, host, host, ctypes.byref(grads), None, None)

    def step(part=0):
        return L.mmf_hybrid_train_step_part(part, ctypes.byref(d), ctypes.byref(params),
                                            ctypes.cast(xs, ctypes.c_void_p), host, host, 0.05, 1.0,
                                            ctypes.addressof(rng), host, host, None, host, host, host, host,
                                            ctypes.byref(grads), None, None, None, None, 0, None)

    for call in (fwd, bwd, step, lambda: step(2)):
        d.saved_capacity, d.workspace_capacity = 0, n_ws          # (no capacity declared)
        assert call() == 1 and b"saved buffer too small" in L.mmf_last_error()
        d.saved_capacity, d.workspace_capacity = n_saved, 64
        if call is not fwd:                                      # (the forward takes no workspace)
            assert call() == 1 and b"workspace too small" in L.mmf_last_error()
        d.saved_capacity, d.workspace_capacity = n_saved, n_ws
        monkeypatch.setenv("MMF_NO_L1_LEAN", "1")                # a plan switch set after sizing
        assert call() == 1 and b"plan switches" in L.mmf_last_error()
        monkeypatch.delenv("MMF_NO_L1_LEAN")


def test_saved_region_query(nat):
    """mmf_hybrid_saved_region: the P_m / classifier-hidden regions lie inside `saved`, 256-B
    aligned, sized (B, L_m, H) / (B, H) fp32, disjoint; unknown regions and indices refused."""
    L = nat.lib()
    d = _desc(nat)
    for m in range(3):
        d.seq_len[m] = 8 * (m + 1)
    total = L.mmf_hybrid_saved_bytes(ctypes.byref(d))
    off, nb = ctypes.c_uint64(), ctypes.c_uint64()
    spans = []
    for m in range(3):
        assert L.mmf_hybrid_saved_region(ctypes.byref(d), 0, m, ctypes.byref(off), ctypes.byref(nb)) == 0
        assert nb.value == 4 * d.batch * d.seq_len[m] * d.hidden
        spans.append((off.value, off.value + nb.value))
    assert L.mmf_hybrid_saved_region(ctypes.byref(d), 1, 0, ctypes.byref(off), ctypes.byref(nb)) == 0
    assert nb.value == 4 * d.batch * d.hidden
    spans.append((off.value, off.value + nb.value))
    for a, b in spans:
        assert a % 256 == 0 and b <= total
    spans.sort()
    assert all(spans[i][1] <= spans[i + 1][0] for i in range(len(spans) - 1))
    assert L.mmf_hybrid_saved_region(ctypes.byref(d), 0, 3, ctypes.byref(off), ctypes.byref(nb)) != 0
    assert b"modality" in L.mmf_last_error()
    assert L.mmf_hybrid_saved_region(ctypes.byref(d), 1, 1, ctypes.byref(off), ctypes.byref(nb)) != 0
    assert L.mmf_hybrid_saved_region(ctypes.byref(d), 2, 0, ctypes.byref(off), ctypes.byref(nb)) != 0
    assert b"unknown region" in L.mmf_last_error()
