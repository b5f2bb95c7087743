"""PAMAP2 logits / ECE parity on the GPU (BASELINE.json north_star: "logits/ECE on
PAMAP2 must reproduce the reference within tolerance").

Inputs are the reference's own encoder outputs for the 44 present test chunks
(tests/golden/gen_pamap2.py: reference LSTM encoders + LayerNorm on the shipped
PAMAP2 shards, chunk 1024).  The HybridFusion weights are the seeded
``hybrid_state`` plus the fusion head the reference fitted on the present
train chunks.  The drop-in module runs the HIP path on cuda:0 in eval mode; the
caller-side chain (calibration.py, restating src/eval.py:80-103 and
src/uncertainty.py:84-192) scores its logits.

Tolerances: logits max|d| <= 1e-3 * max|ref| (fp32 parity); ECE / MCE within
1/N (one sample crossing a bin edge moves them by at most 1/N);
NLL 1e-3 relative; predictions identical.
"""
import numpy as np
import pytest
import torch

from _util import close, load_fixture
from cases import (PAMAP2_CLASSES, PAMAP2_HEADS, PAMAP2_HIDDEN, PAMAP2_MODALITIES, PAMAP2_OUT_DIM,
                   PAMAP2_SEED, hybrid_state)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup(pkg_on_path):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    import calibration
    import fusion
    fx = load_fixture("pamap2_test")
    names = PAMAP2_MODALITIES
    dims = {m: PAMAP2_OUT_DIM for m in names}
    model = fusion.HybridFusion(dims, hidden_dim=PAMAP2_HIDDEN, num_classes=PAMAP2_CLASSES,
                                num_heads=PAMAP2_HEADS, dropout=0.1)
    sd = hybrid_state(names, dims, PAMAP2_HIDDEN, PAMAP2_CLASSES, PAMAP2_SEED)
    for k in list(sd):
        if f"head/{k}" in fx:
            sd[k] = fx[f"head/{k}"]
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    return model.cuda().eval(), calibration, fx


def test_pamap2_logits_and_calibration(setup):
    model, cal, fx = setup
    enc = fx["enc"]
    feats = {m: torch.from_numpy(enc[:, j]).cuda() for j, m in enumerate(PAMAP2_MODALITIES)}
    with torch.no_grad():
        logits = model(feats, torch.ones(enc.shape[0], len(PAMAP2_MODALITIES)).cuda())
    torch.cuda.synchronize()
    assert close(logits.cpu(), fx["logits"], 1e-3, 1e-5)
    out = cal.evaluate_logits(logits, torch.from_numpy(fx["labels"]))
    n = out["num_samples"]
    assert np.array_equal(out["predictions"].numpy(), fx["preds"])
    assert abs(out["ece"] - float(fx["ece"][0])) <= 1.0 / n
    assert abs(out["mce"] - float(fx["mce"][0])) <= 1.0 / n
    assert abs(out["nll"] - float(fx["nll"][0])) <= 1e-3 * abs(float(fx["nll"][0]))
    assert out["accuracy"] == pytest.approx(float(fx["accuracy"][0]), abs=1e-7)


def test_pamap2_missing_modality_sweep(setup):
    """src/eval.py:342-424: every modality subset (zeroed raw inputs -> enc_zero, subset mask)."""
    model, _, fx = setup
    enc, zero = fx["enc"], fx["enc_zero"]
    labels = torch.from_numpy(fx["labels"])
    for s, sub in enumerate(fx["subset_mask"]):
        feats = {m: torch.from_numpy(enc[:, j] if sub[j] else zero[:, j]).cuda()
                 for j, m in enumerate(PAMAP2_MODALITIES)}
        mask = torch.from_numpy(np.tile(sub, (enc.shape[0], 1))).cuda()
        with torch.no_grad():
            lg = model(feats, mask).cpu()
        assert close(lg, fx["subset_logits"][s], 1e-3, 1e-5), s
        acc = float((lg.argmax(dim=1) == labels).float().mean())
        assert acc == pytest.approx(float(fx["subset_accuracy"][s]), abs=1e-7), s
