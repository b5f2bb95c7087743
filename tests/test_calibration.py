"""CPU checks of the caller-side evaluation chain (calibration.py) and of the
oracle on real PAMAP2 features, against the reference-generated fixture
tests/golden/pamap2_test.npz (tests/golden/gen_pamap2.py)."""
import numpy as np
import pytest
import torch

from _util import load_fixture, rel_err
from cases import (PAMAP2_CLASSES, PAMAP2_HEADS, PAMAP2_HIDDEN, PAMAP2_MODALITIES, PAMAP2_OUT_DIM,
                   PAMAP2_SEED, hybrid_state)


@pytest.fixture(scope="module")
def cal(pkg_on_path):
    import calibration
    return calibration


@pytest.fixture(scope="module")
def fx():
    return load_fixture("pamap2_test")


def test_metrics_reproduce_reference_on_reference_logits(cal, fx):
    """CalibrationMetrics (src/uncertainty.py:84-192) on the reference's own logits."""
    out = cal.evaluate_logits(torch.from_numpy(fx["logits"]), torch.from_numpy(fx["labels"]))
    assert np.array_equal(out["predictions"].numpy(), fx["preds"])
    assert np.allclose(out["confidences"].numpy(), fx["confidences"], rtol=0, atol=1e-7)
    assert abs(out["ece"] - float(fx["ece"][0])) <= 1e-6
    assert abs(out["mce"] - float(fx["mce"][0])) <= 1e-6
    assert abs(out["nll"] - float(fx["nll"][0])) <= 1e-6
    assert out["accuracy"] == pytest.approx(float(fx["accuracy"][0]), abs=1e-7)
    assert out["num_samples"] == 44


def test_bin_edges_known_answers(cal):
    """Edges belong to the upper bin; 1.0 belongs to the last (closed) bin; empty bins skipped."""
    conf = torch.tensor([0.0, 0.5, 1.0, 1.0])
    preds = torch.tensor([0, 1, 2, 3])
    labels = torch.tensor([0, 0, 2, 0])
    # bins (2): [0, .5) holds {0.0: correct}; [.5, 1] holds {.5: wrong, 1: right, 1: wrong}
    ece = cal.expected_calibration_error(conf, preds, labels, num_bins=2)
    exp = 0.25 * abs(1.0 - 0.0) + 0.75 * abs(1 / 3 - (0.5 + 1 + 1) / 3)
    assert ece == pytest.approx(exp, abs=1e-6)
    mce = cal.maximum_calibration_error(conf, preds, labels, num_bins=2)
    assert mce == pytest.approx(1.0, abs=1e-6)
    assert cal.expected_calibration_error(torch.tensor([]), torch.tensor([]), torch.tensor([])) == 0.0


def test_perfectly_calibrated_is_zero(cal):
    conf = torch.full((10,), 0.7)
    preds = torch.arange(10)
    labels = torch.where(torch.arange(10) < 7, preds, preds + 1)
    assert cal.expected_calibration_error(conf, preds, labels) == pytest.approx(0.0, abs=1e-6)


def _pamap2_params(fx):
    names = PAMAP2_MODALITIES
    sd = hybrid_state(names, {m: PAMAP2_OUT_DIM for m in names}, PAMAP2_HIDDEN, PAMAP2_CLASSES, PAMAP2_SEED)
    for k in list(sd):
        if f"head/{k}" in fx:
            sd[k] = fx[f"head/{k}"]
    return {k: torch.from_numpy(v) for k, v in sd.items()}


def test_oracle_reproduces_reference_pamap2_logits(fx):
    """The oracle on the reference's PAMAP2 encoder outputs: full set and every modality subset."""
    from oracle.hybrid_cpu import hybrid_forward
    params = _pamap2_params(fx)
    names = PAMAP2_MODALITIES
    enc, zero = fx["enc"], fx["enc_zero"]
    feats = {m: torch.from_numpy(enc[:, j]) for j, m in enumerate(names)}
    logits, _ = hybrid_forward(params, names, feats, torch.ones(enc.shape[0], len(names)), PAMAP2_HEADS)
    assert rel_err(logits, fx["logits"]) <= 1e-5
    for s, sub in enumerate(fx["subset_mask"]):
        f = {m: torch.from_numpy(enc[:, j] if sub[j] else zero[:, j]) for j, m in enumerate(names)}
        mk = torch.from_numpy(np.tile(sub, (enc.shape[0], 1)))
        lg, _ = hybrid_forward(params, names, f, mk, PAMAP2_HEADS)
        assert rel_err(lg, fx["subset_logits"][s]) <= 1e-5, s
