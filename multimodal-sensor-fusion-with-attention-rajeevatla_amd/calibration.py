"""Caller-side evaluation of HybridFusion logits: accuracy, ECE, MCE, NLL.

The reference evaluates a trained model by running it over the test split
(src/eval.py:39-130: ``logits = model(features, mask)`` :80, ``softmax`` and
``max`` :89-90, accuracy :103) and scoring the confidences with
``CalibrationMetrics`` (src/uncertainty.py:74-192; 15 bins from
``evaluation.num_calibration_bins``, src/eval.py:563-565).  This module restates
that chain for the logits the HIP path produces, so a PAMAP2 evaluation on
MI355X reports the same numbers the reference does (tests/test_gpu_pamap2.py).

It is a separate module name (not ``uncertainty``) so that putting this package
ahead of ``src/`` on ``sys.path`` never shadows the reference's own
``uncertainty`` module, which carries much more (MC dropout, temperature
scaling) than the metrics needed here.

Binning (src/uncertainty.py:109-129): equal-width bins from
``torch.linspace(0, 1, num_bins + 1)`` (float32 edges); a confidence c falls in
bin [lo, hi) except the last bin, which is closed [lo, 1]; empty bins are
skipped; ECE = sum_b (n_b / N) |acc_b - conf_b|, MCE = max_b |acc_b - conf_b|.
"""

from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F


def _bin_membership(confidences: torch.Tensor, num_bins: int) -> torch.Tensor:
    """(N, num_bins) bool: bin b holds c iff lo_b <= c < hi_b (hi_b == 1: c <= 1)."""
    edges = torch.linspace(0.0, 1.0, steps=num_bins + 1)
    lo, hi = edges[:-1], edges[1:]
    c = confidences.detach().cpu().to(torch.float32).reshape(-1, 1)
    below = torch.where(hi == 1.0, c <= hi, c < hi)
    return (c >= lo) & below


def _bin_stats(confidences, predictions, labels, num_bins: int):
    member = _bin_membership(confidences, num_bins)
    conf = confidences.detach().cpu().to(torch.float32).reshape(-1, 1)
    correct = (predictions.detach().cpu().reshape(-1, 1) == labels.detach().cpu().reshape(-1, 1)).to(torch.float32)
    count = member.sum(dim=0)
    denom = count.clamp_min(1).to(torch.float32)
    bin_conf = (conf * member).sum(dim=0) / denom
    bin_acc = (correct * member).sum(dim=0) / denom
    return count, (bin_acc - bin_conf).abs()


def expected_calibration_error(confidences: torch.Tensor, predictions: torch.Tensor, labels: torch.Tensor,
                               num_bins: int = 15) -> float:
    """src/uncertainty.py:84-131."""
    total = confidences.numel()
    if total == 0:
        return 0.0
    count, gap = _bin_stats(confidences, predictions, labels, num_bins)
    return float(((count.to(torch.float32) / total) * gap).sum())


def maximum_calibration_error(confidences: torch.Tensor, predictions: torch.Tensor, labels: torch.Tensor,
                              num_bins: int = 15) -> float:
    """src/uncertainty.py:133-171 (0 when every bin is empty)."""
    count, gap = _bin_stats(confidences, predictions, labels, num_bins)
    gap = torch.where(count > 0, gap, torch.zeros_like(gap))
    return float(gap.max()) if gap.numel() else 0.0


def negative_log_likelihood(logits: torch.Tensor, labels: torch.Tensor) -> float:
    """src/uncertainty.py:173-192: mean cross-entropy of the raw logits."""
    return float(F.cross_entropy(logits.detach().float().cpu(), labels.detach().cpu().long(), reduction="mean"))


def evaluate_logits(logits: torch.Tensor, labels: torch.Tensor, num_bins: int = 15) -> Dict[str, object]:
    """The src/eval.py:80-103 + src/uncertainty.py chain on a (N, C) logit matrix."""
    logits = logits.detach().float().cpu()
    labels = labels.detach().cpu().long()
    probs = torch.softmax(logits, dim=1)
    confidences, preds = torch.max(probs, dim=1)
    return {
        "accuracy": float((preds == labels).float().mean()),
        "ece": expected_calibration_error(confidences, preds, labels, num_bins),
        "mce": maximum_calibration_error(confidences, preds, labels, num_bins),
        "nll": negative_log_likelihood(logits, labels),
        "num_samples": int(labels.numel()),
        "confidences": confidences,
        "predictions": preds,
    }
