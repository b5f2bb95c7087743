"""CPU restatement of the SequenceEncoder LSTM (ORACLE).

TEST INFRASTRUCTURE ONLY (same rules as ``oracle/hybrid_cpu.py``): only
``tests/`` may import it, as the checker; the package never does.

The reference's SequenceEncoder 'lstm' branch (src/encoders.py:67-75 builds
nn.LSTM(batch_first=True, dropout between layers), :135-166 runs it, packed by
``lengths`` when given, and projects ``dropout(h_n[-1])``).  The recurrence is
torch.nn.LSTM's (a third-party dependency of the reference; torch 2.10 here),
restated in float64 numpy with an explicit BPTT backward:

  pre_t = x_t W_ih^T + b_ih + h_{t-1} W_hh^T + b_hh      gates (i, f, g, o) = 4 H slices
  i, f, o = sigmoid(.), g = tanh(.);  c_t = f c_{t-1} + i g;  h_t = o tanh(c_t)
  packed sequences: h_n[b] = h_{len_b - 1}[b] (the recurrence is causal)

Pinning: ``tests/golden/gen_golden.py`` runs the reference's own
SequenceEncoder on seeded inputs (SEQENC_CASES); ``tests/test_oracle_golden.py``
checks this restatement against those outputs and gradients.
"""

from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np


def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


def lstm_forward(x: np.ndarray, w_ih: np.ndarray, w_hh: np.ndarray, b_ih: np.ndarray, b_hh: np.ndarray):
    """One layer, zero initial state.  x (B, T, D) -> h, c (B, T, H), gates (B, T, 4H) activated."""
    x = x.astype(np.float64)
    B, T, _ = x.shape
    H = w_hh.shape[1]
    xproj = x @ w_ih.astype(np.float64).T + (b_ih.astype(np.float64) + b_hh.astype(np.float64))
    whh = w_hh.astype(np.float64)
    h = np.zeros((B, T, H))
    c = np.zeros((B, T, H))
    gates = np.zeros((B, T, 4 * H))
    hp = np.zeros((B, H))
    cp = np.zeros((B, H))
    for t in range(T):
        pre = xproj[:, t] + hp @ whh.T
        i, f = _sig(pre[:, :H]), _sig(pre[:, H:2 * H])
        g, o = np.tanh(pre[:, 2 * H:3 * H]), _sig(pre[:, 3 * H:])
        cp = f * cp + i * g
        hp = o * np.tanh(cp)
        h[:, t], c[:, t] = hp, cp
        gates[:, t] = np.concatenate([i, f, g, o], axis=1)
    return h, c, gates


def lstm_backward(w_hh: np.ndarray, c: np.ndarray, gates: np.ndarray, dh: np.ndarray) -> np.ndarray:
    """BPTT: dh (B, T, H) upstream gradient of every h_t -> dgates (B, T, 4H), the gradient of
    the pre-activation gates (= d xproj; dW_hh = sum_t dgates_t^T h_{t-1})."""
    B, T, H = c.shape
    whh = w_hh.astype(np.float64)
    dgates = np.zeros((B, T, 4 * H))
    dh_rec = np.zeros((B, H))
    dc = np.zeros((B, H))
    for t in range(T - 1, -1, -1):
        i, f = gates[:, t, :H], gates[:, t, H:2 * H]
        g, o = gates[:, t, 2 * H:3 * H], gates[:, t, 3 * H:]
        ct = c[:, t]
        cprev = c[:, t - 1] if t > 0 else np.zeros_like(ct)
        d = dh[:, t] + dh_rec
        tc = np.tanh(ct)
        dc = dc + d * o * (1 - tc * tc)
        dg = np.concatenate([dc * g * i * (1 - i), dc * cprev * f * (1 - f), dc * i * (1 - g * g),
                             d * tc * o * (1 - o)], axis=1)
        dgates[:, t] = dg
        dc = dc * f
        dh_rec = dg @ whh
    return dgates


def sequence_encoder(params: Dict[str, np.ndarray], layers: int, x: np.ndarray, lengths: Optional[np.ndarray],
                     g_out: np.ndarray) -> Tuple[np.ndarray, np.ndarray, np.ndarray, Dict[str, np.ndarray]]:
    """SequenceEncoder.forward in eval mode and the gradients of sum(encoding * g_out):
    returns (encoding, top-layer outputs, d sequence, {param: grad})."""
    B, T, _ = x.shape
    cur = x.astype(np.float64)
    saved: List[tuple] = []
    for k in range(layers):
        w_ih, w_hh = params[f"rnn.weight_ih_l{k}"], params[f"rnn.weight_hh_l{k}"]
        h, c, gates = lstm_forward(cur, w_ih, w_hh, params[f"rnn.bias_ih_l{k}"], params[f"rnn.bias_hh_l{k}"])
        saved.append((cur, h, c, gates))
        cur = h
    last = np.full(B, T - 1) if lengths is None else np.asarray(lengths, dtype=np.int64) - 1
    final = cur[np.arange(B), last]                                   # (B, H)
    pw, pb = params["projection.weight"].astype(np.float64), params["projection.bias"].astype(np.float64)
    enc = final @ pw.T + pb
    grads: Dict[str, np.ndarray] = {}
    g = g_out.astype(np.float64)
    grads["projection.weight"] = g.T @ final
    grads["projection.bias"] = g.sum(0)
    dh = np.zeros_like(cur)
    dh[np.arange(B), last] = g @ pw
    for k in range(layers - 1, -1, -1):
        xin, h, c, gates = saved[k]
        w_ih, w_hh = params[f"rnn.weight_ih_l{k}"].astype(np.float64), params[f"rnn.weight_hh_l{k}"]
        dg = lstm_backward(w_hh, c, gates, dh)
        H = h.shape[2]
        dg2 = dg.reshape(B * T, 4 * H)
        grads[f"rnn.weight_ih_l{k}"] = dg2.T @ xin.reshape(B * T, -1)
        grads[f"rnn.weight_hh_l{k}"] = dg[:, 1:].reshape(-1, 4 * H).T @ h[:, :-1].reshape(-1, H)
        grads[f"rnn.bias_ih_l{k}"] = dg2.sum(0)
        grads[f"rnn.bias_hh_l{k}"] = dg2.sum(0)
        dh = (dg2 @ w_ih).reshape(xin.shape)
    return enc, cur, dh, grads
