"""FrameEncoder with its attention pooling on the HIP path.

Mirrors src/encoders.py::FrameEncoder (:210-336) of the reference: the same
constructor (frame_dim, hidden_dim=256, output_dim=128,
temporal_pooling="attention", dropout=0.1), attributes and state_dict keys
(frame_processor.0.*, attention.*, projection.0.*, projection.3.*), the same
forward(frames, mask=None) and the same errors:

  * ValueError("Unknown pooling: ...") at construction (:246-247);
  * ValueError("Expected 3D frame tensor, got shape ...") (:275-278);
  * ValueError("Unknown pooling strategy: ...") at run time (:306-309);
  * RuntimeError("Attention layer not initialized.") from attention_pool (:330-331).

attention_pool (:313-336) -- scores = attention(frames), -inf where mask == 0,
softmax over frames, nan_to_num, weighted sum -- runs forward and backward as
the HIP kernels behind mmf_attention_pool_forward / _backward
(csrc/softmax_pool.hip).  The frame MLP and the projection are nn.Linear
layers on PyTorch-ROCm (encoders are outside the fused path), and the
'average' / 'max' pooling branches stay plain torch (:288-305).  
SequenceEncoder (src/encoders.py:34-166) mirrors the
reference's 'lstm' branch: the same constructor, parameter names
(rnn.weight_ih_l{k}, rnn.weight_hh_l{k}, rnn.bias_*, projection.*), forward
(sequence, lengths=None) and errors.  The recurrence runs as one persistent
HIP launch per layer (csrc/lstm.hip, mmf_lstm_forward / _backward); the
time-parallel input projection and weight gradients are rocBLAS GEMMs.
``encode_sequences`` batches the LSTMs of several modalities into the same
launches.  The recurrence's workgroups wait on each other: the library refuses
a grid that cannot be co-resident, every launch gets a fresh timeout word, and
a wait that gives up poisons its outputs with NaN; ``lstm_timed_out()`` /
``check_lstm_timeouts()`` report such launches (one stream sync per check).  The 'gru' / 'cnn' / 'transformer' encoder types are not on the
path and raise NotImplementedError.
"""

from __future__ import annotations

import os
import sys
from typing import Any, Dict, List, Optional, Sequence, cast

import torch
import torch.nn as nn

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import mmf_native as _nat  # noqa: E402
import mmf_ops as _ops  # noqa: E402


def attention_pool(frames: torch.Tensor, attention: nn.Linear, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Learned-score softmax pooling over the frame axis (src/encoders.py:313-336) on HIP."""
    _nat.require_device(frames, "FrameEncoder input")
    frames = _nat.f32c(frames)
    m = None
    if mask is not None:
        m = mask.to(device=frames.device, dtype=torch.float32).contiguous()
        if m.shape != frames.shape[:2]:
            raise ValueError(f"mask shape {tuple(m.shape)} does not match frames {tuple(frames.shape[:2])}")
    pooled, _ = torch.ops.mmfusion.attention_pool_fwd(frames, attention.weight, attention.bias, m)
    return pooled


class FrameEncoder(nn.Module):
    """Frame-level features -> video-level embedding (src/encoders.py:210-310)."""

    temporal_pooling: str
    attention: Optional[nn.Linear]

    def __init__(self, frame_dim: int, hidden_dim: int = 256, output_dim: int = 128,
                 temporal_pooling: str = "attention", dropout: float = 0.1):
        super().__init__()
        cast_self = cast(Any, self)
        cast_self.temporal_pooling = temporal_pooling
        self.frame_processor = nn.Sequential(nn.Linear(frame_dim, hidden_dim), nn.ReLU(), nn.Dropout(dropout))
        cast_self.attention = None
        if temporal_pooling == "attention":
            cast_self.attention = nn.Linear(hidden_dim, 1)
        elif temporal_pooling not in ("average", "max"):
            raise ValueError(f"Unknown pooling: {temporal_pooling}")
        self.projection = nn.Sequential(nn.Linear(hidden_dim, hidden_dim), nn.ReLU(), nn.Dropout(dropout),
                                        nn.Linear(hidden_dim, output_dim))

    def forward(self, frames: torch.Tensor, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        if frames.dim() != 3:
            raise ValueError(f"Expected 3D frame tensor, got shape {frames.shape}")
        processed = self.frame_processor(frames)
        if mask is not None:
            mask = mask.to(device=processed.device, dtype=processed.dtype)
        if self.temporal_pooling == "attention":
            pooled = self.attention_pool(processed, mask)
        elif self.temporal_pooling == "average":
            if mask is None:
                pooled = processed.mean(dim=1)
            else:
                wts = mask.unsqueeze(-1)
                pooled = (processed * wts).sum(dim=1) / wts.sum(dim=1).clamp_min(1e-8)
        elif self.temporal_pooling == "max":
            if mask is None:
                pooled = processed.max(dim=1).values
            else:
                pooled = processed.masked_fill(mask.unsqueeze(-1) == 0, float("-inf")).max(dim=1).values
                pooled = torch.nan_to_num(pooled, nan=0.0, neginf=0.0)
        else:
            raise ValueError(f"Unknown pooling strategy: {self.temporal_pooling}")
        return self.projection(pooled)

    def attention_pool(self, frames: torch.Tensor, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        if self.attention is None:
            raise RuntimeError("Attention layer not initialized.")
        return attention_pool(frames, self.attention, mask)


# ---------------------------------------------------------------------------
# SequenceEncoder (LSTM) on the persistent HIP recurrence
# ---------------------------------------------------------------------------

_LSTM_TIMEOUT: Dict[int, torch.Tensor] = {}


def _timeout_flag(dev: torch.device) -> torch.Tensor:
    """A fresh timeout word for one LSTM launch (the library zeroes it on the stream)."""
    return torch.zeros(1, dtype=torch.int32, device=dev)


def _timeout_acc(dev: torch.device) -> torch.Tensor:
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    t = _LSTM_TIMEOUT.get(idx)
    if t is None:
        t = torch.zeros(1, dtype=torch.int32, device=dev)
        _LSTM_TIMEOUT[idx] = t
    return t


def _record_timeout(flag: torch.Tensor) -> None:
    # device-side OR into the per-device accumulator: no host sync, graph-capturable
    _timeout_acc(flag.device).bitwise_or_(flag)


def _drain_op_flags() -> None:
    """Fold the timeout words of the eager LSTM operator launches (mmf_ops.LSTM_FLAGS)."""
    while _ops.LSTM_FLAGS:
        flag = _ops.LSTM_FLAGS.pop()
        if _ops.eager_tensor(flag):
            _record_timeout(flag)


def lstm_timed_out(device=None, reset: bool = True) -> bool:
    """True if any LSTM launch on `device` since the last check gave up an inter-workgroup
    wait.  Such a launch also writes NaN into the values it never received, so its
    encodings / gradients are NaN, never silently wrong.  Reading syncs the stream;
    call it once per step (or per epoch) rather than per launch."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    _drain_op_flags()
    acc = _timeout_acc(dev)
    hit = bool(int(acc.item()))
    if reset:
        acc.zero_()
    return hit


def check_lstm_timeouts(device=None) -> None:
    """Raise RuntimeError if an LSTM launch timed out since the last check (see lstm_timed_out)."""
    if lstm_timed_out(device):
        raise RuntimeError("mmfusion LSTM recurrence: an inter-workgroup wait timed out (the grid was not "
                           "fully co-resident); the affected encodings / gradients are NaN")


class LSTM(nn.Module):
    """nn.LSTM's constructor, attributes, parameter names / shapes / registration order and
    initialisation (uniform(-1/sqrt(hidden), 1/sqrt(hidden)) over the parameters in order), so
    the same seed gives the same weights and state dicts load either way -- but not an
    nn.RNNBase: TorchDynamo refuses to trace RNNBase modules at all ("Attempted to wrap RNN"),
    which would break the reference's torch.compile of its encoders (src/train.py:203-214).
    The recurrence runs on HIP (csrc/lstm.hip) through lstm_layers.  Supported: biased,
    unidirectional, no projection, zero initial state (the reference's configuration,
    src/encoders.py:68-76)."""

    def __init__(self, input_size: int, hidden_size: int, num_layers: int = 1, bias: bool = True,
                 batch_first: bool = False, dropout: float = 0.0, bidirectional: bool = False, proj_size: int = 0):
        super().__init__()
        if not bias or bidirectional or proj_size:
            raise NotImplementedError("LSTM path: biased, unidirectional, no projection")
        if num_layers < 1:
            raise ValueError("num_layers must be >= 1")
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.bias, self.batch_first, self.dropout = bias, batch_first, float(dropout)
        self.bidirectional, self.proj_size = False, 0
        for k in range(num_layers):
            din = input_size if k == 0 else hidden_size
            self.register_parameter(f"weight_ih_l{k}", nn.Parameter(torch.empty(4 * hidden_size, din)))
            self.register_parameter(f"weight_hh_l{k}", nn.Parameter(torch.empty(4 * hidden_size, hidden_size)))
            self.register_parameter(f"bias_ih_l{k}", nn.Parameter(torch.empty(4 * hidden_size)))
            self.register_parameter(f"bias_hh_l{k}", nn.Parameter(torch.empty(4 * hidden_size)))
        self.reset_parameters()

    def reset_parameters(self) -> None:
        stdv = 1.0 / (self.hidden_size ** 0.5) if self.hidden_size > 0 else 0.0
        for w in self.parameters():
            nn.init.uniform_(w, -stdv, stdv)

    def extra_repr(self) -> str:
        s = f"{self.input_size}, {self.hidden_size}, num_layers={self.num_layers}"
        if self.batch_first:
            s += ", batch_first=True"
        if self.dropout:
            s += f", dropout={self.dropout}"
        return s

    def forward(self, input: torch.Tensor, hx=None):
        """-> output, (h_n, c_n) as nn.LSTM (zero initial state only).  c_n carries no gradient:
        the recurrence's backward takes d(h) only, which is all the encoders use."""
        if hx is not None:
            raise NotImplementedError("LSTM path: zero initial state only")
        if input.dim() != 3:
            raise ValueError(f"Expected 3-D input, got shape {tuple(input.shape)}")
        x = input if self.batch_first else input.transpose(0, 1)
        finals: List[tuple] = []
        out = lstm_layers([self], [x], finals)[0]
        h_n = torch.stack([h for h, _ in finals])
        c_n = torch.stack([c for _, c in finals]).detach()
        return (out if self.batch_first else out.transpose(0, 1)), (h_n, c_n)


def lstm_layers(rnns: Sequence[LSTM], inputs: Sequence[torch.Tensor],
                finals: Optional[List[tuple]] = None) -> List[torch.Tensor]:
    """Run several LSTM parameter sets (batch_first inputs, zero initial state) over their inputs on
    the HIP recurrence, every layer of all of them in one launch; returns each LSTM's top-layer
    output sequence (B, T, H).  Inter-layer dropout follows nn.LSTM (training only).  With
    `finals`, the first LSTM's last (h, c) of every layer is appended to it."""
    n = len(rnns)
    if n == 0:
        return []
    H = rnns[0].hidden_size
    layers = rnns[0].num_layers
    for r in rnns:
        if not r.bias or r.bidirectional or r.proj_size:
            raise NotImplementedError("LSTM path: unidirectional, biased, no projection")
        if r.hidden_size != H or r.num_layers != layers:
            raise ValueError("lstm_layers: all LSTMs need the same hidden_size and num_layers")
    B, T = inputs[0].shape[:2]
    for x in inputs:
        _nat.require_device(x, "SequenceEncoder input")
        if x.shape[:2] != (B, T):
            raise ValueError("lstm_layers: all sequences need the same (batch, seq_len)")
    cur = list(inputs)
    for k in range(layers):
        # time-parallel input projection on PyTorch-ROCm (xproj = x W_ih^T + b_ih + b_hh; autograd
        # gives dx, dW_ih, db), the recurrence as one persistent HIP launch for all LSTMs
        xproj = []
        for r, x in zip(rnns, cur):
            x2 = _nat.f32c(x).reshape(B * T, -1)
            b = getattr(r, f"bias_ih_l{k}") + getattr(r, f"bias_hh_l{k}")
            xproj.append(torch.addmm(b, x2, getattr(r, f"weight_ih_l{k}").t()).view(B, T, -1))
        hs, cs, _gates, flag = torch.ops.mmfusion.lstm_layer_fwd(
            xproj, [_nat.f32c(getattr(r, f"weight_hh_l{k}")) for r in rnns])
        if _ops.eager_tensor(flag):
            _record_timeout(flag)
        if finals is not None:
            finals.append((hs[0][:, -1], cs[0][:, -1]))
        cur = list(hs)
        if k + 1 < layers:
            cur = [torch.nn.functional.dropout(o, rnns[i].dropout, rnns[i].training) for i, o in enumerate(cur)]
    return cur


def _final_state(out: torch.Tensor, lengths: Optional[torch.Tensor]) -> torch.Tensor:
    if lengths is None:
        return out[:, -1]
    idx = lengths.to(device=out.device, dtype=torch.int64) - 1
    if bool((idx < 0).any()) or bool((idx >= out.shape[1]).any()):
        raise RuntimeError("lengths must be in [1, seq_len]")
    return out[torch.arange(out.shape[0], device=out.device), idx]


class SequenceEncoder(nn.Module):
    """Time-series sequence -> fixed embedding (src/encoders.py:22-166), 'lstm' on the HIP path."""

    encoder_type: str
    hidden_dim: int
    output_dim: int
    rnn: Optional[LSTM]
    conv_net: Optional[nn.Module]
    pool: Optional[nn.Module]
    input_projection: Optional[nn.Linear]
    transformer: Optional[nn.TransformerEncoder]
    projection: nn.Module

    def __init__(self, input_dim: int, hidden_dim: int = 256, output_dim: int = 128, num_layers: int = 2,
                 encoder_type: str = "lstm", dropout: float = 0.1):
        super().__init__()
        cast_self = cast(Any, self)
        cast_self.encoder_type = encoder_type
        cast_self.hidden_dim = hidden_dim
        cast_self.output_dim = output_dim
        self.dropout_layer = nn.Dropout(dropout)
        cast_self.rnn = None
        cast_self.conv_net = None
        cast_self.pool = None
        cast_self.input_projection = None
        cast_self.transformer = None
        self.projection = nn.Identity()
        if encoder_type == "lstm":
            cast_self.rnn = LSTM(input_dim, hidden_dim, num_layers=num_layers, batch_first=True,
                                 dropout=dropout if num_layers > 1 else 0.0)
            self.projection = nn.Linear(hidden_dim, output_dim)
        elif encoder_type in ("gru", "cnn", "transformer"):
            raise NotImplementedError(f"encoder_type '{encoder_type}' is not on the MI355X path (only 'lstm')")
        else:
            raise ValueError(f"Unknown encoder type: {encoder_type}")

    def encode_final_state(self, final_state: torch.Tensor) -> torch.Tensor:
        return self.projection(self.dropout_layer(final_state))

    def forward(self, sequence: torch.Tensor, lengths: Optional[torch.Tensor] = None) -> torch.Tensor:
        if sequence.dim() != 3:
            raise ValueError(f"Expected 3D input sequence, got shape {sequence.shape}")
        if self.rnn is None:
            raise RuntimeError("RNN module not initialized.")
        out = lstm_layers([self.rnn], [sequence])[0]
        return self.encode_final_state(_final_state(out, lengths))


def encode_sequences(encoders: Dict[str, SequenceEncoder], sequences: Dict[str, torch.Tensor],
                     lengths: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
    """{m: encoders[m](sequences[m], lengths)} with every modality's LSTM layers sharing launches
    (the modalities of one chunk have the same (B, T))."""
    names = list(sequences)
    for m in names:
        if sequences[m].dim() != 3:
            raise ValueError(f"Expected 3D input sequence, got shape {sequences[m].shape}")
    rnns = []
    for m in names:
        r = encoders[m].rnn
        if r is None:
            raise RuntimeError("RNN module not initialized.")
        rnns.append(r)
    outs = lstm_layers(rnns, [sequences[m] for m in names])
    return {m: encoders[m].encode_final_state(_final_state(o, lengths)) for m, o in zip(names, outs)}
