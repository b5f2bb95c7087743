"""SequenceEncoder LSTM on the persistent HIP recurrence (SURVEY §8f rank 3,
src/encoders.py:34-166): the module against fixtures the reference produced
(tests/golden/gen_golden.py, SEQENC_CASES), the raw C-ABI recurrence against
the CPU oracle (oracle/lstm_cpu.py) including batch instances of <= 4 rows and
several LSTMs per launch, and the C3 shape (T = 1024, H = 256) at full length.
Tolerance: 1e-3 relative (BASELINE.json fp32 parity)."""
import ctypes

import numpy as np
import pytest
import torch

from _util import close, load_fixture, rel_err
from cases import SEQENC_CASES, seqenc_inputs, seqenc_state

TOL = 1e-3


@pytest.fixture(scope="module")
def enc_mod(pkg_on_path):
    import encoders
    return encoders


@pytest.fixture(scope="module")
def nat(pkg_on_path):
    import mmf_native
    return mmf_native


def test_sequence_encoder_surface_cpu(enc_mod):
    """Constructor / validation of the reference (src/encoders.py:113-114, 129-132)."""
    with pytest.raises(ValueError, match="Unknown encoder type"):
        enc_mod.SequenceEncoder(8, encoder_type="rnn")
    for kind in ("gru", "cnn", "transformer"):
        with pytest.raises(NotImplementedError):
            enc_mod.SequenceEncoder(8, encoder_type=kind)
    e = enc_mod.SequenceEncoder(8, 64, 16, num_layers=2)
    assert sorted(e.state_dict()) == sorted(
        ["projection.weight", "projection.bias"]
        + [f"rnn.{p}_l{k}" for k in range(2) for p in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")])
    assert e.rnn.dropout == 0.1 and e.hidden_dim == 64 and e.output_dim == 16
    with pytest.raises(ValueError, match="Expected 3D input sequence"):
        e(torch.randn(4, 8))
    with pytest.raises(RuntimeError, match="ROCm device"):
        e(torch.randn(2, 5, 8))


def test_lstm_limits_cpu(nat):
    """Host-side validation returns MMF_ELIMIT before touching the device."""
    L = nat.lib()
    assert L.mmf_lstm_sync_bytes(3, 256) == 2 * 4 * 3 * 256 * 8
    null = nat.ptr_array([0])
    for n, B, T, H in ((1, 1, 4, 96), (1, 1, 4, 320), (9, 1, 4, 64), (4, 33, 4, 64), (1, 0, 4, 64)):
        rc = L.mmf_lstm_forward(n, B, T, H, null, null, null, null, null, null, None, None)
        assert rc == 2, (n, B, T, H)
        rc = L.mmf_lstm_backward(n, B, T, H, null, null, null, null, null, null, None, None)
        assert rc == 2, (n, B, T, H)


def _run_recurrence(nat, enc_mod, xproj_l, w_hh_l, dh_l):
    """Raw C-ABI forward + backward for n LSTMs on cuda:0."""
    L = nat.lib()
    dev = torch.device("cuda", 0)
    n = len(xproj_l)
    B, T, H4 = xproj_l[0].shape
    H = H4 // 4
    xp = [torch.from_numpy(x.astype(np.float32)).to(dev) for x in xproj_l]
    wh = [torch.from_numpy(w.astype(np.float32)).to(dev) for w in w_hh_l]
    h = [torch.empty(B, T, H, device=dev) for _ in range(n)]
    c = [torch.empty(B, T, H, device=dev) for _ in range(n)]
    g = [torch.empty(B, T, 4 * H, device=dev) for _ in range(n)]
    sync = [torch.empty(L.mmf_lstm_sync_bytes(B, H), dtype=torch.uint8, device=dev) for _ in range(n)]
    tmo = torch.zeros(1, dtype=torch.int32, device=dev)
    arr = lambda ts: nat.ptr_array([t.data_ptr() for t in ts])  # noqa: E731
    st = nat.stream_ptr(dev)
    rc = L.mmf_lstm_forward(n, B, T, H, arr(xp), arr(wh), arr(h), arr(c), arr(g), arr(sync), tmo.data_ptr(), st)
    assert rc == 0, nat.lib().mmf_last_error()
    dh = [torch.from_numpy(d.astype(np.float32)).to(dev) for d in dh_l]
    dg = [torch.empty(B, T, 4 * H, device=dev) for _ in range(n)]
    rc = L.mmf_lstm_backward(n, B, T, H, arr(wh), arr(c), arr(g), arr(dh), arr(dg), arr(sync), tmo.data_ptr(), st)
    assert rc == 0, nat.lib().mmf_last_error()
    torch.cuda.synchronize(dev)
    assert int(tmo.item()) == 0, "inter-workgroup wait timed out"
    cpu = lambda ts: [t.cpu().double().numpy() for t in ts]  # noqa: E731
    return cpu(h), cpu(c), cpu(g), cpu(dg)


@pytest.mark.gpu
@pytest.mark.parametrize("n,B,T,H", [(1, 1, 7, 64), (3, 5, 33, 64), (2, 4, 20, 192), (4, 9, 16, 256)])
def test_recurrence_matches_oracle(nat, enc_mod, n, B, T, H):
    from oracle.lstm_cpu import lstm_backward, lstm_forward
    rng = np.random.default_rng(1000 * n + B + T + H)
    bound = 1.0 / np.sqrt(H)
    xproj_l, w_l, dh_l, ref = [], [], [], []
    for _ in range(n):
        xproj = rng.standard_normal((B, T, 4 * H)).astype(np.float32)
        w = rng.uniform(-bound, bound, size=(4 * H, H)).astype(np.float32)
        dh = rng.standard_normal((B, T, H)).astype(np.float32)
        # the oracle takes x W_ih^T + b: identity input weights reproduce xproj
        h, c, g = lstm_forward(xproj, np.eye(4 * H, dtype=np.float32), w, np.zeros(4 * H, np.float32),
                               np.zeros(4 * H, np.float32))
        ref.append((h, c, g, lstm_backward(w, c, g, dh)))
        xproj_l.append(xproj); w_l.append(w); dh_l.append(dh)
    hs, cs, gs, dgs = _run_recurrence(nat, enc_mod, xproj_l, w_l, dh_l)
    for i in range(n):
        h, c, g, dg = ref[i]
        assert rel_err(torch.from_numpy(hs[i]), h) <= TOL, i
        assert rel_err(torch.from_numpy(cs[i]), c) <= TOL, i
        assert rel_err(torch.from_numpy(gs[i]), g) <= TOL, i
        assert rel_err(torch.from_numpy(dgs[i]), dg) <= TOL, i


@pytest.mark.gpu
def test_recurrence_c3_length(nat, enc_mod):
    """The C3 chunk: T = 1024 steps, H = 256, one row, all 4 modalities in one launch."""
    from oracle.lstm_cpu import lstm_backward, lstm_forward
    rng = np.random.default_rng(7)
    n, B, T, H = 4, 1, 1024, 256
    bound = 1.0 / np.sqrt(H)
    xproj_l = [rng.standard_normal((B, T, 4 * H)).astype(np.float32) for _ in range(n)]
    w_l = [rng.uniform(-bound, bound, size=(4 * H, H)).astype(np.float32) for _ in range(n)]
    dh_l = [np.zeros((B, T, H), np.float32) for _ in range(n)]
    for d in dh_l:
        d[:, -1] = rng.standard_normal((B, H))       # only the final state feeds the projection
    hs, cs, gs, dgs = _run_recurrence(nat, enc_mod, xproj_l, w_l, dh_l)
    eye, z = np.eye(4 * H, dtype=np.float32), np.zeros(4 * H, np.float32)
    for i in (0, 3):
        h, c, g = lstm_forward(xproj_l[i], eye, w_l[i], z, z)
        assert rel_err(torch.from_numpy(hs[i]), h) <= TOL
        assert rel_err(torch.from_numpy(dgs[i]), lstm_backward(w_l[i], c, g, dh_l[i])) <= TOL


def _module(enc_mod, case):
    m = enc_mod.SequenceEncoder(case.input_dim, hidden_dim=case.hidden, output_dim=case.out_dim,
                                num_layers=case.layers, encoder_type="lstm", dropout=0.1)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in seqenc_state(case).items()}, strict=True)
    return m.to("cuda:0").eval()


@pytest.mark.gpu
@pytest.mark.parametrize("case", SEQENC_CASES, ids=lambda c: c.name)
def test_sequence_encoder_matches_reference(enc_mod, case):
    fx = load_fixture(case.name)
    model = _module(enc_mod, case)
    seq_np, len_np, g_out = seqenc_inputs(case)
    seq = torch.from_numpy(seq_np).to("cuda:0").requires_grad_(True)
    lengths = torch.from_numpy(len_np) if len_np is not None else None
    enc = model(seq, lengths)
    (enc * torch.from_numpy(g_out).to("cuda:0")).sum().backward()
    assert rel_err(enc.detach(), fx["encoding"]) <= TOL
    assert rel_err(seq.grad, fx["dsequence"]) <= TOL
    for name, p in model.named_parameters():
        assert close(p.grad, fx[f"grad/{name}"], TOL, 1e-7), name
    assert not enc_mod.lstm_timed_out("cuda:0")


@pytest.mark.gpu
def test_encode_sequences_batches_modalities(enc_mod):
    """Several modalities' LSTMs in shared launches == each encoder on its own."""
    torch.manual_seed(3)
    dims = {"imu_hand": 17, "imu_chest": 17, "heart_rate": 1}
    encs = {m: enc_mod.SequenceEncoder(d, 128, 32, num_layers=2).to("cuda:0").eval() for m, d in dims.items()}
    seqs = {m: torch.randn(3, 40, d, device="cuda:0") for m, d in dims.items()}
    lengths = torch.tensor([40, 17, 2])
    together = enc_mod.encode_sequences(encs, seqs, lengths)
    for m in dims:
        alone = encs[m](seqs[m], lengths)
        assert torch.equal(together[m], alone), m


def test_lstm_module_matches_torch_layout_cpu(enc_mod):
    """encoders.LSTM keeps nn.LSTM's parameter names, shapes, order and initialisation (same seed ->
    same weights, state dicts interchangeable) without being an nn.RNNBase (Dynamo refuses those)."""
    for layers, first in ((1, True), (2, True), (3, False)):
        torch.manual_seed(11)
        ref = torch.nn.LSTM(9, 32, num_layers=layers, batch_first=first, dropout=0.2 if layers > 1 else 0.0)
        torch.manual_seed(11)
        mine = enc_mod.LSTM(9, 32, num_layers=layers, batch_first=first, dropout=0.2 if layers > 1 else 0.0)
        assert not isinstance(mine, torch.nn.RNNBase)
        a, b = ref.state_dict(), mine.state_dict()
        assert list(a) == list(b)
        assert all(torch.equal(a[k], b[k]) for k in a)
        mine.load_state_dict(a)
        assert (mine.hidden_size, mine.num_layers, mine.batch_first) == (32, layers, first)
    with pytest.raises(NotImplementedError):
        enc_mod.LSTM(9, 32, bidirectional=True)
    with pytest.raises(NotImplementedError):
        enc_mod.LSTM(9, 32, proj_size=8)


@pytest.mark.gpu
@pytest.mark.parametrize("batch_first", [True, False])
def test_lstm_module_forward_matches_torch(enc_mod, batch_first):
    """LSTM(...)(x) -> output, (h_n, c_n) on the HIP recurrence == torch's nn.LSTM with the
    same weights; d(input) and parameter gradients through output and h_n."""
    torch.manual_seed(5)
    # train mode (MIOpen's RNN backward refuses eval mode), no dropout: deterministic
    ref = torch.nn.LSTM(12, 64, num_layers=2, batch_first=batch_first).to("cuda:0").train()
    mine = enc_mod.LSTM(12, 64, num_layers=2, batch_first=batch_first).to("cuda:0").train()
    mine.load_state_dict(ref.state_dict())
    x = torch.randn(3, 25, 12, device="cuda:0")
    if not batch_first:
        x = x.transpose(0, 1).contiguous()
    outs = []
    for m in (ref, mine):
        xi = x.clone().requires_grad_(True)
        out, (h, c) = m(xi)
        (out.square().sum() + h.sum()).backward()
        outs.append((out.detach(), h.detach(), c.detach(), xi.grad, [p.grad for p in m.parameters()]))
    (ro, rh, rc, rdx, rg), (mo, mh, mc, mdx, mg) = outs
    assert mo.shape == ro.shape and mh.shape == rh.shape == (2, 3, 64) and mc.shape == rc.shape
    for a, b in ((mo, ro), (mh, rh), (mc, rc), (mdx, rdx)):
        assert rel_err(a, b.double().cpu().numpy()) <= TOL
    for a, b in zip(mg, rg):
        assert rel_err(a, b.double().cpu().numpy()) <= TOL
