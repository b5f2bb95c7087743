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


# --------------------------------------------------------------------------- C3 as stated
def _bins(conf, nb=15):
    """The 15 equal-width bins of src/uncertainty.py:84-131 (last bin closed)."""
    return torch.clamp((conf * nb).floor().long(), max=nb - 1)


def test_pamap2_medium_bf16_bounds(setup, pkg_on_path):
    """BASELINE.json C3 runs HybridFusion in bf16 (training.matmul_precision "medium",
    config/base.yaml:80).  At the PAMAP2 shape (M = 4, D = 128, H = 256, C = 25) against the
    reference's fp32 logits: SURVEY §8d's bf16 bounds -- logits max|d| <= 3e-2 max|ref|, argmax
    agreement >= 99 % -- and the calibration metrics within the bound their definition gives:
    ECE moves by at most mean|d conf| while no sample changes bin, and by at most 2/N more per
    sample that does (|acc - conf| <= 1); MCE by at most max|d conf| when no sample changes bin."""
    model, cal, fx = setup
    import mmf_native as nat
    enc = fx["enc"]
    feats = {m: torch.from_numpy(enc[:, j]).cuda() for j, m in enumerate(PAMAP2_MODALITIES)}
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision("medium")
    try:
        nat.profile_begin()
        with torch.no_grad():
            logits = model(feats, torch.ones(enc.shape[0], len(PAMAP2_MODALITIES)).cuda())
        torch.cuda.synchronize()
        _, launches = nat.profile_end()
    finally:
        torch.set_float32_matmul_precision(prev)
    mfma = [k for _, k, *_ in launches if k.startswith(("gemm_lds", "gemm_wsr"))]
    assert mfma and all(k.endswith("1>") for k in mfma), mfma      # the bf16 instantiations ran
    ref = torch.from_numpy(fx["logits"]).double()
    got = logits.cpu().double()
    assert float((got - ref).abs().max()) <= 3e-2 * float(ref.abs().max())
    assert float((got.argmax(1) == ref.argmax(1)).double().mean()) >= 0.99
    out = cal.evaluate_logits(logits, torch.from_numpy(fx["labels"]))
    n = out["num_samples"]
    conf_ref = torch.from_numpy(fx["confidences"]).double()
    conf = torch.softmax(got, dim=1).max(dim=1).values
    moved = int((_bins(conf) != _bins(conf_ref)).sum())
    dconf = (conf - conf_ref).abs()
    assert abs(out["ece"] - float(fx["ece"][0])) <= float(dconf.mean()) + 2.0 * moved / n + 1e-6
    if moved == 0:
        assert abs(out["mce"] - float(fx["mce"][0])) <= float(dconf.max()) + 1e-6


@pytest.mark.parametrize("precision", ["highest", "medium"])
def test_pamap2_chain_end_to_end(setup, precision, tmp_path):
    """Config C3 end to end on the HIP path from RAW rows: the manifest loader (HBM table,
    one-launch chunk gather: mmf_gather_chunks) -> the four SequenceEncoder LSTMs (one
    persistent recurrence launch, csrc/lstm.hip) -> LayerNorm -> HybridFusion, for the first
    chunk of each present test shard (chunk 1024; tests/golden/gen_pamap2_chain.py), against
    the reference's encoder outputs and logits for the same chunks (pamap2_test.npz).  The
    encoders are built as the reference builds them (torch.manual_seed(42), build_encoder per
    config/base.yaml); their weights are checked against the reference's parameter sums.
    fp32 ("highest"): encodings 1e-3, logits 1e-3 of max|ref|.  bf16 ("medium", the fusion's
    MFMA operands; the LSTM recurrence stays fp32): logits 3e-2 of max|ref|, argmax equal."""
    model, _, fx = setup
    import encoders
    import harness
    from manifest import ManifestShards
    ch = load_fixture("pamap2_chain")
    columns = [str(c) for c in ch["columns"]]
    # the raw rows as .pt shards behind a manifest (the reference's on-disk format,
    # data/preprocess.py:130-139; manifest paths absolute, src/data.py:129-131)
    (tmp_path / "splits").mkdir()
    lines = []
    table = torch.from_numpy(ch["table"])
    for i in range(3):
        p = tmp_path / f"shard{i}.pt"
        torch.save({"columns": columns, "data": table[i * 1024:(i + 1) * 1024].clone()}, p)
        lines.append(f"{p},1024")
    (tmp_path / "splits" / "test.txt").write_text("\n".join(lines) + "\n")
    shards = ManifestShards(tmp_path, "test", PAMAP2_MODALITIES, chunk_size=1024)
    assert len(shards) == 3
    feats, labels, lens = shards.gather(torch.arange(3))
    assert labels.cpu().tolist() == fx["labels"][ch["test_index"]].tolist()
    torch.manual_seed(42)   # config/base.yaml:117, as the reference builds its encoders
    encs = {}
    for m in PAMAP2_MODALITIES:
        encs[m] = encoders.SequenceEncoder(shards.modality_dims[m], output_dim=PAMAP2_OUT_DIM,
                                           encoder_type="lstm", num_layers=1)
        s = sum(float(p.detach().double().sum()) for p in encs[m].parameters())
        assert s == float(ch[f"encoder_checksum/{m}"][0]), m
    full = harness.MultimodalFusionModel(encs, model, PAMAP2_OUT_DIM, layer_norm=True).cuda().eval()
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision(precision)
    try:
        with torch.no_grad():
            enc = full.encode(feats)
            logits = full.fusion_model(enc, torch.ones(3, len(PAMAP2_MODALITIES), device="cuda"))
        torch.cuda.synchronize()
    finally:
        torch.set_float32_matmul_precision(prev)
    idx = ch["test_index"]
    ref_enc = torch.from_numpy(fx["enc"][idx])
    got_enc = torch.stack([enc[m].cpu() for m in PAMAP2_MODALITIES], dim=1)
    ref = torch.from_numpy(fx["logits"][idx])
    if precision == "highest":
        assert close(got_enc, ref_enc, 1e-3, 1e-5)
        assert close(logits.cpu(), ref, 1e-3, 1e-5)
    else:
        assert float((got_enc - ref_enc).abs().max()) <= 3e-2 * float(ref_enc.abs().max())
        assert float((logits.cpu() - ref).abs().max()) <= 3e-2 * float(ref.abs().max())
    assert torch.equal(logits.cpu().argmax(1), ref.argmax(1))
