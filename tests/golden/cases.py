"""Deterministic parity cases shared by the fixture generator and the tests.

Test infrastructure only.  Every tensor here (weights, inputs, upstream
gradients) is a pure function of a seed through numpy's PCG64
(``numpy.random.default_rng``), which is stable across numpy versions, so the
GPU box can rebuild the exact inputs the golden outputs were produced from
without ever seeing ``/root/reference``.

Weight key names follow the reference's ``state_dict`` layout:
``projections.{m}.0.{weight,bias}`` (src/fusion.py:291-298),
``attention_modules.{q}_to_{k}.{query,key,value,out}_proj.{weight,bias}``
(src/fusion.py:300-314, src/attention.py:61-64),
``gating_layers.{m}.{weight,bias}`` (src/fusion.py:316-321),
``classifier.{0,3}.{weight,bias}`` (src/fusion.py:323-328).
Init bounds follow nn.Linear's default U(-1/sqrt(fan_in), 1/sqrt(fan_in)).
"""

from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np


def _linear(rng: np.random.Generator, out_f: int, in_f: int) -> Tuple[np.ndarray, np.ndarray]:
    bound = 1.0 / np.sqrt(max(in_f, 1))
    w = rng.uniform(-bound, bound, size=(out_f, in_f)).astype(np.float32)
    b = rng.uniform(-bound, bound, size=(out_f,)).astype(np.float32)
    return w, b


def pair_names(names: Sequence[str], deleted: Sequence[str] = ()) -> List[str]:
    out = []
    for q in names:
        for k in names:
            if q != k and f"{q}_to_{k}" not in deleted:
                out.append(f"{q}_to_{k}")
    return out


def hybrid_state(names: Sequence[str], dims: Dict[str, int], hidden: int,
                 num_classes: int, seed: int, deleted: Sequence[str] = ()) -> "OrderedDict[str, np.ndarray]":
    rng = np.random.default_rng(seed)
    sd: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for m in names:
        w, b = _linear(rng, hidden, dims[m])
        sd[f"projections.{m}.0.weight"] = w
        sd[f"projections.{m}.0.bias"] = b
    for q in names:
        for k in names:
            if q == k:
                continue
            for proj in ("query_proj", "key_proj", "value_proj", "out_proj"):
                w, b = _linear(rng, hidden, hidden)
                if f"{q}_to_{k}" in deleted:
                    continue  # keep the rng stream identical with/without deletion
                sd[f"attention_modules.{q}_to_{k}.{proj}.weight"] = w
                sd[f"attention_modules.{q}_to_{k}.{proj}.bias"] = b
    for m in names:
        w, b = _linear(rng, 1, hidden)
        sd[f"gating_layers.{m}.weight"] = w
        sd[f"gating_layers.{m}.bias"] = b
    w, b = _linear(rng, hidden, hidden)
    sd["classifier.0.weight"] = w
    sd["classifier.0.bias"] = b
    w, b = _linear(rng, num_classes, hidden)
    sd["classifier.3.weight"] = w
    sd["classifier.3.bias"] = b
    return sd


def cma_state(query_dim: int, key_dim: int, hidden: int, seed: int) -> "OrderedDict[str, np.ndarray]":
    rng = np.random.default_rng(seed)
    sd: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for proj, fan_in in (("query_proj", query_dim), ("key_proj", key_dim),
                         ("value_proj", key_dim), ("out_proj", hidden)):
        w, b = _linear(rng, hidden, fan_in)
        sd[f"{proj}.weight"] = w
        sd[f"{proj}.bias"] = b
    return sd


@dataclass
class HybridCase:
    """One HybridFusion parity case (eval mode: dropout is identity)."""
    name: str
    names: List[str]
    dims: Dict[str, int]
    seq: Dict[str, int]          # per-modality sequence length; 0 => 2-D (B, D) input
    batch: int
    hidden: int
    heads: int
    classes: int
    seed: int
    mask: Optional[List[List[float]]] = None     # explicit mask rows (cycled); None => seeded
    mask_keep: float = 1.0                       # seeded Bernoulli keep-rate when mask is None
    deleted: List[str] = field(default_factory=list)
    full: bool = True            # store full gradient tensors (small cases)
    attn_slice: int = 0          # > 0: store attention maps as flat[::attn_slice] (large maps)

    @property
    def seq_mode(self) -> bool:
        return any(v > 0 for v in self.seq.values())


def hybrid_inputs(case: HybridCase) -> Tuple[Dict[str, np.ndarray], np.ndarray, np.ndarray]:
    """Returns (features, mask (B,M) float32, upstream grad dlogits (B,C))."""
    rng = np.random.default_rng(case.seed + 7919)
    feats: Dict[str, np.ndarray] = {}
    for m in case.names:
        L = case.seq[m]
        shape = (case.batch, L, case.dims[m]) if L > 0 else (case.batch, case.dims[m])
        feats[m] = rng.standard_normal(shape).astype(np.float32)
    M = len(case.names)
    if case.mask is not None:
        rows = [case.mask[i % len(case.mask)] for i in range(case.batch)]
        mask = np.asarray(rows, dtype=np.float32)
    else:
        mask = (rng.uniform(size=(case.batch, M)) < case.mask_keep).astype(np.float32)
        # keep >= 1 modality per row except ~1% all-masked rows (SURVEY §8d C5 recipe)
        for b in range(case.batch):
            if mask[b].sum() == 0 and rng.uniform() > 0.01:
                mask[b, rng.integers(M)] = 1.0
    grad = rng.standard_normal((case.batch, case.classes)).astype(np.float32)
    return feats, mask, grad


@dataclass
class CMACase:
    """Standalone CrossModalAttention parity case (eval mode)."""
    name: str
    batch: int
    lq: int        # 0 => 2-D query (B, Dq)
    lk: int        # 0 => 2-D key/value (B, Dk)
    query_dim: int
    key_dim: int
    hidden: int
    heads: int
    seed: int
    mask_kind: str = "none"    # none | 1d | 2d
    mask_1d: Optional[List[float]] = None


def cma_inputs(case: CMACase):
    rng = np.random.default_rng(case.seed + 104729)
    qs = (case.batch, case.lq, case.query_dim) if case.lq else (case.batch, case.query_dim)
    ks = (case.batch, case.lk, case.key_dim) if case.lk else (case.batch, case.key_dim)
    query = rng.standard_normal(qs).astype(np.float32)
    key = rng.standard_normal(ks).astype(np.float32)
    value = rng.standard_normal(ks).astype(np.float32)
    mask = None
    if case.mask_kind == "1d":
        mask = np.asarray(case.mask_1d, dtype=np.float32)
    elif case.mask_kind == "2d":
        lk = max(case.lk, 1)
        mask = (rng.uniform(size=(case.batch, lk)) < 0.7).astype(np.float32)
        mask[0, :] = 0.0          # a fully masked sample -> NaN -> 0 path
        mask[1, :] = 1.0
    lq = max(case.lq, 1)
    gshape = (case.batch, lq, case.hidden) if case.lq else (case.batch, case.hidden)
    grad = rng.standard_normal(gshape).astype(np.float32)
    return query, key, value, mask, grad


_MASK_ROWS = [[1, 1, 1], [1, 0, 1], [0, 0, 1], [0, 0, 0], [1, 1, 0], [0, 1, 0], [0.5, 1, 1], [1, 1, 0.25]]

HYBRID_CASES: List[HybridCase] = [
    # Reference semantics (2-D inputs, L=1 attention), small, full gradients.
    HybridCase("tiny_l1", ["m0", "m1", "m2"], {"m0": 12, "m1": 20, "m2": 16},
               {"m0": 0, "m1": 0, "m2": 0}, batch=8, hidden=32, heads=4, classes=5,
               seed=11, mask=_MASK_ROWS),
    HybridCase("tiny_l1_deleted_pair", ["m0", "m1", "m2"], {"m0": 12, "m1": 20, "m2": 16},
               {"m0": 0, "m1": 0, "m2": 0}, batch=8, hidden=32, heads=4, classes=5,
               seed=12, mask=_MASK_ROWS, deleted=["m0_to_m1", "m2_to_m0"]),
    # tests/test_fusion.py:50-80 shape: video/imu, hidden 8, heads 1.
    HybridCase("known_answer_2mod", ["video", "imu"], {"video": 4, "imu": 4},
               {"video": 0, "imu": 0}, batch=3, hidden=8, heads=1, classes=3,
               seed=13, mask=[[1, 1], [1, 0], [0, 0]]),
    # BASELINE config 2 at reference semantics (L=1): B=256, M=3, D=H=128, h=4, C=5.
    HybridCase("c2_l1", ["m0", "m1", "m2"], {"m0": 128, "m1": 128, "m2": 128},
               {"m0": 0, "m1": 0, "m2": 0}, batch=256, hidden=128, heads=4, classes=5,
               seed=21, mask_keep=0.9, full=False),
    # Sequence mode (composed oracle): equal and mixed lengths.
    HybridCase("seq_equal", ["m0", "m1", "m2"], {"m0": 24, "m1": 32, "m2": 16},
               {"m0": 16, "m1": 16, "m2": 16}, batch=4, hidden=32, heads=4, classes=5,
               seed=31, mask=[[1, 1, 1], [1, 0, 1], [0, 0, 0], [0.5, 1, 0]]),
    HybridCase("seq_mixed", ["video", "imu", "hr"], {"video": 40, "imu": 24, "hr": 8},
               {"video": 30, "imu": 50, "hr": 20}, batch=3, hidden=64, heads=4, classes=11,
               seed=32, mask=[[1, 1, 1], [0, 1, 1], [1, 0, 0]]),
    HybridCase("seq_hd64", ["m0", "m1"], {"m0": 32, "m1": 48},
               {"m0": 40, "m1": 72}, batch=2, hidden=128, heads=2, classes=4,
               seed=33, mask=[[1, 1], [1, 0]]),
    # The benchmark's per-sample shape (C2 seq mode: L=128, D=H=128, 4 heads) at
    # B=3: every key length a multiple of 32 (the lean pooled-attention kernels)
    # and float4-able GEMM operands (the LDS-DMA GEMM).
    HybridCase("seq_c2_b3", ["m0", "m1", "m2"], {"m0": 128, "m1": 128, "m2": 128},
               {"m0": 128, "m1": 128, "m2": 128}, batch=3, hidden=128, heads=4, classes=5,
               seed=34, mask=[[1, 1, 1], [1, 0, 1], [0.5, 1, 1]], full=False, attn_slice=29),
    # Mixed multiples of 32 with head_dim 64 (lean kernels, HDP = 64).
    HybridCase("seq_lean_hd64", ["a", "b"], {"a": 64, "b": 32},
               {"a": 64, "b": 96}, batch=2, hidden=128, heads=2, classes=4,
               seed=35, mask=[[1, 1], [1, 0]], full=False, attn_slice=7),
    # The reference's heads ablation at hidden_dim 256 (num_heads in {1, 4, 8},
    # .github/workflows/parallel_run.yml:79-97): num_heads 1 / 2 = head_dim 256 / 128, on the
    # 2-D inputs src/train.py feeds HybridFusion (single-key attention) ...
    HybridCase("heads1_l1", ["imu_hand", "imu_chest", "heart_rate"],
               {"imu_hand": 128, "imu_chest": 128, "heart_rate": 128},
               {"imu_hand": 0, "imu_chest": 0, "heart_rate": 0}, batch=6, hidden=256, heads=1, classes=25,
               seed=36, mask=[[1, 1, 1], [1, 0, 1], [0, 0, 0], [0.5, 1, 0]], full=False),
    HybridCase("heads2_l1", ["imu_hand", "imu_chest", "heart_rate"],
               {"imu_hand": 128, "imu_chest": 128, "heart_rate": 128},
               {"imu_hand": 0, "imu_chest": 0, "heart_rate": 0}, batch=6, hidden=256, heads=2, classes=25,
               seed=37, mask=[[1, 1, 1], [0, 1, 1], [1, 1, 0]], full=False),
    # ... and on sequences (materialised scores + GEMMs, csrc/wide.hip)
    HybridCase("seq_wide_h2", ["a", "b"], {"a": 32, "b": 48},
               {"a": 24, "b": 40}, batch=2, hidden=256, heads=2, classes=4,
               seed=38, mask=[[1, 1], [1, 0]], full=False, attn_slice=5),
    HybridCase("seq_wide_h1", ["a", "b", "c"], {"a": 16, "b": 24, "c": 8},
               {"a": 12, "b": 20, "c": 9}, batch=2, hidden=256, heads=1, classes=5,
               seed=39, mask=[[1, 1, 1], [0, 1, 0.5]], full=False, attn_slice=3),
    # hidden 64 at L = 128: the projection GEMM's column-sum epilogue with N < 128 (threads
    # past the last column still reach its barrier)
    HybridCase("seq_h64_l128", ["a", "b"], {"a": 16, "b": 24},
               {"a": 128, "b": 128}, batch=2, hidden=64, heads=4, classes=3,
               seed=40, mask=[[1, 1], [1, 0.5]], full=False, attn_slice=11),
    # hidden 256, keys <= 128, odd batch: the two-samples-per-workgroup pair tail with its
    # padding slot
    HybridCase("seq_h256_odd", ["a", "b"], {"a": 32, "b": 24},
               {"a": 32, "b": 64}, batch=3, hidden=256, heads=4, classes=5,
               seed=46, mask=[[1, 1], [0, 1], [1, 0.5]], full=False, attn_slice=13),
]

CMA_CASES: List[CMACase] = [
    CMACase("cma_2d_mask1d", batch=4, lq=0, lk=0, query_dim=512, key_dim=64, hidden=256,
            heads=4, seed=41, mask_kind="1d", mask_1d=[1, 1, 0, 1]),
    CMACase("cma_3d_mask2d", batch=4, lq=30, lk=50, query_dim=24, key_dim=40, hidden=64,
            heads=4, seed=42, mask_kind="2d"),
    CMACase("cma_3d_nomask_hd8", batch=3, lq=17, lk=9, query_dim=16, key_dim=16, hidden=32,
            heads=4, seed=43),
    CMACase("cma_3d_long", batch=2, lq=160, lk=200, query_dim=32, key_dim=32, hidden=128,
            heads=4, seed=44, mask_kind="1d", mask_1d=[1, 0]),
    # head_dim 128 / 256 (materialised scores, csrc/wide.hip)
    CMACase("cma_3d_wide_hd128", batch=4, lq=20, lk=33, query_dim=24, key_dim=40, hidden=256,
            heads=2, seed=47, mask_kind="2d"),
    CMACase("cma_3d_wide_hd256", batch=2, lq=17, lk=12, query_dim=16, key_dim=16, hidden=256,
            heads=1, seed=48, mask_kind="1d", mask_1d=[1, 0]),
    CMACase("cma_2d_hd256", batch=4, lq=0, lk=0, query_dim=64, key_dim=32, hidden=256,
            heads=1, seed=49, mask_kind="1d", mask_1d=[1, 0, 1, 1]),
]


# PAMAP2 logits / ECE parity (tests/golden/gen_pamap2.py): the config/base.yaml
# model on the four PAMAP2 modalities (dataset.modalities, model.output_dim 128,
# model.hidden_dim 256, model.num_heads 4, dataset.num_classes 25, chunk 1024).
PAMAP2_MODALITIES = ["imu_hand", "imu_chest", "imu_ankle", "heart_rate"]
PAMAP2_OUT_DIM = 128
PAMAP2_HIDDEN = 256
PAMAP2_HEADS = 4
PAMAP2_CLASSES = 25
PAMAP2_CHUNK = 1024
PAMAP2_SEED = 81


def case_by_name(name: str):
    for c in HYBRID_CASES + CMA_CASES:
        if c.name == name:
            return c
    raise KeyError(name)


# ----------------------------------------------------------------------------
# TemporalAttention (src/attention.py:149-281) and PairwiseModalityAttention
# (src/attention.py:284-424): the rest of the attention module's import surface.
# ----------------------------------------------------------------------------
@dataclass
class TemporalCase:
    name: str
    batch: int
    seq: int
    feature_dim: int
    hidden: int
    heads: int
    seed: int
    mask_kind: str = "none"     # none | 1d (per time step, shared) | 2d (B, L)


TEMPORAL_CASES: List[TemporalCase] = [
    TemporalCase("temporal_nomask", batch=3, seq=40, feature_dim=32, hidden=64, heads=4, seed=61),
    TemporalCase("temporal_mask2d", batch=2, seq=10, feature_dim=24, hidden=32, heads=4, seed=62, mask_kind="2d"),
    TemporalCase("temporal_mask1d", batch=2, seq=6, feature_dim=16, hidden=32, heads=2, seed=63, mask_kind="1d"),
]


def temporal_inputs(case: TemporalCase):
    """(sequence, mask or None, upstream grad with the output's shape)."""
    rng = np.random.default_rng(case.seed + 15485863)
    seq = rng.standard_normal((case.batch, case.seq, case.feature_dim)).astype(np.float32)
    mask = None
    out_shape = (case.batch, case.seq, case.hidden)
    if case.mask_kind == "2d":
        mask = np.zeros((case.batch, case.seq), dtype=np.float32)
        for b in range(case.batch):
            mask[b, : max(1, case.seq - 3 - 2 * b)] = 1.0
        out_shape = (case.batch, 1, case.batch, case.seq, case.hidden)   # the reference's broadcast
    elif case.mask_kind == "1d":
        mask = np.asarray([1, 0, 1, 0, 1, 1][: case.seq], dtype=np.float32)
        out_shape = (1, 1, case.batch, case.seq, case.hidden)
    grad = rng.standard_normal(out_shape).astype(np.float32)
    return seq, mask, grad


@dataclass
class PairwiseCase:
    name: str
    names: List[str]
    dims: Dict[str, int]
    batch: int
    hidden: int
    heads: int
    seed: int
    mask: Optional[List[List[float]]] = None
    deleted: List[str] = field(default_factory=list)


PAIRWISE_CASES: List[PairwiseCase] = [
    PairwiseCase("pairwise_3mod", ["video", "audio", "imu"], {"video": 24, "audio": 16, "imu": 8},
                 batch=4, hidden=32, heads=4, seed=71,
                 mask=[[1, 0, 1], [1, 1, 1], [0, 1, 1], [1, 1, 0]], deleted=["video_to_audio"]),
]


def pairwise_state(case: PairwiseCase) -> "OrderedDict[str, np.ndarray]":
    """Keys of the reference PairwiseModalityAttention (projections + attention_layers)."""
    full = hybrid_state(case.names, case.dims, case.hidden, 2, case.seed, case.deleted)
    sd: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for k, v in full.items():
        if k.startswith("projections."):
            sd[k] = v
        elif k.startswith("attention_modules."):
            sd["attention_layers." + k[len("attention_modules."):]] = v
    return sd


def pairwise_inputs(case: PairwiseCase):
    rng = np.random.default_rng(case.seed + 32452843)
    feats = {m: rng.standard_normal((case.batch, case.dims[m])).astype(np.float32) for m in case.names}
    mask = np.asarray(case.mask, dtype=np.float32)
    grads = {m: rng.standard_normal((case.batch, case.hidden)).astype(np.float32) for m in case.names}
    return feats, mask, grads


# ----------------------------------------------------------------------------
# FrameEncoder attention pooling (src/encoders.py:210-336) and the LateFusion
# weighting (src/fusion.py:126-245): the §8(f) masked-softmax weighting ops.
# ----------------------------------------------------------------------------
@dataclass
class FramePoolCase:
    name: str
    batch: int
    frames: int
    frame_dim: int
    hidden: int
    out_dim: int
    seed: int
    masked: bool = False


FRAMEPOOL_CASES: List[FramePoolCase] = [
    FramePoolCase("framepool_nomask", batch=4, frames=30, frame_dim=48, hidden=32, out_dim=16, seed=81),
    FramePoolCase("framepool_mask", batch=4, frames=13, frame_dim=24, hidden=40, out_dim=8, seed=82, masked=True),
]


def framepool_state(case: FramePoolCase) -> "OrderedDict[str, np.ndarray]":
    rng = np.random.default_rng(case.seed)
    sd: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for key, (o, i) in (("frame_processor.0", (case.hidden, case.frame_dim)), ("attention", (1, case.hidden)),
                        ("projection.0", (case.hidden, case.hidden)), ("projection.3", (case.out_dim, case.hidden))):
        w, b = _linear(rng, o, i)
        if key == "attention":
            w = w * 4.0   # sharper frame weights than the default init
        sd[f"{key}.weight"], sd[f"{key}.bias"] = w, b
    return sd


def framepool_inputs(case: FramePoolCase):
    """(frames, mask or None, upstream grad of the pooled (B, hidden) and of the encoding (B, out))."""
    rng = np.random.default_rng(case.seed + 982451653)
    frames = rng.standard_normal((case.batch, case.frames, case.frame_dim)).astype(np.float32)
    mask = None
    if case.masked:
        mask = np.zeros((case.batch, case.frames), dtype=np.float32)
        lengths = [case.frames, 5, 0, 1][: case.batch]      # full, ragged, all masked, single frame
        for b, n in enumerate(lengths):
            mask[b, :n] = 1.0
    g_pool = rng.standard_normal((case.batch, case.hidden)).astype(np.float32)
    g_out = rng.standard_normal((case.batch, case.out_dim)).astype(np.float32)
    return frames, mask, g_pool, g_out


@dataclass
class LateCase:
    name: str
    names: List[str]
    dims: Dict[str, int]
    batch: int
    hidden: int
    classes: int
    seed: int
    mask: List[List[float]]


LATE_CASES: List[LateCase] = [
    LateCase("late_3mod", ["video", "audio", "imu"], {"video": 12, "audio": 8, "imu": 6}, batch=5, hidden=16,
             classes=4, seed=91, mask=[[1, 1, 1], [1, 0, 1], [0, 0, 0], [0, 0, 1], [0.5, 1, 0]]),
]


# EarlyFusion (src/fusion.py:17-123): BASELINE config C1's fusion (CPU plumbing, no HIP part)
EARLY_CASES: List[LateCase] = [
    LateCase("early_3mod", ["imu_hand", "imu_chest", "imu_ankle"], {"imu_hand": 17, "imu_chest": 17, "imu_ankle": 17},
             batch=6, hidden=32, classes=12, seed=93,
             mask=[[1, 1, 1], [1, 0, 1], [0, 0, 0], [0, 0, 1], [0.5, 1, 0], [1, 1, 0]]),
]


def early_state(case: LateCase) -> "OrderedDict[str, np.ndarray]":
    rng = np.random.default_rng(case.seed)
    sd: "OrderedDict[str, np.ndarray]" = OrderedDict()
    width = sum(case.dims[m] for m in case.names)
    for i, (o, k) in enumerate(((case.hidden, width), (case.hidden, case.hidden), (case.classes, case.hidden))):
        sd[f"fusion.{3 * i}.weight"], sd[f"fusion.{3 * i}.bias"] = _linear(rng, o, k)
    return sd


def late_state(case: LateCase) -> "OrderedDict[str, np.ndarray]":
    rng = np.random.default_rng(case.seed)
    sd: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for m in case.names:
        w, b = _linear(rng, case.hidden, case.dims[m])
        sd[f"classifiers.{m}.0.weight"], sd[f"classifiers.{m}.0.bias"] = w, b
        w, b = _linear(rng, case.classes, case.hidden)
        sd[f"classifiers.{m}.3.weight"], sd[f"classifiers.{m}.3.bias"] = w, b
    sd["weight_logits"] = rng.standard_normal(len(case.names)).astype(np.float32)
    return sd


def late_inputs(case: LateCase):
    rng = np.random.default_rng(case.seed + 49979687)
    feats = {m: rng.standard_normal((case.batch, case.dims[m])).astype(np.float32) for m in case.names}
    mask = np.asarray(case.mask, dtype=np.float32)
    grad = rng.standard_normal((case.batch, case.classes)).astype(np.float32)
    return feats, mask, grad


@dataclass
class SeqEncCase:
    """SequenceEncoder(encoder_type="lstm") (src/encoders.py:34-166)."""
    name: str
    batch: int
    steps: int
    input_dim: int
    hidden: int
    out_dim: int
    layers: int
    seed: int
    lengths: Optional[List[int]] = None


SEQENC_CASES: List[SeqEncCase] = [
    SeqEncCase("seqenc_1layer", batch=3, steps=40, input_dim=17, hidden=64, out_dim=16, layers=1, seed=91),
    # batch 6 -> instances of 4 + 2 rows; packed-sequence lengths incl. 1 and full
    SeqEncCase("seqenc_2layer_len", batch=6, steps=25, input_dim=9, hidden=128, out_dim=8, layers=2, seed=92,
               lengths=[25, 10, 1, 25, 7, 3]),
    # the C3 encoder shape (imu 17 features, hidden 256 -> 128)
    SeqEncCase("seqenc_h256", batch=2, steps=48, input_dim=17, hidden=256, out_dim=128, layers=1, seed=93),
]


def seqenc_state(case: SeqEncCase) -> "OrderedDict[str, np.ndarray]":
    rng = np.random.default_rng(case.seed)
    sd: "OrderedDict[str, np.ndarray]" = OrderedDict()
    H = case.hidden
    bound = 1.0 / np.sqrt(H)
    for k in range(case.layers):
        in_f = case.input_dim if k == 0 else H
        sd[f"rnn.weight_ih_l{k}"] = rng.uniform(-bound, bound, size=(4 * H, in_f)).astype(np.float32)
        sd[f"rnn.weight_hh_l{k}"] = rng.uniform(-bound, bound, size=(4 * H, H)).astype(np.float32)
        sd[f"rnn.bias_ih_l{k}"] = rng.uniform(-bound, bound, size=(4 * H,)).astype(np.float32)
        sd[f"rnn.bias_hh_l{k}"] = rng.uniform(-bound, bound, size=(4 * H,)).astype(np.float32)
    sd["projection.weight"], sd["projection.bias"] = _linear(rng, case.out_dim, H)
    return sd


def seqenc_inputs(case: SeqEncCase):
    """(sequence (B, T, D), lengths or None, upstream grad of the encoding (B, out))."""
    rng = np.random.default_rng(case.seed + 15485863)
    seq = rng.standard_normal((case.batch, case.steps, case.input_dim)).astype(np.float32)
    lengths = np.array(case.lengths, dtype=np.int64) if case.lengths is not None else None
    g_out = rng.standard_normal((case.batch, case.out_dim)).astype(np.float32)
    return seq, lengths, g_out
