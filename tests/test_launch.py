"""The reference-side binding (VERDICT r05 missing #1): mmf_launch.py runs a
script of the reference's layout unchanged, with `fusion` / `attention` resolving to this package
and every other module the reference has (`encoders`, `data`, ...) to its own `src/`.

A stub `src/` tree stands in for the reference (PyTorch Lightning and Hydra, which the real
src/train.py imports, are not installed here): its train.py makes the reference's three imports
(/root/reference/src/train.py:24-26), builds the fusion model the way src/train.py:175-182 does and
runs the isinstance check of src/train.py:247; its fusion.py / attention.py are decoys that fail
the run if imported.  CPU only (module construction, no kernels)."""
from __future__ import annotations

import json
import os
import subprocess
import sys
import textwrap
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "multimodal-sensor-fusion-with-attention-rajeevatla_amd"
LAUNCH = PKG / "mmf_launch.py"

TRAIN = '''
import json, os, sys
from data import create_dataloaders
from fusion import HybridFusion, build_fusion_model
from encoders import build_encoder
import attention, data, encoders, fusion

model_fusion = build_fusion_model(
    fusion_type="hybrid",
    modality_dims={"imu": 16, "video": 16},
    num_classes=5,
    hidden_dim=32,
    num_heads=4,
    dropout=0.1,
)
enc = build_encoder(modality="imu", input_dim=8, output_dim=16, encoder_config={"type": "sequence"})
out = {
    "name": __name__,
    "argv": sys.argv,
    "path0": sys.path[0],
    "fusion": fusion.__file__,
    "attention": attention.__file__,
    "encoders": encoders.__file__,
    "data": data.__file__,
    "create_dataloaders": create_dataloaders(),
    "encoder": type(enc).__module__ + "." + type(enc).__name__,
    "isinstance": isinstance(model_fusion, HybridFusion),
    "cma_module": type(model_fusion.attention_modules["imu_to_video"]).__module__,
    "cma_is_attention_module": type(model_fusion.attention_modules["imu_to_video"]) is attention.CrossModalAttention,
    "state_keys": sorted(model_fusion.state_dict())[:3],
    "patched": bool(getattr(encoders, "_mmf_patched", False)),
}
with open(sys.argv[1], "w") as f:
    json.dump(out, f)
'''

DECOY = '''
raise ImportError("the reference's {name}.py was imported: the package's module must win")
'''

ENCODERS = '''
import torch.nn as nn

class FrameEncoder(nn.Module):
    def attention_pool(self, frames, mask=None):
        return "reference attention_pool"

class SequenceEncoder(nn.Module):
    def __init__(self, input_dim, output_dim, encoder_type="lstm"):
        super().__init__()
        self.encoder_type = encoder_type
    def forward(self, sequence, lengths=None):
        return "reference forward"

def build_encoder(modality, input_dim, output_dim, encoder_config=None):
    return SequenceEncoder(input_dim, output_dim)
'''

DATA = '''
def create_dataloaders(*args, **kwargs):
    return "reference data"
'''

TEST_FUSION = '''
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).parent.parent / "src"))
from fusion import HybridFusion, build_fusion_model
from attention import CrossModalAttention

def test_resolves_to_package():
    import fusion
    assert "rajeevatla_amd" in fusion.__file__
    m = build_fusion_model("hybrid", {"a": 8, "b": 8}, num_classes=3, hidden_dim=16, num_heads=2, dropout=0.0)
    assert isinstance(m, HybridFusion)
    assert isinstance(m.attention_modules["a_to_b"], CrossModalAttention)
'''


def _stub_tree(tmp_path: Path) -> Path:
    src = tmp_path / "src"
    src.mkdir()
    (src / "train.py").write_text(TRAIN)
    (src / "fusion.py").write_text(DECOY.format(name="fusion"))
    (src / "attention.py").write_text(DECOY.format(name="attention"))
    (src / "encoders.py").write_text(ENCODERS)
    (src / "data.py").write_text(DATA)
    tests = tmp_path / "tests"
    tests.mkdir()
    (tests / "test_ref_fusion.py").write_text(TEST_FUSION)
    return src


def _run(args, cwd, extra_env=None):
    env = dict(os.environ)
    env.pop("PYTHONPATH", None)
    env.update(extra_env or {})
    return subprocess.run([sys.executable, str(LAUNCH)] + args, cwd=cwd, env=env, capture_output=True, text=True,
                          timeout=300)


def test_launcher_swaps_fusion_and_attention_only(tmp_path):
    src = _stub_tree(tmp_path)
    out = tmp_path / "out.json"
    r = _run(["src/train.py", str(out)], cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    o = json.loads(out.read_text())
    assert o["name"] == "__main__"
    assert o["argv"] == ["src/train.py", str(out)]
    assert o["path0"] == str(src)                                   # as `python src/train.py` sets it
    assert Path(o["fusion"]).resolve() == PKG / "fusion.py"          # the package wins for the hot path
    assert Path(o["attention"]).resolve() == PKG / "attention.py"
    assert Path(o["encoders"]).resolve() == src / "encoders.py"      # ... and only there
    assert Path(o["data"]).resolve() == src / "data.py"
    assert o["create_dataloaders"] == "reference data"
    assert o["encoder"] == "encoders.SequenceEncoder"
    assert o["isinstance"] is True                                  # src/train.py:247
    assert o["cma_module"] == "attention" and o["cma_is_attention_module"] is True
    assert o["state_keys"][0].startswith("attention_modules.")       # the reference's state-dict keys
    assert o["patched"] is False


def test_launcher_patches_reference_encoders_on_request(tmp_path):
    _stub_tree(tmp_path)
    out = tmp_path / "out.json"
    r = _run(["--mmf-encoders", "src/train.py", str(out)], cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    o = json.loads(out.read_text())
    assert o["patched"] is True
    assert Path(o["encoders"]).resolve() == tmp_path / "src" / "encoders.py"   # the reference's module, patched
    assert Path(o["fusion"]).resolve() == PKG / "fusion.py"


def test_plain_pythonpath_does_not_swap(tmp_path):
    """Why the launcher exists: with the package on PYTHONPATH, `python src/train.py` still imports
    src/fusion.py (the script's directory precedes PYTHONPATH) -- here the decoy raises."""
    _stub_tree(tmp_path)
    env = dict(os.environ, PYTHONPATH=str(PKG))
    r = subprocess.run([sys.executable, "src/train.py", str(tmp_path / "o.json")], cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "the package's module must win" in r.stderr


def test_launcher_runs_reference_tests_under_pytest(tmp_path):
    """`-m pytest`: the reference's tests insert src/ at sys.path[0] and import fusion / attention
    (tests/test_fusion.py:14-16); they get the package's modules."""
    _stub_tree(tmp_path)
    r = _run(["-m", "pytest", "-q", "-p", "no:cacheprovider", "tests/test_ref_fusion.py"], cwd=tmp_path)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "1 passed" in r.stdout


def test_install_refuses_after_reference_import(tmp_path):
    """install() after the reference's fusion was imported would leave two HybridFusion classes
    (the isinstance check of src/train.py:247 against the wrong one): refused."""
    src = _stub_tree(tmp_path)
    (src / "fusion.py").write_text("X = 1\n")
    code = textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {str(src)!r})
        import fusion
        sys.path.insert(0, {str(PKG)!r})
        import mmf_launch
        try:
            mmf_launch.install()
        except RuntimeError as e:
            print("refused:", e)
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert "refused:" in r.stdout and "already imported" in r.stdout, (r.stdout, r.stderr)
