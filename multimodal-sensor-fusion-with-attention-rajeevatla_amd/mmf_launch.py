"""Run the reference's own scripts on the MI355X fusion path, unchanged.

    python <pkg>/mmf_launch.py [--mmf-encoders] src/train.py [hydra overrides ...]
    python <pkg>/mmf_launch.py [--mmf-encoders] src/eval.py  [args ...]
    python <pkg>/mmf_launch.py [--mmf-encoders] -m pytest tests/test_fusion.py ...

The reference's scripts import the hot path by bare module name --
``from fusion import HybridFusion, build_fusion_model`` (src/train.py:25) and
``from attention import CrossModalAttention`` (src/fusion.py:14) -- and Python puts a
script's own directory (``src/``) at ``sys.path[0]``, ahead of PYTHONPATH.  So a
PYTHONPATH entry cannot swap those two modules in, and putting this package's directory
first would also shadow ``src/encoders.py`` (``from encoders import build_encoder``,
src/train.py:26), which this package's ``encoders.py`` does not replace.

This launcher does exactly what a ``python src/train.py`` start does (the script's directory
first on ``sys.path``, ``sys.argv[0]`` = the script, ``__name__ == "__main__"`` via
``runpy``), with two differences:

* ``sys.modules["fusion"]`` / ``sys.modules["attention"]`` are this package's
  ``fusion.py`` / ``attention.py`` (loaded by file, attention first since fusion imports
  it), so every ``import fusion`` / ``from attention import ...`` in the reference --
  train.py, eval.py (through ``from train import MultimodalFusionModule``), the reference's
  tests -- gets the HIP-backed HybridFusion / CrossModalAttention (and EarlyFusion,
  LateFusion, build_fusion_model with the reference's signatures);
* this package's directory is appended LAST to ``sys.path``: its private modules
  (``mmf_native``, ``mmf_ops``, the ``mmf_torch`` extension) resolve, while every module the
  reference has -- ``encoders``, ``data``, ``uncertainty``, ``train`` -- keeps coming from
  ``src/``.

``--mmf-encoders`` (opt-in): after importing the reference's ``encoders``
module, route its ``FrameEncoder.attention_pool`` (src/encoders.py:313-336) and the
'lstm' branch of ``SequenceEncoder.forward`` (src/encoders.py:135-166) through this
package's HIP kernels (csrc/softmax_pool.hip, csrc/lstm.hip).  The modules, their
parameters and state-dict keys stay the reference's own; other encoder types and
pooling strategies run the reference's code.

No reference source is modified.  ``install()`` is the same swap for a caller that
starts its own interpreter (a notebook, a test runner's conftest).
"""

from __future__ import annotations

import importlib.util
import os
import runpy
import sys
from typing import List, Optional

PKG = os.path.dirname(os.path.abspath(__file__))
SWAPPED = ("attention", "fusion")   # (load order: the package's fusion imports attention)


def _load(name: str, filename: str):
    spec = importlib.util.spec_from_file_location(name, os.path.join(PKG, filename))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        sys.modules.pop(name, None)
        raise
    return mod


def install(encoders: bool = False) -> None:
    """Make ``fusion`` / ``attention`` this package's modules for every later import, with this
    package's directory at the END of sys.path (the reference's modules keep resolving first).
    encoders=True: also patch the reference's ``encoders`` module (importable from sys.path)."""
    while PKG in sys.path:
        sys.path.remove(PKG)
    sys.path.append(PKG)
    for name in SWAPPED:
        have = sys.modules.get(name)
        if have is not None and os.path.dirname(os.path.abspath(getattr(have, "__file__", "") or "")) != PKG:
            raise RuntimeError(f"mmf_launch.install: module '{name}' was already imported from {have.__file__}; "
                               "install() must run before the reference imports it")
        if have is None:
            _load(name, name + ".py")
    if encoders:
        import encoders as ref_encoders   # the reference's src/encoders.py
        patch_encoders(ref_encoders)


def patch_encoders(ref_encoders) -> None:
    """Route the reference's FrameEncoder.attention_pool and SequenceEncoder's 'lstm' forward through
    this package's HIP kernels (same arguments, same results as the package's own encoders, which are
    pinned to the reference's outputs: tests/test_gpu_softmax_pool.py, tests/test_gpu_lstm.py)."""
    mmf_enc = sys.modules.get("mmf_encoders") or _load("mmf_encoders", "encoders.py")
    if getattr(ref_encoders, "_mmf_patched", False):
        return
    fe, se = ref_encoders.FrameEncoder, ref_encoders.SequenceEncoder

    def attention_pool(self, frames, mask=None):
        if self.attention is None:
            raise RuntimeError("Attention layer not initialized.")
        return mmf_enc.attention_pool(frames, self.attention, mask)

    ref_seq_forward = se.forward

    def forward(self, sequence, lengths=None):
        if self.encoder_type != "lstm":
            return ref_seq_forward(self, sequence, lengths)
        if sequence.dim() != 3:
            raise ValueError(f"Expected 3D input sequence, got shape {sequence.shape}")
        if self.rnn is None:
            raise RuntimeError("RNN module not initialized.")
        out = mmf_enc.lstm_layers([self.rnn], [sequence])[0]   # (the module's own nn.LSTM parameters)
        return self.projection(self.dropout_layer(mmf_enc._final_state(out, lengths)))

    fe.attention_pool = attention_pool
    se.forward = forward
    ref_encoders._mmf_patched = True


def main(argv: Optional[List[str]] = None) -> int:
    args = list(sys.argv[1:] if argv is None else argv)
    encoders = False
    while args and args[0].startswith("--mmf-"):
        flag = args.pop(0)
        if flag == "--mmf-encoders":
            encoders = True
        else:
            raise SystemExit(f"mmf_launch: unknown option {flag}")
    if not args:
        raise SystemExit(__doc__)
    if args[0] == "-m":
        if len(args) < 2:
            raise SystemExit("mmf_launch: -m needs a module name")
        # `python -m mod`: the current directory first on sys.path
        sys.path[0] = os.getcwd()
        sys.argv = [args[1]] + args[2:]
        install(encoders)
        runpy.run_module(args[1], run_name="__main__", alter_sys=True)
        return 0
    script = os.path.abspath(args[0])
    if not os.path.isfile(script):
        raise SystemExit(f"mmf_launch: no such script: {args[0]}")
    # `python script`: the script's directory first on sys.path (this launcher's own directory,
    # which Python put there, goes to the end in install())
    sys.path[0] = os.path.dirname(script)
    sys.argv = [args[0]] + args[1:]
    install(encoders)
    runpy.run_path(args[0], run_name="__main__")   # (sets sys.argv[0] to the path as given)
    return 0


if __name__ == "__main__":
    sys.exit(main())
