"""Checkpoints in the reference's safetensors layout, so weights round-trip with p1atdev/vision-pt.

The reference saves `model.state_dict()` of JiTModel (src/saving/safetensors.py:14-35) -- keys
`denoiser.<JiT param>` and `class_encoder.embedding.weight` -- and loads them back by stripping those
prefixes (JiTModel._load_checkpoint, src/models/jit/pipeline.py:51-87). The engine keeps every
parameter under the JiT/ClassEncoder names and shapes in one flat bf16 buffer; these helpers map the
prefixes and copy through that buffer (no per-parameter allocations on load).
"""

from __future__ import annotations

import torch
from safetensors.torch import load_file, save_file

from .engine import JiTEngine

CLASS_KEY = "class_encoder.embedding.weight"


def to_reference_state_dict(engine: JiTEngine) -> dict[str, torch.Tensor]:
    """JiTModel.state_dict() equivalent (views of the engine's flat buffer, on the device)."""
    out = {}
    for name, t in engine.state_dict().items():
        out[name if name == CLASS_KEY else "denoiser." + name] = t
    return out


def from_reference_state_dict(engine: JiTEngine, sd: dict[str, torch.Tensor], strict: bool = True) -> None:
    """Loads a JiTModel state dict (pipeline.py:51-87 key handling) into the engine."""
    mine = {}
    for k, v in sd.items():
        if k.startswith("denoiser."):
            mine[k[len("denoiser."):]] = v
        elif k == CLASS_KEY:
            mine[k] = v
        elif strict:
            raise KeyError(f"unexpected checkpoint key {k!r}")
    if CLASS_KEY not in engine.p:
        mine.pop(CLASS_KEY, None)
    engine.load_state_dict(mine, strict=strict)


def save_checkpoint(engine: JiTEngine, path: str, metadata: dict[str, str] | None = None,
                    dtype: torch.dtype | None = None) -> str:
    """safetensors file with the reference's keys (save_file(state_dict, path, metadata))."""
    sd = {k: (v if dtype is None else v.to(dtype)).detach().cpu().contiguous()
          for k, v in to_reference_state_dict(engine).items()}
    save_file(sd, path, metadata)
    return path


def load_checkpoint(engine: JiTEngine, path: str, strict: bool = True) -> None:
    from_reference_state_dict(engine, load_file(path), strict=strict)
