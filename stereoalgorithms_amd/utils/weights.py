"""Weight files: our on-disk format is safetensors (header + named tensors, no code execution on
load), with ``__metadata__["model"]`` naming the preset.  This replaces the reference's ONNX file +
serialized TensorRT engine cache (common/ONNX2TRT.cpp:121-127, RAFTStereo/src/TRTRAFTStereo.cpp:25-46).
"""
from __future__ import annotations

import json
from pathlib import Path

import torch
from safetensors import safe_open
from safetensors.torch import save_file

FORMAT = "stereoalgorithms_amd/1"


def save_model(model: torch.nn.Module, path: str | Path, preset: str, extra: dict | None = None) -> Path:
    # clone: aliased parameters (e.g. norm3 == downsample.1) must be stored as separate tensors
    sd = {k: v.detach().to(torch.float32).cpu().clone().contiguous() for k, v in model.state_dict().items()
          if v.dtype.is_floating_point}
    meta = {"model": preset, "format": FORMAT}
    if extra:
        meta.update({k: json.dumps(v) if not isinstance(v, str) else v for k, v in extra.items()})
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    save_file(sd, str(path), metadata=meta)
    return path


def read_metadata(path: str | Path) -> dict:
    with safe_open(str(path), framework="pt") as f:
        return dict(f.metadata() or {})


def load_into(model: torch.nn.Module, path: str | Path, strict: bool = True):
    from safetensors.torch import load_file
    sd = load_file(str(path))
    missing, unexpected = model.load_state_dict(sd, strict=False)
    missing = [m for m in missing if not m.endswith("num_batches_tracked")]
    if strict and (missing or unexpected):
        raise KeyError(f"missing={missing} unexpected={unexpected}")
    return model
