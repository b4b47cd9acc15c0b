"""Reader for engine activation taps (StereoEngine::tap, csrc/runtime/engine.cpp): run an engine with
SA_NO_GRAPH=1 and SA_TAP_DIR=<dir>; each tapped tensor lands in <dir>/<name>.sat."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import torch

_DT = {0: np.float16, 1: np.float32, 2: np.uint8}


def load_tap(path: str | Path) -> torch.Tensor:
    """-> fp32 tensor [n, d, h, w, c] (padding channels of the strided layout dropped)."""
    raw = Path(path).read_bytes()
    n, d, h, w, c, stride, dt = np.frombuffer(raw[:28], dtype=np.int32).tolist()
    a = np.frombuffer(raw[28:], dtype=_DT[dt]).reshape(n, d, h, w, stride)[..., :c]
    return torch.from_numpy(a.astype(np.float32))


def load_taps(directory: str | Path) -> dict[str, torch.Tensor]:
    return {p.stem: load_tap(p) for p in sorted(Path(directory).glob("*.sat"))}
