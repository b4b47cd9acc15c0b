"""The native engine built from an IMPORTED upstream-layout checkpoint (utils/import_ckpt.py) runs exactly the seeded
model it was made from: bitwise-equal disparity against the engine built from the seeded model's own save."""
import numpy as np
import pytest
import torch

from stereoalgorithms_amd import _native as N
from stereoalgorithms_amd.utils import import_ckpt as IC
from stereoalgorithms_amd.utils.synthetic import batch_pairs
from stereoalgorithms_amd.utils.weights import save_model

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not (torch.cuda.is_available() and N.available()), reason="needs GPU + native lib")]


@pytest.mark.parametrize("preset", ["raftstereo-realtime", "crestereo-iter2"])
def test_engine_from_imported_checkpoint(preset, tmp_path):
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    seeded = IC.build_oracle(preset, seed=5)
    prefix = "module." if preset.startswith("raft") else ""
    torch.save({prefix + k: v for k, v in seeded.state_dict().items()}, tmp_path / "up.pth")
    _, imported = IC.convert(tmp_path / "up.pth", tmp_path / "imp.safetensors", preset=preset)  # iterations: not in the weights
    ref = save_model(seeded, tmp_path / "ref.safetensors", preset)
    l, r = batch_pairs(1, 480, 640, seed=11)
    outs = []
    for w in (ref, imported):
        e = NativeStereoEngine("", str(w), 480, 640, batch=1, device=0)
        d, _, _ = e.run_host(l, r, cloud=False)
        outs.append(d.copy())
        e.close()
    assert np.isfinite(outs[0]).all() and np.array_equal(outs[0], outs[1])
