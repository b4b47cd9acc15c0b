"""Upstream checkpoint import (stereoalgorithms_amd/utils/import_ckpt.py), on the CPU.

Synthetic checkpoints are laid out the way each upstream project saves them -- RAFT-Stereo's ``nn.DataParallel``
state dict (``module.`` prefix), Fast-ACVNet's ``{"model": ...}`` container, the CREStereo port's plain state dict,
HITNet under this framework's names -- from a seeded oracle, converted, and must give back that seeded model bit for
bit: the same tensors in the safetensors file, the same oracle output.  Parity with the real released checkpoints is
unpinned (none ships with the reference; no network)."""
import pytest
import torch
from safetensors.torch import load_file

from stereoalgorithms_amd.utils import import_ckpt as IC
from stereoalgorithms_amd.utils.weights import read_metadata, save_model

CASES = [
    ("raftstereo-sceneflow", "dp"),
    ("raftstereo-realtime", "dp"),
    ("fastacvnet-plus", "model"),
    ("crestereo-iter5", "plain"),
    ("hitnet-d400", "plain"),
    ("hitnet-xl", "plain"),
]


def _upstream_file(model, layout, path):
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    if layout == "dp":
        obj = {"module." + k: v for k, v in sd.items()}
    elif layout == "model":
        obj = {"model": {"module." + k: v for k, v in sd.items()}, "epoch": torch.tensor(63)}
    else:
        obj = sd
    torch.save(obj, path)
    return path


@pytest.mark.parametrize("preset,layout", CASES)
def test_import_roundtrip(preset, layout, tmp_path):
    seeded = IC.build_oracle(preset, seed=7)
    src = _upstream_file(seeded, layout, tmp_path / "upstream.pth")
    got_preset, out = IC.convert(src, tmp_path / "imported.safetensors")
    assert got_preset == preset
    assert read_metadata(out)["model"] == preset
    ref = load_file(str(save_model(seeded, tmp_path / "ref.safetensors", preset)))
    imp = load_file(str(out))
    assert set(imp) == set(ref)
    for k in ref:
        assert torch.equal(imp[k], ref[k]), k


def test_import_oracle_output_bitwise(tmp_path):
    """The imported RAFT-Stereo realtime weights drive the oracle to the seeded model's exact disparity."""
    seeded = IC.build_oracle("raftstereo-realtime", seed=3)
    src = _upstream_file(seeded, "dp", tmp_path / "rt.pth")
    _, model = IC.load_checkpoint(src)
    g = torch.Generator().manual_seed(0)
    left = torch.randint(0, 255, (1, 3, 128, 256), generator=g).float()
    right = torch.randint(0, 255, (1, 3, 128, 256), generator=g).float()
    with torch.no_grad():
        a = seeded(left, right, iters=2)[1]
        b = model(left, right, iters=2)[1]
    assert torch.equal(a, b)


def test_import_preset_override_and_errors(tmp_path):
    seeded = IC.build_oracle("crestereo-iter5", seed=1)
    src = _upstream_file(seeded, "plain", tmp_path / "cre.pth")
    p, out = IC.convert(src, tmp_path / "cre10.safetensors", preset="crestereo-iter10")
    assert p == "crestereo-iter10" and read_metadata(out)["model"] == "crestereo-iter10"
    # a realtime checkpoint forced onto the sceneflow architecture: the mismatch is reported, nothing written
    rt = _upstream_file(IC.build_oracle("raftstereo-realtime", 0), "dp", tmp_path / "rt.pth")
    with pytest.raises(KeyError, match="does not match raftstereo-sceneflow"):
        IC.convert(rt, tmp_path / "bad.safetensors", preset="raftstereo-sceneflow")
    assert not (tmp_path / "bad.safetensors").exists()
    # a wrong-shaped tensor is named
    sd = {k: v.clone() for k, v in seeded.state_dict().items()}
    sd["conv_offset_8.weight"] = torch.zeros(18, 128, 3, 3)
    torch.save(sd, tmp_path / "shape.pth")
    with pytest.raises(KeyError, match="conv_offset_8.weight"):
        IC.convert(tmp_path / "shape.pth", tmp_path / "x.safetensors")
    torch.save({"unrelated.weight": torch.zeros(3)}, tmp_path / "junk.pth")
    with pytest.raises(ValueError, match="cannot infer"):
        IC.convert(tmp_path / "junk.pth", tmp_path / "y.safetensors")


def test_import_cli(tmp_path):
    seeded = IC.build_oracle("fastacvnet-plus", seed=2)
    src = _upstream_file(seeded, "model", tmp_path / "facv.ckpt")
    assert IC.main([str(src), str(tmp_path / "facv.safetensors")]) == 0
    assert read_metadata(tmp_path / "facv.safetensors")["model"] == "fastacvnet-plus"
