"""Import upstream PyTorch checkpoints of the four networks into this framework's safetensors weight format.

The reference's ``Initialize`` takes the user's downloaded model file (``RAFTStereo/src/TRTRAFTStereo.cpp:25-46``;
download links ``README_en.md:105,135,164,215,267``) -- ONNX exports of the upstream PyTorch checkpoints.  ONNX is not
readable here (no ``onnx`` package, and the graph would have to be re-derived), so the importer reads the upstream
*training checkpoints* the ONNX files were exported from, maps them onto the oracle modules (whose parameter names
mirror upstream: ``update_block.gru08``, ``context_zqr_convs``, ``self_att_fn.layers.N.q_proj`` ...), checks every
name and shape, and writes the ``.safetensors`` file that ``NativeStereoEngine`` / the C ABI ``Initialize`` load.

Layouts handled (``torch.load(weights_only=True)`` only: nothing in the file is executed):

* RAFT-Stereo (princeton-vl/RAFT-Stereo ``raftstereo-*.pth``): a state dict saved from ``nn.DataParallel``, every key
  prefixed ``module.``.  The sceneflow / realtime preset is inferred from the shared-backbone ``conv2`` head.
* Fast-ACVNet+ (gangweiX/Fast-ACVNet ``*.ckpt``): ``{"model": state_dict, ...}`` with ``module.`` keys.
* CREStereo (the PyTorch port of the MegEngine release, ``crestereo_*.pth``): a plain state dict.  The iteration
  count is not part of the weights (``--preset crestereo-iter2/5/10``; default iter5, the reference demo's,
  ``CREStereo/test/main.cpp:31``).
* HITNet: the upstream release is TensorFlow; state dicts under this framework's names (``feature.*``, ``init.N``,
  ``prop.N``, ``refine.N``) are accepted, d400 vs XL inferred from the number of levels.
* Any of the above already in ``.safetensors`` form (upstream names, optional ``module.`` prefix).

Parity with the real released checkpoints is unpinned: none ships with the reference and there is no network here.
``tests/test_import_ckpt_cpu.py`` converts synthetic state dicts laid out under the upstream names.

CLI::

    python -m stereoalgorithms_amd.utils.import_ckpt raftstereo-sceneflow.pth raft_sf.safetensors
    python -m stereoalgorithms_amd.utils.import_ckpt crestereo_eth3d.pth cre10.safetensors --preset crestereo-iter10
"""
from __future__ import annotations

import argparse
from pathlib import Path

import torch

FAMILY_OF = {
    "raftstereo-sceneflow": "raft", "raftstereo-realtime": "raft",
    "crestereo-iter2": "crestereo", "crestereo-iter5": "crestereo", "crestereo-iter10": "crestereo",
    "hitnet-d400": "hitnet", "hitnet-xl": "hitnet",
    "fastacvnet-plus": "fastacvnet",
}


def read_state_dict(path: str | Path) -> dict[str, torch.Tensor]:
    """Tensors of an upstream checkpoint, unwrapped (``model`` / ``state_dict`` containers) and with the
    ``nn.DataParallel`` ``module.`` prefix removed.  ``.safetensors`` files are read with safetensors, everything else
    with ``torch.load(weights_only=True)``."""
    path = Path(path)
    if path.suffix == ".safetensors":
        from safetensors.torch import load_file
        obj = load_file(str(path))
    else:
        obj = torch.load(str(path), map_location="cpu", weights_only=True)
    for key in ("model", "state_dict", "model_state_dict", "net"):
        if isinstance(obj, dict) and key in obj and isinstance(obj[key], dict):
            obj = obj[key]
            break
    if not isinstance(obj, dict):
        raise ValueError(f"{path}: not a state dict (got {type(obj).__name__})")
    sd = {}
    for k, v in obj.items():
        if not isinstance(v, torch.Tensor):
            continue
        while k.startswith("module."):
            k = k[len("module."):]
        sd[k] = v
    if not sd:
        raise ValueError(f"{path}: no tensors found")
    return sd


def infer_preset(sd: dict[str, torch.Tensor]) -> str:
    """Model preset from the key set (CREStereo's iteration count is not in the weights: iter5)."""
    keys = set(sd)
    if any(k.startswith("update_block.gru08.") for k in keys) or any(k.startswith("context_zqr_convs.") for k in keys):
        # realtime: --shared_backbone, the feature map is conv2 on the context network's stem (no fnet)
        return "raftstereo-realtime" if any(k.startswith("conv2.") for k in keys) else "raftstereo-sceneflow"
    if any(k.startswith("self_att_fn.") for k in keys) or any(k.startswith("conv_offset_16.") for k in keys):
        return "crestereo-iter5"
    if any(k.startswith("hourglass_att.") for k in keys) or any(k.startswith("corr_feature_att_4.") for k in keys):
        return "fastacvnet-plus"
    if any(k.startswith("init.") for k in keys) and any(k.startswith("prop.") for k in keys):
        levels = len({k.split(".")[1] for k in keys if k.startswith("init.")})
        from stereoalgorithms_amd.models import hitnet as HN
        for p in ("hitnet-d400", "hitnet-xl"):
            if len({k.split(".")[1] for k in HN.build(p).state_dict() if k.startswith("init.")}) == levels:
                if _shapes_match(HN.build(p).state_dict(), sd):
                    return p
        raise ValueError("HITNet-like state dict matches neither hitnet-d400 nor hitnet-xl")
    raise ValueError("cannot infer the model from the checkpoint's keys; pass --preset")


def _shapes_match(ref: dict, sd: dict) -> bool:
    return all(k in sd and tuple(sd[k].shape) == tuple(v.shape) for k, v in ref.items()
               if v.dtype.is_floating_point)


def build_oracle(preset: str, seed: int = 0):
    fam = FAMILY_OF[preset]
    if fam == "raft":
        from stereoalgorithms_amd.models import raft_stereo as M
    elif fam == "crestereo":
        from stereoalgorithms_amd.models import crestereo as M
    elif fam == "hitnet":
        from stereoalgorithms_amd.models import hitnet as M
    else:
        from stereoalgorithms_amd.models import fast_acvnet as M
    return M.build(preset, seed)


def load_checkpoint(path: str | Path, preset: str | None = None):
    """-> (preset, oracle module with the checkpoint's weights).  Raises with the list of missing / unexpected /
    mis-shaped tensors when the checkpoint does not fit the preset's architecture."""
    sd = read_state_dict(path)
    preset = preset or infer_preset(sd)
    if preset not in FAMILY_OF:
        raise ValueError(f"unknown preset {preset!r}; one of {sorted(FAMILY_OF)}")
    model = build_oracle(preset)
    ref = model.state_dict()
    missing = [k for k, v in ref.items() if k not in sd and not k.endswith("num_batches_tracked")]
    unexpected = [k for k in sd if k not in ref]
    shapes = [f"{k}: checkpoint {tuple(sd[k].shape)} vs model {tuple(v.shape)}" for k, v in ref.items()
              if k in sd and tuple(sd[k].shape) != tuple(v.shape)]
    if missing or unexpected or shapes:
        lines = [f"checkpoint {path} does not match {preset}:"]
        for title, items in (("missing", missing), ("unexpected", unexpected), ("shape", shapes)):
            if items:
                lines.append(f"  {len(items)} {title}: " + ", ".join(items[:12]) + (" ..." if len(items) > 12 else ""))
        raise KeyError("\n".join(lines))
    model.load_state_dict({k: sd[k].to(ref[k].dtype) for k in ref if k in sd}, strict=False)
    return preset, model


def convert(src: str | Path, dst: str | Path, preset: str | None = None) -> tuple[str, Path]:
    """Upstream checkpoint -> this framework's ``.safetensors`` (metadata names the preset)."""
    from stereoalgorithms_amd.utils.weights import save_model
    preset, model = load_checkpoint(src, preset)
    return preset, save_model(model, dst, preset, extra={"source": Path(src).name})


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("src", help="upstream checkpoint (.pth / .ckpt / .pt / .safetensors)")
    ap.add_argument("dst", help="output .safetensors")
    ap.add_argument("--preset", default=None, help=f"model preset (default: inferred); one of {sorted(FAMILY_OF)}")
    a = ap.parse_args(argv)
    preset, out = convert(a.src, a.dst, a.preset)
    print(f"{a.src} -> {out} ({preset})")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
