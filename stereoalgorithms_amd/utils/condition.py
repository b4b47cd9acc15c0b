"""Weight conditioning by a short supervised run on synthetic stereo pairs (option b).

A random-init Fast-ACVNet+ is numerically chaotic: its top-24 / top-2 selections sit on near-equal logits, so the
fp32 oracle re-run with fp16 activation storage -- or merely with fp64 instead of fp32 accumulation under the same
fp16 storage -- agrees with itself within 1 px on only ~45-55 % of the pixels (measured at 240x320; no per-pixel
parity test of ANY fp16 engine can pass against it).  A few hundred Adam steps on pairs with known disparity
(``utils.synthetic.stereo_pair``) give the cost volumes real margins: after 300 steps (128x256, lr 1e-3, or the default
96x192, lr 5e-4) the same fp16-storage oracle agrees with the fp32 oracle on 99.94-99.98 % of the pixels (mean |diff|
0.004-0.005 px), and the prediction tracks the ground truth (mean |err| 2-3.3 px at 240x320).  The network keeps its
architecture; its activations must stay inside the fp16 range (lr 2e-3 overflowed them), which
``fp16_storage_agreement`` checks before any engine is compared against the oracle.

The reference ships no checkpoint (/root/reference/README_en.md:267-272 points to a download), so trained upstream
weights stay unpinned; this is the stand-in for "a trained network" that per-pixel parity needs.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def imagenet_input(bgr_u8: np.ndarray | torch.Tensor, device=None) -> torch.Tensor:
    """u8 BGR [B,H,W,3] -> ImageNet-normalised RGB float [B,3,H,W] (FastACVNet_plus_preprocess.cu:21-29), on
    ``device`` (default: where the input is)."""
    t = torch.as_tensor(bgr_u8)
    if device is not None:
        t = t.to(device)
    x = t.flip(-1).permute(0, 3, 1, 2).float() / 255.0
    mean = torch.tensor(IMAGENET_MEAN, device=x.device).view(1, 3, 1, 1)
    std = torch.tensor(IMAGENET_STD, device=x.device).view(1, 3, 1, 1)
    return (x - mean) / std


def train_synthetic(model: torch.nn.Module, steps: int = 300, h: int = 96, w: int = 192, batch: int = 2,
                    lr: float = 5e-4, seed: int = 1000, device="cpu", log_every: int = 0) -> list[float]:
    """Adam on smooth-L1(prediction, ground-truth disparity) over fresh synthetic pairs (pair i of step s is
    ``stereo_pair(h, w, seed=seed + s * batch + i)``).  The model must map ImageNet-normalised RGB pairs to positive
    disparity [B,H,W] (Fast-ACVNet+).  Batch norms stay in eval mode (their affine parameters train).  Returns the
    loss per step; the model is left on ``device`` in eval mode."""
    from stereoalgorithms_amd.utils.synthetic import stereo_pair
    torch.manual_seed(seed)
    model = model.to(device).eval()
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    losses = []
    for s in range(steps):
        ls, rs, ds = zip(*[stereo_pair(h, w, seed=seed + s * batch + i) for i in range(batch)])
        left, right = imagenet_input(np.stack(ls), device), imagenet_input(np.stack(rs), device)
        gt = torch.from_numpy(np.stack(ds)).to(device)
        loss = F.smooth_l1_loss(model(left, right), gt)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
        if log_every and s % log_every == 0:
            print(f"[condition] step {s}: loss {losses[-1]:.3f}", flush=True)
    model.eval()
    for p in model.parameters():
        p.requires_grad_(False)
    return losses


def fp16_storage_agreement(model: torch.nn.Module, left: torch.Tensor, right: torch.Tensor,
                           keep_fp32=("hourglass.conv1_up", "hourglass_att.conv1_up")) -> float:
    """Fraction of pixels within 1 px between the fp32 oracle and the same oracle with every conv / batch-norm output
    rounded to fp16 (the engine's storage; the two selection-logit heads stay fp32 as in the engine).  A
    well-conditioned network is ~1.0; a random-init one ~0.45; fp16 overflow shows up as ~0."""
    import torch.nn as nn
    rounded = (nn.Conv2d, nn.Conv3d, nn.ConvTranspose2d, nn.ConvTranspose3d, nn.BatchNorm2d, nn.BatchNorm3d)

    def hook(mod, inp, out):
        return out.half().float()
    with torch.no_grad():
        ref = model(left, right)
        hs = [mod.register_forward_hook(hook) for n, mod in model.named_modules()
              if isinstance(mod, rounded) and not n.startswith(keep_fp32)]
        try:
            out = model(left, right)
        finally:
            for h in hs:
                h.remove()
    return float(((out - ref).abs() <= 1.0).float().mean())
