"""Fast-ACVNet+ precision study on the CPU oracle (the engine's mean disparity sat 4 px below the
fp32 oracle's).  The engine stores activations in fp16 between layers; the oracle is rerun with every conv / batch-norm
output rounded to fp16 to see which rounding moves the result:

* rounding the two selection-logit heads (``hourglass_att.conv1_up`` -> top-24, ``hourglass.conv1_up`` -> top-2) turns
  near-equal logits into exact ties, which the ONNX TopK rule (lower index first) resolves towards small disparities:
  a bias of several px in the mean disparity.  The engine now writes both heads in fp32 (fast_acvnet.cpp).
* with fp32 logits and fp16 storage everywhere else the mean disparity is unbiased; per pixel, the random-init
  network's near-tied top-2 cost logits still flip under the ~1e-3 perturbations -- the fp32 oracle itself does so
  under fp16 storage, so this is tie-breaking on an untrained network, not an arithmetic defect (the teacher-forced
  GPU test pins the arithmetic given the discrete choices).
"""
import pytest
import torch
import torch.nn as nn

from stereoalgorithms_amd.models import fast_acvnet as FA
from stereoalgorithms_amd.utils.synthetic import batch_pairs

MEAN = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
STD = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
LOGIT_HEADS = ("hourglass.conv1_up", "hourglass_att.conv1_up")
ROUNDED = (nn.Conv2d, nn.Conv3d, nn.ConvTranspose2d, nn.ConvTranspose3d, nn.BatchNorm2d, nn.BatchNorm3d)


def _fp16_storage(m, keep_logits_fp32):
    def hook(mod, inp, out):
        return out.half().float()
    return [mod.register_forward_hook(hook) for n, mod in m.named_modules()
            if isinstance(mod, ROUNDED) and not (keep_logits_fp32 and n.startswith(LOGIT_HEADS))]


@pytest.mark.timeout(600)
def test_fp16_storage_flips_come_from_near_ties():
    torch.set_num_threads(max(1, min(8, torch.get_num_threads())))
    m = FA.sharpen(FA.build("fastacvnet-plus", seed=0))
    l8, r8 = batch_pairs(1, 240, 320, seed=5)
    L = (torch.from_numpy(l8).permute(0, 3, 1, 2).flip(1).float() / 255 - MEAN) / STD
    R = (torch.from_numpy(r8).permute(0, 3, 1, 2).flip(1).float() / 255 - MEAN) / STD
    with torch.no_grad():
        ref = m(L, R)
    out = {}
    for keep in (False, True):
        hs = _fp16_storage(m, keep)
        with torch.no_grad():
            out[keep] = m(L, R)
        for h in hs:
            h.remove()
    bias16 = (out[False].mean() - ref.mean()).item()
    bias32 = (out[True].mean() - ref.mean()).item()
    print(f"mean disparity shift: fp16 logits {bias16:+.3f} px, fp32 logits {bias32:+.3f} px (ref {ref.mean():.2f})")
    assert bias16 < -2.0  # fp16 logits: ties -> lower indices -> smaller disparities
    assert abs(bias32) < 0.6


def test_conditioning_trainer_reduces_loss():
    """utils.condition.train_synthetic (the conditioned weights of the GPU parity test): deterministic fresh pairs,
    loss falls, the model comes back in eval mode with frozen parameters."""
    from stereoalgorithms_amd.utils.condition import train_synthetic
    torch.set_num_threads(max(1, min(8, torch.get_num_threads())))
    m = FA.build("fastacvnet-plus", seed=0)
    losses = train_synthetic(m, steps=12, h=64, w=128, batch=1)
    assert len(losses) == 12 and losses[-1] < losses[0]
    assert not m.training and not any(p.requires_grad for p in m.parameters())
