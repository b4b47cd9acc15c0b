"""Engine vs fp32 oracle at the reference's fixed configuration:
480x640 (/root/reference/RAFTStereo/src/TRTRAFTStereo.cpp:13-14) with the benchmarked iteration counts
(README_en.md:139-141 RAFT-Stereo sceneflow 32 / realtime 7, :244-246 CREStereo iter10), at batch 1 and
at the headline batch 8 — the exact graphs bench.py times, with the tactics the tuner picks at that size.

Random-init networks predict near-zero disparity, which would leave the correlation lookup, the pyramid
levels and the convex upsampling untested away from zero offset.  The oracles' ``scale_heads`` gives the
flow / mask heads a well-scaled init so the outputs are non-degenerate: every test
asserts mean |disparity| >= 5 px before comparing.  Each test also checks graph-replay determinism
(bitwise) and prints the selected conv tactics.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

H, W = 480, 640


def _pairs(b):
    from stereoalgorithms_amd.utils.synthetic import batch_pairs
    l, r = batch_pairs(b, H, W, seed=3)
    return torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()


def _rgb(t):
    return t.flip(-1).permute(0, 3, 1, 2).float()


def _stats(disp, ref, tag):
    err = (disp - ref).abs()
    rel = (err.norm() / ref.norm()).item()
    within = (err < 1.0).float().mean().item()
    print(f"{tag}: |ref| {ref.abs().mean().item():.3f} px (std {ref.std().item():.3f})  rel {rel:.3e}  "
          f"mean|err| {err.mean().item():.4f}  max {err.max().item():.3f}  <1px {within:.5f}")
    return rel, within, err


def _plan(path):
    from stereoalgorithms_amd.utils.plan import read_plan
    if os.path.exists(path):
        build, entries = read_plan(path)
        print(f"tactic plan (build {build}): {len(entries)} new entries")
        for e in entries[:40]:
            print(f"  cfg {e.cfg} splitk {e.splitk} {e.us:8.1f} us  {e.key}")


def _engine(tmp_path, monkeypatch, model, preset, batch, iters=-1):
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.utils.weights import save_model
    plan = str(tmp_path / "plan.txt")
    monkeypatch.setenv("SA_PLAN_CACHE", plan)
    path = save_model(model, tmp_path / "w.safetensors", preset)
    eng = NativeStereoEngine("", str(path), H, W, batch=batch, iters=iters)
    return eng, plan


@pytest.mark.parametrize("preset,iters,batch,tol", [
    ("raftstereo-sceneflow", 32, 1, 2e-2),
    ("raftstereo-sceneflow", 32, 8, 2e-2),
    ("raftstereo-realtime", 7, 1, 2e-2),
])
def test_raft_full_config(tmp_path, monkeypatch, preset, iters, batch, tol):
    from stereoalgorithms_amd.models import raft_stereo as R
    gains = {"raftstereo-sceneflow": (4.0, -0.25), "raftstereo-realtime": (4.0, -0.4)}[preset]
    m = R.scale_heads(R.build(preset, seed=0), *gains)
    eng, plan = _engine(tmp_path, monkeypatch, m, preset, batch, iters)
    left, right = _pairs(batch)
    disp = eng.run(left, right).clone()
    disp2 = eng.run(left, right)
    torch.cuda.synchronize()
    _plan(plan)
    assert torch.equal(disp, disp2), "graph replays differ"
    assert torch.isfinite(disp).all()
    m = m.cuda()
    with torch.no_grad():
        ref = torch.cat([-m(_rgb(left[i:i + 1]), _rgb(right[i:i + 1]), iters=iters)[1][:, 0] for i in range(batch)])
    assert ref.abs().mean().item() >= 5.0, "degenerate oracle output"
    rel, within, _ = _stats(disp, ref, f"{preset} b{batch} {iters} iters")
    assert rel < tol
    assert within > 0.98


def test_crestereo_iter10_full_config(tmp_path, monkeypatch):
    from stereoalgorithms_amd.models import crestereo as C
    m = C.scale_heads(C.build("crestereo-iter10", seed=0), 4.0, -0.15)
    eng, plan = _engine(tmp_path, monkeypatch, m, "crestereo-iter10", 1)
    left, right = _pairs(1)
    disp = eng.run(left, right).clone()
    disp2 = eng.run(left, right)
    torch.cuda.synchronize()
    _plan(plan)
    assert torch.equal(disp, disp2) and torch.isfinite(disp).all()
    m = m.cuda()
    with torch.no_grad():
        ref = m(_rgb(left), _rgb(right))[:, 0]
    assert ref.abs().mean().item() >= 5.0, "degenerate oracle output"
    rel, within, _ = _stats(disp, ref, "crestereo-iter10 b1")
    assert rel < 2e-2
    assert within > 0.98


def test_fastacvnet_end_to_end(tmp_path, monkeypatch):
    """Per-pixel end-to-end Fast-ACVNet+ parity at 480x640 (option b): >= 98 % of the pixels
    within 1 px of the fp32 oracle and |mean difference| <= 0.25 px.

    The weights are CONDITIONED: the seeded random init plus 300 Adam steps on synthetic pairs with known disparity
    (utils.condition.train_synthetic, on the GPU here).  A random-init network cannot be held to this: its top-24 /
    top-2 selections sit on near-equal logits, and even the fp32 oracle with fp16 activation storage agrees with
    itself within 1 px on ~45-55 % of the pixels when only the accumulation order changes
    (test_fastacvnet_random_weights_precision below keeps that study).  Trained, the same fp16-storage oracle agrees
    on 99.98 % (utils/condition.py), so what is left to measure is the engine's arithmetic."""
    from stereoalgorithms_amd.models import fast_acvnet as FA
    from stereoalgorithms_amd.utils.condition import fp16_storage_agreement, imagenet_input, train_synthetic
    m = FA.build("fastacvnet-plus", seed=0)
    losses = train_synthetic(m, steps=300, device="cuda")
    print(f"conditioning: smooth-L1 {losses[0]:.3f} -> {losses[-1]:.3f}")
    assert losses[-1] < 0.25 * losses[0]
    left, right = _pairs(1)
    # precondition: the network itself tolerates fp16 activation storage (else no fp16 engine could match it)
    agree = fp16_storage_agreement(m, imagenet_input(left), imagenet_input(right))
    print(f"fp16-storage oracle vs fp32 oracle: <1px {agree:.5f}")
    assert agree >= 0.99, agree
    eng, plan = _engine(tmp_path, monkeypatch, m.cpu(), "fastacvnet-plus", 1)
    disp = eng.run(left, right).clone()
    disp2 = eng.run(left, right)
    torch.cuda.synchronize()
    _plan(plan)
    assert torch.equal(disp, disp2) and torch.isfinite(disp).all()
    m = m.cuda()
    with torch.no_grad():
        ref = m(imagenet_input(left), imagenet_input(right)).reshape(disp.shape)
    assert ref.abs().mean().item() >= 5.0, "degenerate oracle output"
    rel, within, err = _stats(disp, ref, "fastacvnet-plus (conditioned) engine vs fp32")
    dm = abs(disp.mean().item() - ref.mean().item())
    print(f"mean disparity: engine {disp.mean().item():.3f} oracle-fp32 {ref.mean().item():.3f}")
    assert within >= 0.98, within
    assert dm <= 0.25, dm


def test_fastacvnet_random_weights_precision(tmp_path, monkeypatch):
    """Random-init Fast-ACVNet+ at 480x640 vs the oracle: a precision-sensitivity study, not a
    parity test (the per-pixel one is test_fastacvnet_end_to_end, on conditioned weights).

    The attention top-24 and the final top-2 candidate selections are discontinuous; on a random-init
    network the candidate logits are nearly tied, so the fp32 oracle itself, re-run with fp16 convs, picks
    different candidates on a large share of pixels.  The engine is therefore held to the oracle's own
    precision sensitivity: its agreement with the fp32 oracle must be at least as good as the oracle's fp16
    autocast run (minus a small margin), and both must agree on the disparity distribution.  Stage-by-stage
    arithmetic at this size is pinned separately (test_fast_acvnet_gpu.py::test_engine_chain_vs_oracle), and so
    is the end-to-end result given the engine's discrete choices: there the oracle recomputes everything in fp32
    from the images with the engine's top-24 / top-2 picks, the picks must be legitimate top-k choices of the
    oracle's own logits, and the disparity must match within 1 px on >= 99 % of the pixels.
    """
    from stereoalgorithms_amd.models import fast_acvnet as FA
    m = FA.sharpen(FA.build("fastacvnet-plus", seed=0))
    eng, plan = _engine(tmp_path, monkeypatch, m, "fastacvnet-plus", 1)
    left, right = _pairs(1)
    disp = eng.run(left, right).clone()
    disp2 = eng.run(left, right)
    torch.cuda.synchronize()
    _plan(plan)
    assert torch.equal(disp, disp2) and torch.isfinite(disp).all()
    m = m.cuda()
    dev = disp.device
    mean = torch.tensor([0.485, 0.456, 0.406], device=dev).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225], device=dev).view(1, 3, 1, 1)
    L, R = (_rgb(left) / 255.0 - mean) / std, (_rgb(right) / 255.0 - mean) / std
    with torch.no_grad():
        ref = m(L, R).reshape(disp.shape)
        with torch.autocast("cuda", dtype=torch.float16):
            ref16 = m(L, R).float().reshape(disp.shape)
    assert ref.abs().mean().item() >= 5.0, "degenerate oracle output"
    _, within16, err16 = _stats(ref16, ref, "fastacvnet-plus oracle fp16-autocast vs fp32")
    rel, within, err = _stats(disp, ref, "fastacvnet-plus engine vs fp32")
    assert within >= within16 - 0.05
    assert err.mean().item() <= 1.25 * err16.mean().item() + 0.1
    dm, d16 = abs(disp.mean().item() - ref.mean().item()), abs(ref16.mean().item() - ref.mean().item())
    print(f"mean disparity: engine {disp.mean().item():.3f} oracle-fp16 {ref16.mean().item():.3f} "
          f"oracle-fp32 {ref.mean().item():.3f}")
    assert dm <= 1.5 * d16 + 0.05 * ref.abs().mean().item()
    # Round 5: the attention / cost logits are fp32 in the engine.  Stored in fp16 they tied, and the lower-index rule
    # biased the mean disparity by ~4 px (42.35 vs 46.29 in round 4, the fp16-autocast oracle still shows it); now the
    # engine tracks the fp32 oracle's mean.  What remains is the top-2 choice among near-equal random-init cost logits
    # flipping under fp16 activation storage inside the hourglass -- the fp32 oracle with fp16-rounded activations and
    # fp32 logits flips as often (tests/test_fast_acvnet_cpu.py::test_fp16_storage_flips_come_from_near_ties).
    assert dm <= 0.6, dm
    assert within >= 0.4, within
