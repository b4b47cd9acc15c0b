"""Native RAFT-Stereo engine (hipGraph, fp16 MFMA kernels) vs. the PyTorch fp32 oracle with the same
seeded weights (exported to safetensors and loaded by the C++ engine)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pairs(b, h, w):
    from stereoalgorithms_amd.utils.synthetic import batch_pairs
    l, r = batch_pairs(b, h, w, seed=3)
    return torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()


@pytest.mark.parametrize("preset,iters,hw,variant", [
    ("raftstereo-realtime", 7, (96, 160), ""),
    ("raftstereo-sceneflow", 6, (96, 128), ""),
    ("raftstereo-sceneflow", 6, (96, 128), "nosplit"),  # z/r + q convs (the batch > 2 default)
    ("raftstereo-sceneflow", 6, (96, 128), "nomenc"),  # motion head kernel + three convs instead of the fused encoder
])
def test_engine_matches_oracle(tmp_path, monkeypatch, preset, iters, hw, variant):
    from stereoalgorithms_amd.models import raft_stereo as R
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.utils.weights import save_model
    h, w = hw
    if variant == "nosplit":
        monkeypatch.setenv("SA_RAFT_GRU_SPLIT", "0")
    elif variant == "nomenc":
        monkeypatch.setenv("SA_RAFT_FUSE_MENC", "0")
    m = R.build(preset, seed=0)
    path = save_model(m, tmp_path / "w.safetensors", preset)
    left, right = _pairs(2, h, w)
    eng = NativeStereoEngine("", str(path), h, w, batch=2, iters=iters)
    disp = eng.run(left, right)
    disp2 = eng.run(left, right)  # graph replay is deterministic
    torch.cuda.synchronize()
    m = m.cuda()
    with torch.no_grad():
        rgb = lambda t: t.flip(-1).permute(0, 3, 1, 2).float()
        _, flow_up = m(rgb(left), rgb(right), iters=iters)
    ref = -flow_up[:, 0]
    err = (disp - ref).abs()
    rel = (err.norm() / ref.norm()).item()
    print(f"{preset}: |ref| mean {ref.abs().mean().item():.4f} max err {err.max().item():.4f} rel {rel:.4e}")
    assert torch.equal(disp, disp2)
    assert torch.isfinite(disp).all()
    assert rel < 3e-2


def test_engine_cloud_and_rectify_roundtrip():
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    h, w = 64, 96
    eng = NativeStereoEngine("raftstereo-realtime", None, h, w, batch=1, iters=2)
    Q = np.array([[1, 0, 0, -w / 2], [0, 1, 0, -h / 2], [0, 0, 0, 400.0], [0, 0, 1 / 60.0, 0]], np.float32)
    eng.set_Q(Q)
    ys, xs = np.mgrid[0:h, 0:w].astype(np.float32)
    ident = np.stack([xs, ys], -1)
    eng.set_rectify_maps(ident, ident)
    left, right = _pairs(1, h, w)
    d0, c0 = eng.run(left, right, cloud=True)
    d1, c1, rl, rr = eng.run(left, right, cloud=True, rectify=True, rectified=True)
    torch.cuda.synchronize()
    assert torch.equal(rl, left) and torch.equal(rr, right)  # identity maps
    assert torch.allclose(d0, d1)
    z = 400.0 / (d0 / 60.0)
    assert torch.allclose(c0[0, ..., 2], z[0], rtol=1e-3)
    # host path (reference timed region) agrees with the device path
    dh, ch, _, _ = eng.run_host(left.cpu().numpy(), right.cpu().numpy(), cloud=True)
    assert np.allclose(dh, d0.cpu().numpy(), atol=1e-5)
    # zero-copy host path: the engine's pinned buffers in and out, the reprojection writes them over PCIe
    hb = eng.host_buffers()
    hb["left"][...] = left.cpu().numpy()
    hb["right"][...] = right.cpu().numpy()
    hb["disp"][...] = -1.0
    hb["cloud"][...] = -1.0
    eng.run_host(hb["left"], hb["right"], cloud=True, out=hb["disp"], cloud_out=hb["cloud"])
    assert np.array_equal(hb["disp"], dh)
    assert np.array_equal(hb["cloud"], ch, equal_nan=True)


@pytest.mark.parametrize("graph", [True, False])
def test_stage_times(monkeypatch, graph):
    """Per-stage device timers (event nodes inside the captured frame graph, or eager events)."""
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    monkeypatch.setenv("SA_STAGE_TIMES", "1")
    h, w = 64, 96
    eng = NativeStereoEngine("raftstereo-sceneflow", None, h, w, batch=1, iters=3, use_graph=graph)
    left, right = _pairs(1, h, w)
    for _ in range(2):
        eng.run(left, right)
    torch.cuda.synchronize()
    st = dict(eng.stage_times())
    assert set(st) >= {"encoders+corr", "gru_iterations", "network"}
    assert all(v >= 0 for v in st.values()) and st["gru_iterations"] > 0


def test_replay_determinism_race_screen():
    """Race screen for the multi-stream frame graph: with parallel branches, split-K last-arriver
    reductions and slotted statistics, repeated replays and an eager (no-graph) run of the same
    engine configuration must agree bitwise."""
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    h, w = 96, 128
    left, right = _pairs(2, h, w)
    eng = NativeStereoEngine("raftstereo-sceneflow", None, h, w, batch=2, iters=4, seed=1)
    outs = [eng.run(left, right).clone() for _ in range(6)]
    eager = NativeStereoEngine("raftstereo-sceneflow", None, h, w, batch=2, iters=4, seed=1, use_graph=False)
    e = eager.run(left, right)
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    assert torch.equal(e, outs[0])
