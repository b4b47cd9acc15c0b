import numpy as np
import pytest
import torch


@pytest.mark.parametrize("graph", [False, True])
def test_rt(graph):
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.utils.synthetic import batch_pairs
    h, w = 64, 96
    eng = NativeStereoEngine("raftstereo-realtime", None, h, w, batch=1, iters=2, use_graph=graph)
    Q = np.array([[1, 0, 0, -w / 2], [0, 1, 0, -h / 2], [0, 0, 0, 400.0], [0, 0, 1 / 60.0, 0]], np.float32)
    eng.set_Q(Q)
    ys, xs = np.mgrid[0:h, 0:w].astype(np.float32)
    ident = np.stack([xs, ys], -1)
    eng.set_rectify_maps(ident, ident)
    l, r = batch_pairs(1, h, w, seed=3)
    left, right = torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()
    d0, c0 = eng.run(left, right, cloud=True)
    torch.cuda.synchronize()
    print("step1 ok", flush=True)
    d1, c1, rl, rr = eng.run(left, right, cloud=True, rectify=True, rectified=True)
    torch.cuda.synchronize()
    print("step2 ok", flush=True)
    dh = eng.run_host(l.copy(), r.copy(), cloud=False)[0]
    print("step3 ok", np.abs(dh - d0.cpu().numpy()).max(), flush=True)
    dh = eng.run_host(l.copy(), r.copy(), cloud=True)[0]
    print("step4 ok", np.abs(dh - d0.cpu().numpy()).max(), flush=True)
    assert np.allclose(dh, d0.cpu().numpy(), atol=1e-5)
