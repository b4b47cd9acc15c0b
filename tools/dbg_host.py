import sys, numpy as np, torch
sys.path.insert(0, "/root/repo")
from stereoalgorithms_amd.models.engine import NativeStereoEngine
from stereoalgorithms_amd.utils.synthetic import batch_pairs
h, w = 64, 96
l, r = batch_pairs(1, h, w, seed=3)
left, right = torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()
for variant in range(4):
    eng = NativeStereoEngine("raftstereo-realtime", None, h, w, batch=1, iters=2)
    Q = np.array([[1, 0, 0, -w / 2], [0, 1, 0, -h / 2], [0, 0, 0, 400.0], [0, 0, 1 / 60.0, 0]], np.float32)
    eng.set_Q(Q)
    ys, xs = np.mgrid[0:h, 0:w].astype(np.float32)
    ident = np.stack([xs, ys], -1)
    if variant >= 1:
        eng.set_rectify_maps(ident, ident)
    d0, c0 = eng.run(left, right, cloud=True)
    if variant >= 2:
        d1, c1, rl, rr = eng.run(left, right, cloud=True, rectify=True, rectified=True)
    torch.cuda.synchronize()
    lh, rh_ = left.cpu().numpy(), right.cpu().numpy()
    if variant == 3:
        lh, rh_ = l.copy(), r.copy()
    res = eng.run_host(lh, rh_, cloud=True)
    dh = res[0]
    print(f"variant {variant}: dev {d0.cpu().numpy().ravel()[:3]} host {dh.ravel()[:3]} maxdiff {np.abs(dh - d0.cpu().numpy()).max()}"
          f" inputs equal {np.array_equal(lh, l)} {lh.dtype} {lh.shape} {lh.flags['C_CONTIGUOUS']}", flush=True)
    eng.close()
