import sys, numpy as np
sys.path.insert(0, "/root/repo")
import torch
flags = sys.argv[1]
if "I" in flags:
    torch.cuda.is_available()
if "Z" in flags:
    torch.zeros(1).cuda()
from stereoalgorithms_amd.models.engine import NativeStereoEngine
from stereoalgorithms_amd.utils.synthetic import batch_pairs
h, w = 64, 96
eng = NativeStereoEngine("raftstereo-realtime", None, h, w, batch=1, iters=2)
Q = np.array([[1, 0, 0, -w / 2], [0, 1, 0, -h / 2], [0, 0, 0, 400.0], [0, 0, 1 / 60.0, 0]], np.float32)
eng.set_Q(Q)
ys, xs = np.mgrid[0:h, 0:w].astype(np.float32)
ident = np.stack([xs, ys], -1)
eng.set_rectify_maps(ident, ident)
l, r = batch_pairs(1, h, w, seed=3)
left, right = torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()
d0, c0 = eng.run(left, right, cloud=True)
if "R" in flags:
    d1, c1, rl, rr = eng.run(left, right, cloud=True, rectify=True, rectified=True)
torch.cuda.synchronize()
if "T" in flags:
    z = 400.0 / (d0 / 60.0)
    ok = torch.allclose(c0[0, ..., 2], z[0], rtol=1e-3)
dh = eng.run_host(left.cpu().numpy(), right.cpu().numpy(), cloud="C" in flags)[0]
print(flags, "maxdiff", np.abs(dh - d0.cpu().numpy()).max(), dh.ravel()[:2], flush=True)
