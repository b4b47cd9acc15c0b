import sys, numpy as np
sys.path.insert(0, "/root/repo")
import torch
mode = sys.argv[1]
from stereoalgorithms_amd.models.engine import NativeStereoEngine
from stereoalgorithms_amd.utils.synthetic import batch_pairs
h, w = 64, 96
l, r = batch_pairs(1, h, w, seed=3)
if mode == "torch_first":
    torch.zeros(1).cuda()
eng = NativeStereoEngine("raftstereo-realtime", None, h, w, batch=1, iters=2)
print("engine created", flush=True)
res = eng.run_host(l.copy(), r.copy(), cloud=False)
print("host only", res[0].ravel()[:3], flush=True)
left, right = torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()
d0 = eng.run(left, right).cpu().numpy()
res = eng.run_host(l.copy(), r.copy(), cloud=False)
print(mode, "dev", d0.ravel()[:3], "host", res[0].ravel()[:3], "maxdiff", np.abs(res[0] - d0).max(), flush=True)
