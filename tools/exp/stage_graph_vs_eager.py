#!/usr/bin/env python3
"""Stage times of one preset with the frame graph vs eager launches (do the graph's parallel branches overlap?)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["SA_STAGE_TIMES"] = "1"
import numpy as np
import torch
import stereoalgorithms_amd  # noqa
from stereoalgorithms_amd.models.engine import NativeStereoEngine
from stereoalgorithms_amd.utils.synthetic import batch_pairs
model = sys.argv[1] if len(sys.argv) > 1 else "raftstereo-sceneflow"
l, r = batch_pairs(1, 480, 640, seed=0)
L, R = torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()
for g in (True, False):
    e = NativeStereoEngine(model, None, 480, 640, batch=1, seed=0, use_graph=g)
    for _ in range(5):
        e.run(L, R)
    torch.cuda.synchronize()
    acc = {}
    for _ in range(10):
        e.run(L, R)
        torch.cuda.synchronize()
        for k, v in e.stage_times():
            acc.setdefault(k, []).append(v)
    print(("graph" if g else "eager"), {k: round(float(np.median(v)), 3) for k, v in acc.items()}, flush=True)
    e.close()
