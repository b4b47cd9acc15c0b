#!/usr/bin/env python3
"""Host-side timeline of bench.py's DP step at world 1 (is the host ahead of the GPU?): per step, host ms spent in the
H2D prefetch load, in engine.run, and the device-side time of the H2D copies vs the previous frame (events)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from stereoalgorithms_amd.models.engine import NativeStereoEngine
from stereoalgorithms_amd.parallel.dp import DataParallelStereo, H2DPrefetcher
from stereoalgorithms_amd.utils.synthetic import batch_pairs

B, H, W = 8, 480, 640
dev = torch.device("cuda", 0)
eng = NativeStereoEngine("raftstereo-sceneflow", None, H, W, batch=B, seed=0)
Q = np.array([[1, 0, 0, -W / 2], [0, 1, 0, -H / 2], [0, 0, 0, 500.0], [0, 0, 1 / 60.0, 0]], np.float32)
eng.set_Q(Q)
dp = DataParallelStereo(eng, world_size=1, rank=0, cloud=True)
l, r = batch_pairs(B, H, W, seed=0)
lh, rh = torch.from_numpy(l).pin_memory(), torch.from_numpy(r).pin_memory()
torch.cuda.set_stream(eng.main_stream)
h2d = H2DPrefetcher([lh, rh], dev, stream=eng.copy_stream)
for _ in range(3):
    a, b = h2d.load([lh, rh]); dp.step_async(a, b)
torch.cuda.synchronize()
t0 = time.perf_counter()
rows = []
for i in range(8):
    ta = time.perf_counter()
    a, b = h2d.load([lh, rh])
    tb = time.perf_counter()
    dp.step_async(a, b)
    tc = time.perf_counter()
    rows.append(((ta - t0) * 1e3, (tb - ta) * 1e3, (tc - tb) * 1e3))
torch.cuda.synchronize()
tend = (time.perf_counter() - t0) * 1e3
for i, (s, ld, run) in enumerate(rows):
    print(f"step {i}: issued at {s:8.3f} ms  load {ld:7.3f} ms  run {run:7.3f} ms")
print(f"all done at {tend:.3f} ms ({tend / 8:.3f} ms/step)")
h2d = None
torch.cuda.set_stream(torch.cuda.default_stream(dev))
eng.close()
