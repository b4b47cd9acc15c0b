#!/usr/bin/env python3
"""bench.py's b8 DP step (world 1) with different H2D staging: where does the per-step input copy land?"""
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
l, r = batch_pairs(B, H, W, seed=0)
lh, rh = torch.from_numpy(l).pin_memory(), torch.from_numpy(r).pin_memory()
torch.cuda.set_stream(eng.main_stream)
cs = eng.main_stream


class Ahead:
    """copies for step t+1 issued (on `stream`) right after step t's frame is enqueued, 3 slots"""
    def __init__(self, stream, slots=3):
        self.s, self.slots = stream, slots
        self.bufs = [[torch.empty_like(lh, device=dev), torch.empty_like(rh, device=dev)] for _ in range(slots)]
        self.ready = [None] * slots
        self.freed = [None] * slots
        self.i = 0
        self._issue(0)

    def _issue(self, k):
        slot = k % self.slots
        with torch.cuda.stream(self.s):
            if self.freed[slot] is not None:
                self.s.wait_event(self.freed[slot])
            for d, h in zip(self.bufs[slot], (lh, rh)):
                d.copy_(h, non_blocking=True)
            ev = torch.cuda.Event(); ev.record(self.s)
            self.ready[slot] = ev

    def step(self, dp):
        k = self.i; self.i += 1
        slot = k % self.slots
        cs.wait_event(self.ready[slot])
        out = dp.step_async(*self.bufs[slot])
        ev = torch.cuda.Event(); ev.record(cs)
        self.freed[slot] = ev
        self._issue(k + 1)
        return out


def run(tag, make_step, steps=20):
    dp = DataParallelStereo(eng, world_size=1, rank=0, cloud=True)
    step = make_step()
    for _ in range(5):
        step(dp)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(dp)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    print(f"{tag:34s} {ms:8.3f} ms/step  {B * 1000 / ms:7.2f} FPS", flush=True)


def cur(stream):
    def mk():
        h = H2DPrefetcher([lh, rh], dev, stream=stream)
        return lambda dp: dp.step_async(*h.load([lh, rh]))
    return mk


dl, dr = lh.to(dev), rh.to(dev)
side_new = torch.cuda.Stream(dev)
only = sys.argv[1] if len(sys.argv) > 1 else ""
if only == "resident":
    run("no H2D (resident inputs)", lambda: (lambda dp: dp.step_async(dl, dr)), steps=6)
    run("plain engine.run loop", lambda: (lambda dp: eng.run(dl, dr)), steps=6)
if only == "cur":
    run("prefetcher on engine side stream", cur(eng.copy_stream), steps=6)
if only == "ahead":
    run("ahead, 3 slots, new stream", lambda: Ahead(side_new).step, steps=6)
for rep in range(0 if only else 2):
    run("no H2D (resident inputs)", lambda: (lambda dp: dp.step_async(dl, dr)))
    run("prefetcher on engine side stream", cur(eng.copy_stream))
    run("prefetcher on a new stream", cur(side_new))
    run("ahead, 3 slots, side stream", lambda: Ahead(eng.copy_stream).step)
    run("ahead, 3 slots, new stream", lambda: Ahead(side_new).step)
torch.cuda.synchronize()
torch.cuda.set_stream(torch.cuda.default_stream(dev))
eng.close()
