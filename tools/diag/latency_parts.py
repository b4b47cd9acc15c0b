#!/usr/bin/env python3
"""Where the batch-1 timed region (bench.py latency block, RAFTStereo/src/TRTRAFTStereo.cpp:119-146) goes:
run_host with / without the point cloud vs the device-only frame (torch tensors already on the GPU), interleaved.

    python3 tools/diag/latency_parts.py --model raftstereo-realtime --frames 30
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="raftstereo-realtime")
    ap.add_argument("--frames", type=int, default=30)
    a = ap.parse_args()
    import numpy as np
    import stereoalgorithms_amd  # noqa: F401
    import torch
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.utils.synthetic import batch_pairs
    l, r = batch_pairs(1, 480, 640, seed=0)
    e = NativeStereoEngine(a.model, None, 480, 640, batch=1)
    Q = np.eye(4, dtype=np.float64)
    Q[2, 3], Q[3, 2] = 500.0, 1.0 / 120.0
    e.set_Q(Q)
    lt, rt = torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()
    arms = {
        "run_host cloud": lambda: e.run_host(l, r, cloud=True),
        "run_host no cloud": lambda: e.run_host(l, r, cloud=False),
        "device frame (+sync)": lambda: (e.run(lt, rt), torch.cuda.synchronize()),
        "device frame + cloud (+sync)": lambda: (e.run(lt, rt, cloud=True), torch.cuda.synchronize()),
    }
    for f in arms.values():
        for _ in range(3):
            f()
    ts = {k: [] for k in arms}
    for _ in range(a.frames):
        for k, f in arms.items():
            t0 = time.perf_counter()
            f()
            ts[k].append((time.perf_counter() - t0) * 1e3)
    for k, v in ts.items():
        print(f"{a.model} {k:30s} p50 {np.median(v):7.3f} ms  min {np.min(v):7.3f}", flush=True)


if __name__ == "__main__":
    main()
