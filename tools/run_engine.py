#!/usr/bin/env python3
"""Run a native engine for N frames (profiling driver for rocprofv3).

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -- python3 tools/run_engine.py --model raftstereo-sceneflow
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="raftstereo-sceneflow")
    p.add_argument("--batch", type=int, default=1)
    p.add_argument("--frames", type=int, default=10)
    p.add_argument("--height", type=int, default=480)
    p.add_argument("--width", type=int, default=640)
    p.add_argument("--iters", type=int, default=-1)
    p.add_argument("--no-graph", action="store_true")
    a = p.parse_args()
    import torch
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.utils.synthetic import batch_pairs
    l, r = batch_pairs(a.batch, a.height, a.width, seed=0)
    left, right = torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()
    eng = NativeStereoEngine(a.model, None, a.height, a.width, batch=a.batch, iters=a.iters,
                             use_graph=not a.no_graph)
    for _ in range(2):
        eng.run(left, right)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.frames):
        d = eng.run(left, right)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.frames * 1e3
    print(f"{a.model} B={a.batch} {a.height}x{a.width}: {dt:.3f} ms/step, {dt / a.batch:.3f} ms/frame, "
          f"mean disp {d.mean().item():.4f}")
    st = eng.stage_times()
    if st:
        print("device stages (ms): " + ", ".join(f"{k} {v:.3f}" for k, v in st))


if __name__ == "__main__":
    main()
