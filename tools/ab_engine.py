#!/usr/bin/env python3
"""In-process A/B of engine variants selected by an environment knob read at engine build time.

    python3 tools/ab_engine.py --knob SA_RAFT_GRU_SPLIT --values 0,1 --model raftstereo-sceneflow --batch 8

Builds one engine per value (the knob is set while that engine is constructed), then times them in
interleaved rounds (cdna_hip_programming.md §5.4 rule 24: cross-process numbers on different boxes
are not comparable) and prints per-variant median / min ms per step.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--knob", required=True)
    p.add_argument("--values", default="0,1")
    p.add_argument("--model", default="raftstereo-sceneflow")
    p.add_argument("--batch", type=int, default=8)
    p.add_argument("--rounds", type=int, default=6)
    p.add_argument("--frames", type=int, default=5)
    p.add_argument("--clear-plan", action="store_true",
                   help="forget the in-process tactic plan before each engine (knobs that change what the tuner picks)")
    a = p.parse_args()
    import numpy as np
    import torch
    import stereoalgorithms_amd  # noqa: F401
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.utils.synthetic import batch_pairs
    l, r = batch_pairs(a.batch, 480, 640, seed=0)
    left, right = torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()
    engines, outs = {}, {}
    for v in a.values.split(","):
        os.environ[a.knob] = v
        if a.clear_plan:
            os.environ["SA_PLAN_DIR"] = ""  # no plan files either: every engine tunes under its own knob value
            from stereoalgorithms_amd import _native as N
            N.require_native().sa_conv_plan_clear()
        e = NativeStereoEngine(a.model, None, 480, 640, batch=a.batch, seed=0)
        for _ in range(2):
            d = e.run(left, right)
        torch.cuda.synchronize()
        outs[v] = d.clone()
        engines[v] = e
    times = {v: [] for v in engines}
    for _ in range(a.rounds):
        for v, e in engines.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.frames):
                e.run(left, right)
            torch.cuda.synchronize()
            times[v].append((time.perf_counter() - t0) / a.frames * 1e3)
    ref = next(iter(outs.values()))
    for v in engines:
        t = np.array(times[v])
        diff = (outs[v] - ref).abs().max().item()
        print(f"{a.knob}={v}: median {np.median(t):.3f} ms/step  min {t.min():.3f}  "
              f"(max |disp - first| {diff:.4g})", flush=True)


if __name__ == "__main__":
    main()
