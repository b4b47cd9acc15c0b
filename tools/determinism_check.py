#!/usr/bin/env python3
"""Run one engine several times on identical inputs and report max |run_i - run_0| (graph-replay determinism)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="raftstereo-realtime")
    p.add_argument("--batch", type=int, default=2)
    p.add_argument("--height", type=int, default=96)
    p.add_argument("--width", type=int, default=128)
    p.add_argument("--iters", type=int, default=2)
    p.add_argument("--runs", type=int, default=4)
    a = p.parse_args()
    import torch
    import stereoalgorithms_amd  # noqa: F401
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.utils.synthetic import batch_pairs
    l, r = batch_pairs(a.batch, a.height, a.width, seed=3)
    eng = NativeStereoEngine(a.model, None, a.height, a.width, batch=a.batch, iters=a.iters)
    L, R = torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()
    outs = [eng.run(L, R).clone() for _ in range(a.runs)]
    torch.cuda.synchronize()
    d = [float((o - outs[0]).abs().max()) for o in outs]
    print(f"{a.model} b{a.batch} env NO_GRAPH={os.environ.get('SA_NO_GRAPH')}: max diff vs run0 {d}")


if __name__ == "__main__":
    main()
