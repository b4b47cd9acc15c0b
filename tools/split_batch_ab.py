#!/usr/bin/env python3
"""A/B: one batch-B engine vs the same B pairs as S concurrent sub-batch engines (B/S pairs each) on S torch
streams, interleaved rounds in one process (cdna_hip_programming.md rule 24).

    python3 tools/split_batch_ab.py --model raftstereo-sceneflow --batch 8 --splits 1,2,4 --rounds 3 --steps 10

The frame graphs of the sub-engines are independent, so the GPU can run one sub-batch's small-grid phases
(motion encoder, coarse GRU levels, flow head) under another's large GEMMs.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="raftstereo-sceneflow")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--splits", default="1,2")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--width", type=int, default=640)
    a = ap.parse_args()
    import stereoalgorithms_amd  # noqa: F401
    import torch
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.utils.synthetic import batch_pairs
    l, r = batch_pairs(a.batch, a.height, a.width, seed=0)
    left, right = torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()
    arms = {}
    for s in map(int, a.splits.split(",")):
        sub = a.batch // s
        engs = [NativeStereoEngine(a.model, None, a.height, a.width, batch=sub) for _ in range(s)]
        streams = [torch.cuda.Stream() for _ in range(s)]
        arms[s] = (engs, streams, sub)

    def step(s):
        engs, streams, sub = arms[s]
        cur = torch.cuda.current_stream()
        outs = []
        for i, (e, st) in enumerate(zip(engs, streams)):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                outs.append(e.run(left[i * sub:(i + 1) * sub], right[i * sub:(i + 1) * sub]))
        for st in streams:
            cur.wait_stream(st)
        return outs

    ref = torch.cat(step(1)) if 1 in arms else None
    for s in arms:
        for _ in range(2):
            step(s)
        if ref is not None and s != 1:
            d = torch.cat(step(s))
            torch.cuda.synchronize()
            print(f"split {s}: max |disp - batch engine| = {(d - ref).abs().max().item():.3e}", flush=True)
    torch.cuda.synchronize()
    res = {s: [] for s in arms}
    for _ in range(a.rounds):
        for s in arms:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step(s)
            torch.cuda.synchronize()
            res[s].append((time.perf_counter() - t0) / a.steps * 1e3)
    for s, v in res.items():
        v = sorted(v)
        print(f"{a.model} B={a.batch} as {s} x {a.batch // s}: median {v[len(v) // 2]:.3f} ms/step  min {v[0]:.3f}  "
              f"({a.batch * 1000.0 / v[len(v) // 2]:.1f} FPS)", flush=True)


if __name__ == "__main__":
    main()
