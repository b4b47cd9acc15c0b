#!/usr/bin/env python3
"""Back-to-back graph replays with nothing in between (like tools/run_engine.py's timing loop), then compare
every replay's disparity with the first one.

    python tools/diag/replay_stress.py --model crestereo-iter10 --reps 24 [--drop]

--drop releases each output tensor right away (the caching allocator recycles it for the next replay, as in
run_engine.py); by default all outputs stay alive.  Prints how many replays differ and the worst one."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="crestereo-iter10")
    p.add_argument("--batch", type=int, default=1)
    p.add_argument("--reps", type=int, default=24)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--drop", action="store_true")
    p.add_argument("--host", action="store_true", help="run_host path (pinned H2D/D2H on the engine stream)")
    p.add_argument("--canary", type=int, default=0,
                   help="allocate this many 1/4/32 MiB torch tensors of a constant after the engine is built and "
                        "check them after every round (stray writes from the frame into freed memory)")
    a = p.parse_args()
    import torch
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.utils.synthetic import batch_pairs
    H, W = 480, 640
    l, r = batch_pairs(a.batch, H, W, seed=0)
    left, right = torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()
    eng = NativeStereoEngine(a.model, None, H, W, batch=a.batch)
    if a.host:
        def run_once():
            return torch.from_numpy(eng.run_host(l, r, cloud=False)[0])
    else:
        def run_once():
            return eng.run(left, right)
    canaries = []
    for i in range(a.canary):
        for mib in (1, 4, 32):
            canaries.append(torch.full((mib << 18,), 7.0, device="cuda"))
    ref = run_once().clone()
    torch.cuda.synchronize()
    ref_host = ref.cpu()
    print(f"after first frame: non-zero split-K counters {eng.nonzero_splitk_counters()}", flush=True)
    tag = (f"{a.model} b{a.batch} pc={os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE', '(default)')} "
           f"blocking={os.environ.get('SA_ENGINE_STREAM_BLOCKING', '0')} drop={a.drop} host={a.host} "
           f"nograph={os.environ.get('SA_NO_GRAPH', '0')} tune={os.environ.get('SA_TUNE', '1')}")
    total_bad = 0
    for rnd in range(a.rounds):
        outs, sums = [], []
        for i in range(a.reps):
            d = run_once()
            if a.drop:
                sums.append(d.double().sum())  # one reduction per replay, on the caller stream
            else:
                outs.append(d)
        torch.cuda.synchronize()
        if a.drop:
            s0 = ref.double().sum()
            bad = [i for i, s in enumerate(sums) if not torch.equal(s, s0)]
            worst = max((abs(float(sums[i] - s0)) for i in bad), default=0.0)
        else:
            diffs = [float((o - ref).abs().max()) if torch.isfinite(o).all() else float("inf") for o in outs]
            bad = [i for i, x in enumerate(diffs) if x != 0.0]
            worst = max(diffs)
        if not a.drop:
            hb = sum(1 for o in outs if not torch.equal(o.cpu(), ref_host))
            print(f"  host-side reference: {hb}/{a.reps} replays differ; device ref still equal to host copy: "
                  f"{torch.equal(ref.cpu(), ref_host)}", flush=True)
        if canaries:
            hit = [i for i, c in enumerate(canaries) if not bool((c == 7.0).all())]
            print(f"  canaries overwritten: {len(hit)}/{len(canaries)} {hit[:8]}", flush=True)
        total_bad += len(bad)
        print(f"{tag} round {rnd}: {len(bad)}/{a.reps} replays differ (first {bad[:6]}), worst {worst:.4g}, "
              f"non-zero split-K counters {eng.nonzero_splitk_counters()}", flush=True)
    print(f"{tag} TOTAL bad replays {total_bad}", flush=True)
    return 0 if total_bad == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
