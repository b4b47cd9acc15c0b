#!/usr/bin/env python3
"""Stress the caller-stream <-> engine-stream hand-off: fresh engines, first-run output cloned on the
caller's (default) stream, compared against a synchronised re-run.  Prints mismatching trials."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    import torch
    import stereoalgorithms_amd  # noqa: F401
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.utils.synthetic import batch_pairs
    l, r = batch_pairs(2, 96, 128, seed=3)
    bad = 0
    for t in range(trials):
        junk = torch.randn(4 << 20, device="cuda")  # recycled allocator memory holds garbage
        del junk
        eng = NativeStereoEngine("raftstereo-realtime", None, 96, 128, batch=2, iters=2)
        first = eng.run(torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()).clone()
        torch.cuda.synchronize()
        again = eng.run(torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda())
        torch.cuda.synchronize()
        d = float((first - again).abs().max())
        if not d == 0.0:
            bad += 1
            print(f"trial {t}: first-run mismatch max {d}", flush=True)
        eng.close()
    print(f"SA_SYNC_FRAME={os.environ.get('SA_SYNC_FRAME')}: {bad}/{trials} trials mismatched", flush=True)


if __name__ == "__main__":
    main()
