#!/usr/bin/env python3
"""Compare RAFT-Stereo engine outputs across stream modes in one process (same tuned plans).

Each engine reads SA_RAFT_PARALLEL / SA_RAFT_PIPELINE at construction, so the modes are built one after
another with the environment changed in between; plans are process-wide, so every mode launches the same
tactics and the outputs should agree to fp16 rounding of the conv order only (bitwise in practice)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.utils.synthetic import batch_pairs
    model = sys.argv[1] if len(sys.argv) > 1 else "raftstereo-sceneflow"
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    H, W = 480, 640
    l, r = batch_pairs(batch, H, W, seed=0)
    left, right = torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()
    modes = [("serial", {"SA_RAFT_PARALLEL": "0"}), ("par+pipe(auto)", {}), ("par,nopipe", {"SA_RAFT_PIPELINE": "0"}),
             ("par,pipe1", {"SA_RAFT_PIPELINE": "1"}), ("par,pipe2", {"SA_RAFT_PIPELINE": "2"}),
             ("serial,unfused-menc", {"SA_RAFT_PARALLEL": "0", "SA_RAFT_FUSE_MENC": "0"}),
             ("serial,nograph", {"SA_RAFT_PARALLEL": "0", "SA_NO_GRAPH": "1"}),
             ("par,nograph", {"SA_NO_GRAPH": "1"})]
    ref = None
    for name, env in modes:
        saved = {k: os.environ.get(k) for k in ("SA_RAFT_PIPELINE", "SA_RAFT_PARALLEL", "SA_NO_GRAPH",
                                                 "SA_RAFT_FUSE_MENC")}
        for k in saved:
            os.environ.pop(k, None)
        os.environ.update(env)
        eng = NativeStereoEngine(model, None, H, W, batch=batch)
        outs = [eng.run(left, right).clone() for _ in range(2)]
        torch.cuda.synchronize()
        d = outs[-1]
        fin = torch.isfinite(d).float().mean().item()
        msg = f"{name:16s} mean {d.mean().item():.5g} absmax {d.abs().max().item():.4g} finite {fin:.4f}"
        msg += f" replay-equal {torch.equal(outs[0], outs[1])}"
        if ref is None:
            ref = d
        else:
            msg += f" max|d-ref| {(d - ref).abs().max().item():.4g}"
        print(msg, flush=True)
        del eng
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


if __name__ == "__main__":
    main()
