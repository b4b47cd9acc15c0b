#!/usr/bin/env python3
"""Re-tune engines from scratch several times and report tactic-verification rejections.

    python tools/diag/tune_verify.py [model:batch ...] [--reps N]

The tuner compares every candidate tactic's output with the first candidate's (runtime.cpp tune_conv) and
logs / skips a disagreeing one; this driver clears the process-wide plan before each build so every conv
shape is re-timed and re-verified, and prints the engine output's mean so a wrong tactic would show."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("specs", nargs="*", default=["raftstereo-sceneflow:1"])
    p.add_argument("--reps", type=int, default=2)
    a = p.parse_args()
    os.environ["SA_PLAN_DIR"] = ""  # no plan files: every build tunes
    import torch
    from stereoalgorithms_amd._native import dev
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.utils.synthetic import batch_pairs
    L = dev()
    H, W = 480, 640
    for spec in a.specs:
        model, b = spec.split(":")
        b = int(b)
        l, r = batch_pairs(b, H, W, seed=0)
        left, right = torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()
        for rep in range(a.reps):
            L.sa_conv_plan_clear()
            r0 = L.sa_conv_tune_rejects()
            eng = NativeStereoEngine(model, None, H, W, batch=b)
            d = eng.run(left, right)
            torch.cuda.synchronize()
            print(f"{model} b{b} rep {rep}: tuned {eng.tuned_shapes} shapes, rejected "
                  f"{L.sa_conv_tune_rejects() - r0} candidates, mean disp {d.mean().item():.5g}, "
                  f"finite {torch.isfinite(d).float().mean().item():.4f}", flush=True)
            del eng


if __name__ == "__main__":
    main()
