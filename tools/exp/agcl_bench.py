#!/usr/bin/env python3
"""Isolated timing of the AGCL correlation kernels at the CREStereo pyramid sizes (batch 1, 480x640 input).

    python3 tools/exp/agcl_bench.py [--reps 200]

Per (level, window, mode): mean us per launch over back-to-back launches on one stream (events around the loop),
for the per-tap 8-lane kernel (SA_AGCL_TILE=0) and the default dispatch (tiled warp-once kernel in iter mode).
In the engine the kernel shares the chip with the flow branch, so its traced duration there is longer.
"""
import argparse
import os

import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from stereoalgorithms_amd import ops as O


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    torch.manual_seed(0)
    for h, w in ((120, 160), (60, 80), (30, 40)):
        f1 = torch.randn(1, h, w, 256, device="cuda").half()
        f2 = torch.randn(1, h, w, 256, device="cuda").half()
        flow = (torch.randn(1, h, w, 2, device="cuda") * 4).contiguous()
        for small in (False, True):
            for mode in ("iter", "offset"):
                off = None if mode == "iter" else (torch.rand(1, h, w, 18, device="cuda") - 0.5).half()
                row = []
                outs = []
                for tile in ("0", "1"):
                    os.environ["SA_AGCL_TILE"] = tile
                    fn = lambda: O.agcl_corr(f1, f2, flow, off, small_patch=small, iter_mode=mode == "iter",
                                             out_channels=36)
                    outs.append(fn())
                    for _ in range(10):
                        fn()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.reps):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    row.append(e0.elapsed_time(e1) * 1000 / a.reps)
                d = (outs[0].float() - outs[1].float()).abs().max().item()
                print(f"{h:4d}x{w:<4d} {'3x3' if small else '1x9'} {mode:6s}  per-tap {row[0]:7.1f} us  "
                      f"default {row[1]:7.1f} us  max|diff| {d:.2e}", flush=True)


if __name__ == "__main__":
    main()
