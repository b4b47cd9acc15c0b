#!/usr/bin/env python3
"""Isolated bandwidth of the instance-norm apply kernel at the RAFT-SF b8 feature-encoder sizes.

    python3 tools/exp/norm_bench.py

[16, 480, 640, 64] (layer 1, full resolution) and [16, 240, 320, 96] (layer 2) fp16, plain relu(IN(x)) and the
residual form relu(x' + relu(IN(y))), 16 statistic slots as in the engine; reports us per call and the effective
HBM bandwidth (bytes read + written / time).  The stand-alone copy (torch) of the same tensor is the reference.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from stereoalgorithms_amd import ops as O  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


def main():
    torch.manual_seed(0)
    for shape in ((16, 480, 640, 64), (16, 240, 320, 96)):
        n, h, w, c = shape
        x = torch.randn(shape, device="cuda").half()
        r = torch.randn(shape, device="cuda").half()
        out = torch.empty_like(x)
        st = torch.zeros(16, n, c, 2, dtype=torch.int64, device="cuda")
        st[0, ..., 0] = 0
        st[0, ..., 1] = int(h * w * (1 << 24))  # unit variance in the fixed-point scale (value irrelevant for speed)
        nb = x.numel() * 2
        t_copy = timeit(lambda: out.copy_(x))
        t_plain = timeit(lambda: O.instnorm_apply(x, st, act="relu", out=out, slots=16))
        t_res = timeit(lambda: O.instnorm_apply(x, st, act="relu", res=r, act2="relu", out=out, slots=16))
        print(f"{shape}: copy {t_copy:7.1f} us ({2 * nb / t_copy / 1e6:5.2f} TB/s)  apply {t_plain:7.1f} us "
              f"({2 * nb / t_plain / 1e6:5.2f} TB/s)  apply+res {t_res:7.1f} us ({3 * nb / t_res / 1e6:5.2f} TB/s)",
              flush=True)


if __name__ == "__main__":
    main()
