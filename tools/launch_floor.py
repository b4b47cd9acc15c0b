#!/usr/bin/env python3
"""Per-kernel fixed cost inside a replayed graph: chains of N dependent launches of the zeroing kernel (sa_zero)
over buffers of growing size, captured in one hipGraph, replayed and timed.  Separates the launch-to-launch floor
(tiny buffers) from the cost of the dirty data each kernel leaves behind (large buffers) on this chip.

    python3 tools/launch_floor.py [--n 200]
"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    a = ap.parse_args()
    import torch
    from stereoalgorithms_amd import _native as N
    lib = N.dev()
    lib.sa_zero.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p]
    lib.sa_zero.restype = C.c_int
    for kb in (0.25, 4, 64, 1024, 8192, 32768):
        nbytes = int(kb * 1024)
        buf = torch.empty(max(nbytes, 256) // 4, dtype=torch.float32, device="cuda")
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
                for _ in range(a.n):
                    lib.sa_zero(C.c_void_p(buf.data_ptr()), nbytes, st)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (5 * a.n)
        print(f"zero {kb:8.2f} KiB per kernel: {us:7.2f} us per launch in a {a.n}-kernel graph chain "
              f"({nbytes / max(us, 1e-9) / 1e3:.1f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
