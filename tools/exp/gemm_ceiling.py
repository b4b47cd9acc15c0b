#!/usr/bin/env python3
"""Library GEMM ceiling (torch.matmul -> hipBLASLt) for the conv-as-GEMM shapes of the RAFT hot convs."""
import torch
shapes = {"zr8": (153600, 3456, 256), "q8": (153600, 3456, 128), "fh8": (153600, 1152, 256),
          "zr1": (19200, 3456, 384), "q1": (19200, 1152, 128), "big": (8192, 8192, 8192)}
for name, (M, K, N) in shapes.items():
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(K, N, device="cuda", dtype=torch.float16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    reps = 20
    e0.record()
    for _ in range(reps):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    print(f"{name:5s} M={M:6d} K={K:5d} N={N:5d}: {us:8.2f} us  {2 * M * K * N / us / 1e6:8.1f} TFLOP/s", flush=True)
