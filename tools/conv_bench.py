#!/usr/bin/env python3
"""Micro-benchmark of the implicit-GEMM conv kernel on the RAFT-Stereo hot shapes.

    python3 tools/conv_bench.py [--iters 50] [--shapes zr1,q1,...]

Prints per shape: time per call (hipEvent, averaged), TFLOP/s, and the tile config the launcher chose.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# name: (N, H, W, Cin, Cout, k, splitk)   splitk 0 = auto (needs workspace), 1 = off
SHAPES = {
    "zr1": (1, 120, 160, 384, 256, 3, 0),    # GRU 1/4 z,r at batch 1
    "q1": (1, 120, 160, 384, 128, 3, 0),     # GRU 1/4 q at batch 1
    "fh1": (1, 120, 160, 128, 256, 3, 0),    # flow head conv1 at batch 1
    "enc1": (1, 120, 160, 128, 128, 3, 0),   # motion encoder out conv
    "zr16": (1, 60, 80, 384, 256, 3, 0),     # GRU 1/8 z,r
    "zr8": (8, 120, 160, 384, 256, 3, 1),    # GRU 1/4 z,r at batch 8
    "q8": (8, 120, 160, 384, 128, 3, 1),
    "fnet": (2, 240, 320, 64, 64, 3, 1),     # feature encoder layer1 at 1/2
    "fh8": (8, 120, 160, 128, 256, 3, 1),    # flow head conv1 at batch 8
    "enc8": (8, 120, 160, 128, 128, 3, 1),   # motion encoder out conv at batch 8
    "l1b8": (16, 240, 320, 64, 64, 3, 1),    # feature encoder layer1 at batch 8 (both images)
    "zr8s": (8, 60, 80, 384, 256, 3, 0),     # GRU 1/8 z,r at batch 8
    "mc1": (1, 120, 160, 64, 64, 3, 0),      # motion encoder convc2 / convf2 at batch 1 (auto split)
    "mc1s1": (1, 120, 160, 64, 64, 3, 1),    # same, no split
    "cf1": (1, 120, 160, 8, 64, 7, 0),       # motion encoder convf1 (7x7, 2 -> 8 padded channels)
    "zr32": (1, 30, 40, 256, 256, 3, 0),     # GRU 1/16 z,r at batch 1
    "zr8l": (1, 60, 80, 384, 256, 3, 0),     # GRU 1/8 z,r at batch 1
    "q8l": (1, 60, 80, 384, 128, 3, 0),      # GRU 1/8 q at batch 1 (SF 1/8 level, RT finest level)
    "q32": (1, 30, 40, 256, 128, 3, 0),      # GRU 1/16 q at batch 1
    "fhrt": (1, 60, 80, 128, 256, 3, 0),     # RT flow head conv1 at batch 1
    "fr8": (16, 480, 640, 64, 64, 3, 1),     # RAFT-SF fnet layer1 at batch 8 (full resolution, both images)
    # 7x7 stems (3 real of 8 padded channels): RAFT-SF fnet conv1 at batch 1 / 8, RAFT-RT stride 2
    "l2b8": (16, 240, 320, 96, 96, 3, 1),    # RAFT-SF fnet layer2 96 -> 96 at batch 8 (1/2 resolution, both images)
    "l2b1": (2, 240, 320, 96, 96, 3, 1),
    "l2s8": (16, 480, 640, 64, 96, -3, 1),   # layer2.0.conv1 64 -> 96 stride 2 at batch 8
    "l2s1": (2, 480, 640, 64, 96, -3, 1),
    "ds8": (16, 480, 640, 64, 96, -1, 1),    # layer2.0.downsample 1x1 stride 2 at batch 8
    "ds1": (2, 480, 640, 64, 96, -1, 1),
    "ds38": (16, 240, 320, 96, 128, -1, 1),  # layer3.0.downsample
    "stem1": (2, 480, 640, 8, 64, 7, 1),
    "stem8": (16, 480, 640, 8, 64, 7, 1),
    "stemrt": (2, 480, 640, 8, 64, -7, 1),
    # same GEMM as zr8 / q8 but 1x1 over K = 3456 channels: no im2col re-reads (isolates the gather's
    # cache traffic from the main loop)
    "zr8g": (8, 120, 160, 3456, 256, 1, 1),
    # Fast-ACVNet+ small-channel 3x3 convs (tactic 36 candidates) and its 1x1 expand (tactic 35)
    "fa32": (2, 240, 320, 32, 32, 3, 1),
    "fa48": (2, 120, 160, 48, 48, 3, 1),
    "fa64": (1, 240, 320, 64, 64, 3, 1),
    "fa16": (2, 120, 160, 32, 16, 3, 1),
    "faex": (2, 240, 320, 16, 96, 1, 1),
    "q8g": (8, 120, 160, 3456, 128, 1, 1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--cfgs", default="-1", help="comma list of tile configs (-1 = launcher's choice, 4 = glds3)")
    ap.add_argument("--splits", default="", help="comma list of split-K modes (0 = auto, 1 = off, >1 forced, -1 = stream-K); "
                    "default: the shape's own setting")
    ap.add_argument("--gemm-ref", type=int, default=0,
                    help="also time torch.matmul (hipBLASLt) on the conv's GEMM view [M,K] x [K,N], fp16")
    ap.add_argument("--graph", action="store_true",
                    help="time the --iters launches as one captured graph (no host launch overhead between calls)")
    ap.add_argument("--stats", type=int, default=0, help="fuse instance-norm statistics over N slots (engine: 16)")
    a = ap.parse_args()
    import torch
    from stereoalgorithms_amd import ops as O
    torch.manual_seed(0)
    ws = O.splitk_workspace(1 << 25, 8192)
    for name in a.shapes.split(","):
        if name in SHAPES:
            n, h, w, cin, cout, k, sk = SHAPES[name]
        else:  # ad-hoc "NxHxWxCINxCOUTkK" (3x3 / 1x1 / 7x7 stride 1, split auto), e.g. 1x30x40x256x256k3
            import re
            m = re.fullmatch(r"(\d+)x(\d+)x(\d+)x(\d+)x(\d+)k(\d)", name)
            if not m:
                raise SystemExit(f"unknown shape {name}")
            n, h, w, cin, cout, k = map(int, m.groups())
            sk = 0
        stride, k = (2, -k) if k < 0 else (1, k)
        x = torch.randn(n, h, w, cin, device="cuda").half()
        extra = dict(stride=stride)
        if k == 7:  # stem: 3 real channels in an 8-channel pixel
            x[..., 3:] = 0
            wt = torch.randn(cout, 3, k, k, device="cuda") / (3 * k * k) ** 0.5
            wp, kpad, _ = O.pack_conv_weight(wt, [(3, 8)])
            extra["cin_real"] = 3
        else:
            wt = torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5
            wp, kpad, _ = O.pack_conv_weight(wt)
        h, w = (h + 2 * (k // 2) - k) // stride + 1, (w + 2 * (k // 2) - k) // stride + 1
        b = torch.zeros(cout, device="cuda")
        out = torch.empty(n, h, w, cout, device="cuda", dtype=torch.float16)  # output grid
        if a.gemm_ref:
            M, K = n * h * w, cin * k * k
            ga = torch.randn(M, K, device="cuda").half()
            gb = (torch.randn(K, cout, device="cuda") / K ** 0.5).half()
            for _ in range(3):
                torch.matmul(ga, gb)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                torch.matmul(ga, gb)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / a.iters * 1e3
            print(f"{name:6s} hipBLASLt matmul M={M:7d} K={K:5d} N={cout:4d}: {us:8.2f} us  "
                  f"{2.0 * M * K * cout / us / 1e6:7.1f} TFLOP/s", flush=True)
            del ga, gb
        combos = [(cfg, sp) for cfg in map(int, a.cfgs.split(","))
                  for sp in (map(int, a.splits.split(",")) if a.splits else [sk])]
        for cfg, sk in combos:
            kw = dict(bias=b, out=out, splitk=sk, workspace=ws if sk != 1 or cfg in (37, 38) else None, tile_cfg=cfg, **extra)
            if a.stats:
                kw["stats"] = torch.zeros(16, n, cout, 2, dtype=torch.int64, device="cuda")
                kw["stats_slots"] = a.stats
                kw["splitk"], kw["workspace"] = 1, None
            try:
                for _ in range(3):
                    O.conv2d(x, wp, kpad, cout, k, k, **kw)
            except RuntimeError as e:
                print(f"{name:6s} cfg {cfg} split {sk}: {e}", flush=True)
                continue
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if a.graph:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(a.iters):
                        O.conv2d(x, wp, kpad, cout, k, k, **kw)
                g.replay()
                torch.cuda.synchronize()
                e0.record()
                g.replay()
                e1.record()
            else:
                e0.record()
                for _ in range(a.iters):
                    O.conv2d(x, wp, kpad, cout, k, k, **kw)
                e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / a.iters * 1e3
            flop = 2.0 * n * h * w * cout * (3 if k == 7 else cin) * k * k
            print(f"{name:6s} cfg {cfg:2d} split {sk} M={n * h * w:7d} K={cin * k * k:5d} N={cout:4d}: {us:8.2f} us  "
                  f"{flop / us / 1e6:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
