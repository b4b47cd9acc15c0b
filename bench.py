#!/usr/bin/env python3
"""Flagship benchmark: RAFT-Stereo sceneflow 480x640 (32 GRU iterations) throughput on N MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` (N>1 under torch.distributed.run).
One step = every rank runs its shard of stereo pairs (``--per-gpu-batch``, default 8 => 64 pairs on
8 GPUs, BASELINE.json config 5) through the native engine (one hipGraph per frame batch: preprocess,
encoders, corr pyramid, 32 ConvGRU iterations, convex upsample, reprojection), fed by an H2D copy
of the inputs from pinned host memory (copy stream, double-buffered, overlapping the previous step), then an RCCL all-gather of the disparity maps over xGMI
(issued async on the process group's stream, so step t's gather overlaps step t+1's frame graph).
K steps are timed between barrier + device synchronize; rank 0 prints ONE JSON line with the
whole-job FPS (max time over ranks).  Data: synthetic stereo pairs; weights: seeded random init of
the upstream architecture.

Also reported (rank 0, extra fields): batch-1 latency in the reference's timed region (pinned copy,
H2D, network, reprojection, D2H of disparity + point cloud; RAFTStereo/src/TRTRAFTStereo.cpp:119-146)
for the sceneflow and realtime presets.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import stereoalgorithms_amd  # noqa: E402,F401  (HIP runtime env defaults before torch touches the GPU)

BASELINE_MS = {"raftstereo-sceneflow": 38.0, "raftstereo-realtime": 11.0}  # RTX 3090, README_en.md:139-141
# the other model families' published RTX 3090 numbers (README_en.md:192-194,244-246,293-295)
OTHER_MS = {"crestereo-iter2": 12.0, "crestereo-iter5": 23.0, "crestereo-iter10": 42.0, "hitnet-d400": 15.0,
            "fastacvnet-plus": 12.0}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--model", default="raftstereo-sceneflow")
    p.add_argument("--per-gpu-batch", type=int, default=8)
    p.add_argument("--height", type=int, default=480)
    p.add_argument("--width", type=int, default=640)
    p.add_argument("--latency-frames", type=int, default=20)
    p.add_argument("--no-latency", action="store_true")
    return p.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # one rank per GPU; more ranks than GPUs only for a gloo rehearsal of the multi-rank path
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        # bounded collectives: a rank that dies or hangs fails the job instead of stalling it
        from datetime import timedelta
        backend = os.environ.get("SA_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI
        dist.init_process_group(backend, rank=rank, world_size=world,
                                device_id=torch.device("cuda", local) if backend == "nccl" else None,
                                timeout=timedelta(seconds=int(os.environ.get("SA_DIST_TIMEOUT", "600"))))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.parallel.dp import DataParallelStereo
    from stereoalgorithms_amd.utils.synthetic import batch_pairs

    B, H, W = args.per_gpu_batch, args.height, args.width
    Q = np.array([[1, 0, 0, -W / 2], [0, 1, 0, -H / 2], [0, 0, 0, 500.0], [0, 0, 1 / 60.0, 0]], np.float32)
    eng = NativeStereoEngine(args.model, None, H, W, batch=B, device=dev.index, seed=0)
    eng.set_Q(Q)
    dp = DataParallelStereo(eng, world_size=world, rank=rank)
    l_np, r_np = batch_pairs(B, H, W, seed=100 * rank)
    left_h = torch.from_numpy(l_np).pin_memory()
    right_h = torch.from_numpy(r_np).pin_memory()
    from stereoalgorithms_amd.parallel.dp import H2DPrefetcher
    h2d = H2DPrefetcher([left_h, right_h], dev)

    def step():
        # every step copies its inputs H2D (copy stream, double-buffered: overlaps the previous step's
        # frame graph); the all-gather of step t (RCCL's own stream) overlaps step t+1's frame graph
        left, right = h2d.load([left_h, right_h])
        return dp.step_async(left, right)

    for _ in range(args.warmup):
        step()
    dp.flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pending = step()
    out = pending.wait()
    dp.flush()  # every step's collective is complete inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    assert out.shape == (world * B, H, W) and torch.isfinite(out).all()

    ms_step = dt / args.steps * 1e3
    fps = world * B * args.steps / dt
    extra = {}
    # batch-1 latency block: single-process runs only (N = 1 already reports it; in a multi-rank job the
    # other ranks would sit in process-group teardown while rank 0 builds and tunes seven more engines)
    if rank == 0 and world == 1 and not args.no_latency:
        del eng
        os.environ["SA_STAGE_TIMES"] = "1"  # per-stage device times (event nodes in the frame graph)
        for preset in ("raftstereo-sceneflow", "raftstereo-realtime", *OTHER_MS):
            e1 = NativeStereoEngine(preset, None, H, W, batch=1, device=dev.index, seed=0)
            e1.set_Q(Q)
            l1, r1 = l_np[:1].copy(), r_np[:1].copy()
            for _ in range(3):
                e1.run_host(l1, r1, cloud=True)
            ts = []
            for _ in range(args.latency_frames):
                t1 = time.perf_counter()
                e1.run_host(l1, r1, cloud=True)
                ts.append((time.perf_counter() - t1) * 1e3)
            ts = np.array(ts)
            extra[preset] = {"latency_ms_mean": round(float(ts.mean()), 3),
                             "latency_ms_p50": round(float(np.median(ts)), 3),
                             "latency_ms_p99": round(float(np.percentile(ts, 99)), 3),
                             "fps_b1": round(1000.0 / float(ts.mean()), 2),
                             "baseline_ms_rtx3090": {**BASELINE_MS, **OTHER_MS}[preset],
                             "speedup_vs_baseline": round({**BASELINE_MS, **OTHER_MS}[preset] / float(ts.mean()), 3),
                             "device_stages_ms": {k: round(v, 3) for k, v in e1.stage_times()}}
            e1.close()
    if rank == 0:
        base_fps = 1000.0 / BASELINE_MS[args.model]
        rec = {
            "metric": f"{args.model} {H}x{W} throughput (frames/s, whole job)",
            "value": round(fps, 3),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "ms_per_frame_per_gpu": round(ms_step / B, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(fps / base_fps, 3),
            "dtype": "fp16",
            "data": "synthetic stereo pairs, seeded random-init weights",
            "config": {"model": args.model, "global_batch": world * B, "per_gpu_batch": B,
                       "resolution": f"{H}x{W}", "seq_len": None, "parallelism": f"dp{world}",
                       "iters": 32 if args.model == "raftstereo-sceneflow" else 7},
            "latency_b1": extra,
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
