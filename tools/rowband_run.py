#!/usr/bin/env python3
"""Row-band sharded RAFT-Stereo on one frame (stereoalgorithms_amd/parallel/rowband.py), one rank per device:

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/rowband_run.py \\
        --model raftstereo-sceneflow --height 960 --width 1280 --iters 8 [--device cpu]

Every rank runs the fp32 oracle module on its band of rows (RCCL point-to-point halo exchange on GPUs, gloo on the
CPU); rank 0 gathers the bands, compares them with a single-device forward (--check) and prints one JSON line with
the band layout, the per-rank time and the max deviation.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="raftstereo-sceneflow")
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--check", action="store_true", help="compare with a single-device forward on rank 0")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    from stereoalgorithms_amd.models import raft_stereo as R
    from stereoalgorithms_amd.parallel.rowband import RowBands, gather_bands, raft_band_unit, raft_rowband_band

    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    if a.device == "cuda":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dev = torch.device("cpu")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = R.scale_heads(R.build(a.model, seed=0), 4.0, -0.3).to(dev)
        g = torch.Generator().manual_seed(5)
        left = (torch.rand(1, 3, a.height, a.width, generator=g) * 255).to(dev)
        right = torch.roll(left, -4, dims=3)
        bands = RowBands(a.height, world, raft_band_unit(m.cfg))
        b0, b1 = bands.band(rank)
        raft_rowband_band(m, left[:, :, b0:b1], right[:, :, b0:b1], bands, rank, iters=1)  # warm-up
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        band = raft_rowband_band(m, left[:, :, b0:b1], right[:, :, b0:b1], bands, rank, iters=a.iters)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        full = gather_bands(band, bands)
        times = [None] * world
        dist.all_gather_object(times, round(ms, 2))
        if rank == 0:
            rec = {"model": a.model, "frame": f"{a.height}x{a.width}", "iters": a.iters, "world": world,
                   "bands": [bands.band(r) for r in range(world)], "ms_per_rank": times,
                   "shape": list(full.shape), "finite": bool(torch.isfinite(full).all())}
            if a.check:
                with torch.no_grad():
                    _, ref = m(left, right, iters=a.iters)
                rec["max_abs_diff_vs_single"] = float((full - ref).abs().max())
                rec["mean_abs_ref"] = float(ref.abs().mean())
            print(json.dumps(rec), flush=True)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
