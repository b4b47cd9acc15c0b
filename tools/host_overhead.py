#!/usr/bin/env python3
"""Where the host-side time of the reference's timed region goes.

For each preset, batch-1 run_host latency (RAFTStereo/src/TRTRAFTStereo.cpp:119-146: input staging, H2D, network,
reprojection, D2H of disparity + point cloud) is measured three ways:
  fresh    new numpy output arrays every frame (first-touch page faults inside the timed region)
  prealloc caller arrays allocated once, as the reference's demo does (RAFTStereo/test/main.cpp:20)
  pinned   the engine's own pinned staging (host_buffers()): no pageable <-> pinned copies
and split with the engine's host timers (input copies / enqueue / wait + output copies) and, with SA_HOST_TIMES=1,
the device-side H2D / graph / D2H times of the same frames.
Usage (GPU box): SA_HOST_TIMES=1 python tools/host_overhead.py [--presets a,b] [--frames 30]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import stereoalgorithms_amd  # noqa: E402,F401


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--presets", default="raftstereo-realtime,hitnet-d400,fastacvnet-plus,raftstereo-sceneflow")
    ap.add_argument("--frames", type=int, default=30)
    args = ap.parse_args()
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.utils.synthetic import batch_pairs
    H, W = 480, 640
    Q = np.array([[1, 0, 0, -W / 2], [0, 1, 0, -H / 2], [0, 0, 0, 500.0], [0, 0, 1 / 60.0, 0]], np.float32)
    l, r = batch_pairs(1, H, W, seed=0)
    for preset in args.presets.split(","):
        e = NativeStereoEngine(preset, None, H, W, batch=1, seed=0)
        e.set_Q(Q)
        hb = e.host_buffers()
        disp_pre = np.empty((1, H, W), np.float32)
        cloud_pre = np.empty((1, H, W, 6), np.float32)
        rec = {"preset": preset}
        for mode in ("fresh", "prealloc", "pinned"):
            def once():
                if mode == "fresh":
                    return e.run_host(l, r, cloud=True)
                if mode == "prealloc":
                    return e.run_host(l, r, cloud=True, out=disp_pre, cloud_out=cloud_pre)
                hb["left"][...] = l  # the camera writes its frame into pinned memory (outside the timed region)
                hb["right"][...] = r
                t = time.perf_counter()
                e.run_host(hb["left"], hb["right"], cloud=True, out=hb["disp"], cloud_out=hb["cloud"])
                return time.perf_counter() - t
            for _ in range(5):
                once()
            ts, parts = [], []
            for _ in range(args.frames):
                t = time.perf_counter()
                dt = once()
                ts.append((dt if mode == "pinned" else time.perf_counter() - t) * 1e3)
                parts.append(e.host_times())
            ts = np.array(ts)
            mean_parts = {k: round(float(np.mean([p[k] for p in parts])), 4) for k in parts[0]}
            rec[mode] = {"mean_ms": round(float(ts.mean()), 4), "p50_ms": round(float(np.median(ts)), 4),
                         "split_ms": mean_parts}
        # correctness of the zero-copy path: same disparity as the copying path
        d1, c1, _, _ = e.run_host(l, r, cloud=True)
        hb["left"][...] = l
        hb["right"][...] = r
        e.run_host(hb["left"], hb["right"], cloud=True, out=hb["disp"], cloud_out=hb["cloud"])
        rec["pinned_matches"] = bool(np.array_equal(d1, hb["disp"]) and np.array_equal(c1, hb["cloud"], equal_nan=True))
        print(json.dumps(rec), flush=True)
        e.close()


if __name__ == "__main__":
    main()
