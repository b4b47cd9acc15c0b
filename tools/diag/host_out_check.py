#!/usr/bin/env python3
"""run_host output paths of one engine, checked against each other (GPU):  python3 tools/diag/host_out_check.py
[--model raftstereo-sceneflow] [--buffers empty|full] -- copy path (fresh arrays each frame), the engine's pinned
zero-copy buffers, and reused caller buffers (zero-copy when SA_HOST_REGISTER=1).  Prints one line per path."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="raftstereo-sceneflow")
    ap.add_argument("--buffers", default="empty", choices=["empty", "full"])
    ap.add_argument("--order", default="copy,pinned,caller")
    a = ap.parse_args()
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    from stereoalgorithms_amd.utils.synthetic import batch_pairs
    Q = np.array([[1, 0, 0, -320.0], [0, 1, 0, -240.0], [0, 0, 0, 500.0], [0, 0, 1 / 60.0, 0]], np.float32)
    e = NativeStereoEngine(a.model, None, 480, 640, batch=1, device=0)
    e.set_Q(Q)
    l, r = batch_pairs(1, 480, 640, seed=3)
    res = {}
    for path in a.order.split(","):
        if path == "copy":
            d, c, _, _ = e.run_host(l, r, cloud=True)
            res[path] = (d.copy(), c.copy())
        elif path == "pinned":
            hb = e.host_buffers()
            hb["left"][...] = l
            hb["right"][...] = r
            for _ in range(3):
                e.run_host(hb["left"], hb["right"], cloud=True, out=hb["disp"], cloud_out=hb["cloud"])
            res[path] = (hb["disp"].copy(), hb["cloud"].copy())
            hb = None
        else:
            mk = np.empty if a.buffers == "empty" else (lambda s, t: np.full(s, -3.0, t))
            d, c = mk((1, 480, 640), np.float32), mk((1, 480, 640, 6), np.float32)
            for _ in range(3):
                e.run_host(l, r, cloud=True, out=d, cloud_out=c)
            res[path] = (d.copy(), c.copy())
        ref = res[a.order.split(",")[0]]
        ok = np.array_equal(res[path][0], ref[0]) and np.array_equal(res[path][1], ref[1], equal_nan=True)
        print(f"{a.model} {path}: {'ok' if ok else 'MISMATCH'} (register={os.environ.get('SA_HOST_REGISTER', '0')})",
              flush=True)
        if not ok:
            return 1
    e.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
