"""Batch-1 frame latency (graph replay + the reference's host timed region) for the RAFT presets; run under
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 / 1 to price the packet-capture path."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import stereoalgorithms_amd  # noqa: E402,F401
import numpy as np  # noqa: E402
import torch  # noqa: E402

from stereoalgorithms_amd.models.engine import NativeStereoEngine  # noqa: E402
from stereoalgorithms_amd.utils.synthetic import batch_pairs  # noqa: E402

l, r = batch_pairs(1, 480, 640, seed=1)
for preset in ("raftstereo-realtime", "raftstereo-sceneflow", "hitnet-d400"):
    e = NativeStereoEngine(preset, None, 480, 640, batch=1)
    lt, rt = torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()
    for _ in range(5):
        e.run(lt, rt)
    torch.cuda.synchronize()
    n = 50
    t0 = time.perf_counter()
    for _ in range(n):
        e.run(lt, rt)
    torch.cuda.synchronize()
    dev = (time.perf_counter() - t0) / n * 1e3
    ts = []
    for _ in range(20):
        t1 = time.perf_counter()
        e.run_host(l, r, cloud=True)
        ts.append((time.perf_counter() - t1) * 1e3)
    print(f"{preset:22s} packet_capture={os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE')}  back-to-back "
          f"{dev:.3f} ms/frame  host timed region p50 {np.median(ts):.3f} ms", flush=True)
    e.close()
