"""Row-band sharding of one RAFT-Stereo frame (parallel/rowband.py): gloo process groups of 2 and 3
ranks on the CPU, each rank running the unchanged oracle module on its band of rows with halo exchange, must
reproduce the single-process forward; plus the band geometry on its own."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from stereoalgorithms_amd.parallel.rowband import RowBands, raft_band_unit


def test_band_geometry():
    b = RowBands(480, 4, 16)
    bands = [b.band(r) for r in range(4)]
    assert bands[0][0] == 0 and bands[-1][1] == 480
    assert all(x[1] == y[0] for x, y in zip(bands, bands[1:]))
    assert all((e - s) % 16 == 0 and e > s for s, e in bands)
    assert max(e - s for s, e in bands) - min(e - s for s, e in bands) <= 16
    with pytest.raises(ValueError):
        RowBands(100, 2, 16)
    with pytest.raises(ValueError):
        RowBands(32, 3, 16)
    from stereoalgorithms_amd.models.raft_stereo import PRESETS
    assert raft_band_unit(PRESETS["raftstereo-sceneflow"]) == 16
    assert raft_band_unit(PRESETS["raftstereo-realtime"]) == 16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, preset, H, W, iters, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    from datetime import timedelta
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=120))
    try:
        from stereoalgorithms_amd.models import raft_stereo as R
        from stereoalgorithms_amd.parallel.rowband import RowBands, gather_bands, raft_band_unit, raft_rowband_forward
        m = R.scale_heads(R.build(preset, seed=0), 4.0, -0.3)
        g = torch.Generator().manual_seed(77)
        left = torch.rand(1, 3, H, W, generator=g) * 255
        right = torch.roll(left, -3, dims=3) * 0.9 + torch.rand(1, 3, H, W, generator=g) * 25
        band, (a, b) = raft_rowband_forward(m, left, right, iters=iters)
        full = gather_bands(band, RowBands(H, world, raft_band_unit(m.cfg)))
        if rank == 0:
            with torch.no_grad():
                _, ref = m(left, right, iters=iters)
            err = (full - ref).abs().max().item()
            q.put((rank, err, ref.abs().mean().item(), tuple(full.shape)))
        else:
            q.put((rank, 0.0, 0.0, (b - a,)))
    except Exception as e:  # report instead of leaving the parent waiting on the queue
        q.put((rank, f"{type(e).__name__}: {e}", 0.0, ()))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("preset,world,H,W,iters", [
    ("raftstereo-sceneflow", 2, 64, 64, 3),
    ("raftstereo-sceneflow", 3, 96, 64, 2),
    ("raftstereo-realtime", 2, 64, 128, 3),
])
def test_raft_rowband_matches_single_process(preset, world, H, W, iters):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, preset, H, W, iters, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, err, mag, shape = q.get(timeout=300)
        res[r] = (err, mag, shape)
    for p in procs:
        p.join(timeout=60)
    assert not any(isinstance(v[0], str) for v in res.values()), res
    print(f"{preset} world {world}: max |band - single| {res[0][0]:.3e}, mean |flow_up| {res[0][1]:.3f}")
    err, mag, shape = res[0]
    assert shape == (1, 1, H, W)
    assert mag > 0.05, "degenerate reference output"
    assert err < 1e-4 * max(1.0, mag), res  # fp32 summation order only
