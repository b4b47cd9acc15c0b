"""Data-parallel frame sharding (parallel/dp.py) on CPU: gloo process groups, world sizes 2 and 4,
a stand-in engine with the native engine's run() contract.  The RCCL path is the same code with
the nccl backend (bench.py on GPUs)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from stereoalgorithms_amd.parallel import dp


def test_shard_range_covers_all_frames():
    for total in (1, 7, 64, 65):
        for world in (1, 2, 3, 8):
            spans = [dp.shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def test_round_robin_shards_partition():
    got = sorted(i for r in range(3) for i in dp.shard_indices_round_robin(10, 3, r))
    assert got == list(range(10))


Q = [[1, 0, 0, -4.0], [0, 1, 0, -3.0], [0, 0, 0, 500.0], [0, 0, 1 / 60.0, 0]]


class FakeEngine:
    """Deterministic per-frame 'disparity' = mean of the left image + frame marker; point clouds with the
    native engine's reprojection contract."""

    def __init__(self, batch, h, w):
        self.batch, self.height, self.width = batch, h, w

    def run(self, left, right, cloud=False, out=None, cloud_out=None):
        from stereoalgorithms_amd.utils.geometry import reproject_cloud_torch
        d = (left.float().mean(-1) - right.float().mean(-1)).contiguous()
        if out is not None:
            d = out.copy_(d)
        if not cloud:
            return d
        c = reproject_cloud_torch(d, left, Q)
        if cloud_out is not None:
            c = cloud_out.copy_(c)
        return d, c


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, H, W, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(1234)
        all_l = torch.randint(0, 255, (world * B, H, W, 3), generator=g, dtype=torch.uint8)
        all_r = torch.randint(0, 255, (world * B, H, W, 3), generator=g, dtype=torch.uint8)
        s, e = dp.shard_range(world * B, world, rank)
        eng = FakeEngine(B, H, W)
        step = dp.DataParallelStereo(eng, world_size=world, rank=rank)
        out = step.step(all_l[s:e], all_r[s:e])
        ref = eng.run(all_l, all_r)
        ok = out.shape == (world * B, H, W) and torch.equal(out, ref)
        r0 = dp.gather_to_rank0(eng.run(all_l[s:e], all_r[s:e]), world, rank)
        if rank == 0:
            ok = ok and torch.equal(r0, ref)
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_dp_allgather_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 2, 6, 8, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(res[r] for r in range(world)), res


def _worker_async(rank, world, port, B, H, W, steps, q, gdt=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = FakeEngine(B, H, W)
        step = dp.DataParallelStereo(eng, world_size=world, rank=rank, gather_dtype=gdt)
        ok = True
        pending = []
        for t in range(steps):  # keep two steps in flight, check each gathered result a step late
            g = torch.Generator().manual_seed(100 + t)
            all_l = torch.randint(0, 255, (world * B, H, W, 3), generator=g, dtype=torch.uint8)
            all_r = torch.randint(0, 255, (world * B, H, W, 3), generator=g, dtype=torch.uint8)
            s, e = dp.shard_range(world * B, world, rank)
            ref = eng.run(all_l, all_r)
            pending.append((step.step_async(all_l[s:e], all_r[s:e]), ref if gdt is None else ref.to(gdt)))
            if len(pending) == 2:
                h, ref = pending.pop(0)
                ok = ok and torch.equal(h.wait(), ref)
        for h, ref in pending:
            ok = ok and torch.equal(h.wait(), ref)
        step.flush()
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("gdt", [None, torch.float16])
def test_dp_pipelined_allgather_gloo(gdt):
    """step_async: ping-pong send/recv slots, collective of step t in flight during step t+1
    (fp32 gather, and the fp16 gather option)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_async, args=(r, world, port, 2, 6, 8, 5, q, gdt)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(res[r] for r in range(world)), res


def _worker_cloud(rank, world, port, B, H, W, steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from stereoalgorithms_amd.utils.geometry import reproject_cloud_torch
        eng = FakeEngine(B, H, W)
        step = dp.DataParallelStereo(eng, world_size=world, rank=rank, cloud=True)
        ok = True
        for t in range(steps):
            g = torch.Generator().manual_seed(200 + t)
            all_l = torch.randint(0, 255, (world * B, H, W, 3), generator=g, dtype=torch.uint8)
            all_r = torch.randint(0, 255, (world * B, H, W, 3), generator=g, dtype=torch.uint8)
            s, e = dp.shard_range(world * B, world, rank)
            h = step.step_async(all_l[s:e], all_r[s:e])
            disp_all = h.wait()
            ref_disp = eng.run(all_l, all_r)
            # every rank keeps exactly its own frames' clouds [B,H,W,6] (XYZ from Q, RGB from the left image)
            ref_cloud = reproject_cloud_torch(ref_disp[s:e], all_l[s:e], Q)
            ok = ok and h.cloud.shape == (B, H, W, 6) and torch.allclose(h.cloud, ref_cloud, rtol=0, atol=0, equal_nan=True)
            ok = ok and torch.equal(disp_all, ref_disp) and step.last_cloud is h.cloud
            full = dp.gather_clouds_to_rank0(h.cloud, world, rank)
            if rank == 0:
                ok = ok and torch.allclose(full, reproject_cloud_torch(ref_disp, all_l, Q), rtol=0, atol=0, equal_nan=True)
            else:
                ok = ok and full is None
        step.flush()
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_dp_point_clouds_per_rank_gloo():
    """SURVEY §5.8 / VERDICT r2: each rank reprojects its own shard ([B,H,W,6] kept local), disparity is
    all-gathered, and gather_clouds_to_rank0 assembles the job's clouds on rank 0 on request."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_cloud, args=(r, world, port, 2, 6, 8, 3, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(res[r] for r in range(world)), res


class _TunedEngine:
    """Stand-in for an engine build's tactic selection: shapes missing from the process's plan table are 'timed'
    with rank-dependent noise (seeded by rank), i.e. independent tuning picks different tactics on every rank; the
    chosen plan is saved to this rank's own plan path (as the native engine saves <stem>_b8_..._gfx950.plan)."""
    table: dict = {}
    SHAPES = [f"gfx950|{n},120,160,384|k3x3|shape{i}" for i, n in enumerate((1, 8, 8, 1, 8, 2))]

    def __init__(self, plan_dir, rank):
        import random
        rng = random.Random(1000 + 17 * rank)
        self.tuned_shapes = 0
        for k in self.SHAPES:
            if k not in self.table:
                self.table[k] = (rng.choice([4, 10, 26, 28]), rng.choice([0, 1]), round(rng.uniform(20, 300), 2))
                self.tuned_shapes += 1
        d = os.path.join(plan_dir, f"rank{rank}")
        os.makedirs(d, exist_ok=True)
        self.plan_path = os.path.join(d, "raftstereo-sceneflow_seed0_b8_480x640_it-1_gfx950.plan")
        with open(self.plan_path, "w") as f:
            f.write("# sa-plan build=00000000feedbeef\n")
            for k in self.SHAPES:
                cfg, sk, us = self.table[k]
                f.write(f"{k} {cfg} {sk} {us}\n")


    @property
    def tactics_digest(self):
        """What the native engine reports: the (key, cfg, splitk) its graph launches, from the in-process table."""
        import hashlib
        h = hashlib.sha256()
        for k in sorted(self.SHAPES):
            cfg, sk, _ = self.table[k]
            h.update(f"{k} {cfg} {sk}\n".encode())
        return h.hexdigest()[:16]


def _fake_plan_load(path):
    from stereoalgorithms_amd.utils.plan import read_plan
    _, entries = read_plan(path)
    for e in entries:
        _TunedEngine.table[e.key] = (e.cfg, e.splitk, e.us)
    return len(entries)


def _worker_plan(rank, world, port, plan_dir, shared, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if shared:
            eng, digests = dp.build_engine_shared_plan(lambda: _TunedEngine(plan_dir, rank), world, rank,
                                                       load_plan=_fake_plan_load)
        else:
            from stereoalgorithms_amd.utils.plan import tactic_digest
            eng = _TunedEngine(plan_dir, rank)
            digests = [None] * world
            dist.all_gather_object(digests, tactic_digest(eng.plan_path))
        with open(eng.plan_path, "rb") as f:
            data = f.read()
        q.put((rank, (digests, eng.tuned_shapes, data)))
    finally:
        dist.destroy_process_group()


def _run_plan_job(world, tmp_path, shared):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_plan, args=(r, world, port, str(tmp_path), shared, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("world", [2, 4])
def test_dp_ranks_share_rank0_plan_gloo(world, tmp_path):
    """rank 0 tunes and every other rank builds from rank 0's plan bytes (broadcast over the
    process group), so all ranks' plan files are byte-identical, their tactic digests agree, and no rank but 0
    times a shape.  Negative control: independent tuning (rank-seeded timing noise) gives different plans."""
    res = _run_plan_job(world, tmp_path / "shared", shared=True)
    digests0 = res[0][0]
    assert len(set(digests0)) == 1 and digests0[0] is not None, digests0
    assert all(res[r][0] == digests0 for r in range(world))
    assert res[0][1] == len(_TunedEngine.SHAPES)
    assert all(res[r][1] == 0 for r in range(1, world)), {r: res[r][1] for r in res}
    assert all(res[r][2] == res[0][2] for r in range(world))
    indep = _run_plan_job(world, tmp_path / "indep", shared=False)
    assert len(set(indep[0][0])) > 1, "control: independently tuned ranks should disagree"
