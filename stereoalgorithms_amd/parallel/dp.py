"""Data-parallel frame sharding over torch.distributed (RCCL on ROCm, gloo on CPU).

The reference is single-GPU, batch 1 (RAFTStereo/include/TRTRAFTStereo.h:15); this is
the new multi-GPU capability required by BASELINE.json: one process per GPU, each rank owns a
contiguous shard of the stereo pairs, runs them through its own hipGraph-captured engine, and the
disparity maps are all-gathered over xGMI.  xGMI is point-to-point, so one large all-gather of the
whole shard (B x H x W fp32 per rank, ~9.8 MB at B = 8) is issued per step rather than per-frame
collectives.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist


def shard_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block [start, end) of `total` items for `rank`; remainders go to low ranks."""
    base, rem = divmod(total, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def shard_indices_round_robin(total: int, world: int, rank: int) -> list[int]:
    """Frame i goes to rank i % world (stream ordering for camera feeds)."""
    return list(range(rank, total, world))


class PendingGather:
    """Handle of an in-flight disparity all-gather (see DataParallelStereo.step_async).

    ``cloud`` is this rank's point-cloud shard [B,H,W,6] (XYZRGB, reprojected in the same frame graph) when the
    step was run with ``cloud=True``; it stays on the rank and is valid until the step two calls
    later reuses its slot."""

    def __init__(self, out: torch.Tensor, work, cloud: torch.Tensor | None = None):
        self.out, self._work, self.cloud = out, work, cloud

    def wait(self) -> torch.Tensor:
        """Make the current stream wait for the collective; returns the gathered [world*B,H,W] tensor."""
        if self._work is not None:
            self._work.wait()
            self._work = None
        return self.out


@dataclass
class DataParallelStereo:
    """One rank's view of a DP stereo job.

    ``step`` is the synchronous form (gathered result ordered after this step's frames).  ``step_async``
    is the pipelined form used by bench.py: the engine writes into one of two persistent send slots, the
    all-gather is issued with ``async_op=True`` so it runs on the process group's own stream (RCCL's
    internal HIP stream on GPU) while the NEXT step's frame graph runs on the compute stream, and the
    compute stream only waits for the collective that last used the slot it is about to overwrite.
    A gathered buffer stays valid until the step two calls later reuses its slot.

    ``gather_dtype=torch.float16`` halves the gathered bytes (0.61 MB per 480x640 frame instead of 1.23,
    SURVEY.md §5.8); fp16 keeps disparities below 256 px to within 1/8 px.

    ``cloud=True``: every rank also produces the point clouds of its own frames, as the reference does for each
    frame (RAFTStereo/src/TRTRAFTStereo.cpp:140-144: reprojection + copy-out inside its timed region).  The
    engine reprojects in the same frame graph; the cloud shard [B,H,W,6] stays on the rank (``last_cloud``,
    ``PendingGather.cloud``) -- 7.4 MB per 480x640 frame is 6x the disparity, so it is not all-gathered.
    ``gather_clouds_to_rank0`` collects them on rank 0 when a consumer needs them in one place.
    """
    engine: object  # anything with .run(left, right[, out=]) -> [B,H,W] and .batch
    world_size: int = 1
    rank: int = 0
    gather: bool = True
    slots: int = 2
    gather_dtype: torch.dtype | None = None
    force_gather: bool = False  # run the collective even at world size 1 (overlap traces on one GPU)
    cloud: bool = False  # also produce this rank's point clouds (engine needs its Q matrix)

    def __post_init__(self):
        self._out = None
        self._clouds: list = [None] * self.slots
        self.last_cloud = None
        self._cast: list = [None] * self.slots
        self._send: list = [None] * self.slots
        self._recv: list = [None] * self.slots
        self._work: list = [None] * self.slots
        self._i = 0

    def _run(self, left, right, slot, send):
        """engine.run into the slot's buffers -> (disparity [B,H,W], cloud [B,H,W,6] or None)."""
        if self.cloud:
            c = self._clouds[slot]
            disp, cl = self.engine.run(left, right, cloud=True, out=send, cloud_out=c)
            self._clouds[slot] = cl
            self.last_cloud = cl
            return disp, cl
        try:
            disp = self.engine.run(left, right, out=send) if send is not None else self.engine.run(left, right)
        except TypeError:  # engines without an ``out=`` argument
            disp = self.engine.run(left, right)
            if send is not None:
                disp = send.copy_(disp)
        return disp, None

    def step(self, left: torch.Tensor, right: torch.Tensor) -> torch.Tensor:
        """left/right: this rank's shard [B,H,W,3] u8 -> gathered disparity [world*B,H,W]
        (the rank's point clouds in ``last_cloud`` when ``cloud=True``)."""
        disp, _ = self._run(left, right, 0, None)
        if self.world_size == 1 or not self.gather:
            return disp
        if self.gather_dtype is not None:
            disp = disp.to(self.gather_dtype)
        return all_gather_disparity(disp, self.world_size, self._buffer(disp))

    def step_async(self, left: torch.Tensor, right: torch.Tensor) -> PendingGather:
        """Pipelined step: returns a PendingGather whose wait() yields the gathered disparity."""
        slot = self._i % self.slots
        self._i += 1
        if self._work[slot] is not None:  # WAR: the collective still reading/writing this slot
            self._work[slot].wait()
            self._work[slot] = None
        send = self._send[slot]
        disp, cl = self._run(left, right, slot, send)
        self._send[slot] = disp
        if not self.gather or (self.world_size == 1 and not self.force_gather):
            return PendingGather(disp, None, cl)
        if self.gather_dtype is not None and disp.dtype != self.gather_dtype:
            c = self._cast[slot]
            if c is None or c.shape != disp.shape or c.device != disp.device:
                c = self._cast[slot] = torch.empty(disp.shape, dtype=self.gather_dtype, device=disp.device)
            disp = c.copy_(disp)
        shape = (self.world_size * disp.shape[0],) + tuple(disp.shape[1:])
        recv = self._recv[slot]
        if recv is None or recv.shape != shape or recv.device != disp.device:
            recv = self._recv[slot] = torch.empty(shape, dtype=disp.dtype, device=disp.device)
        work = _all_gather_async(disp, self.world_size, recv)
        self._work[slot] = work
        return PendingGather(recv, work, cl)

    def flush(self):
        """Order every outstanding collective before the current stream's next work."""
        for i, w in enumerate(self._work):
            if w is not None:
                w.wait()
                self._work[i] = None

    def _buffer(self, disp):
        shape = (self.world_size * disp.shape[0],) + tuple(disp.shape[1:])
        if self._out is None or self._out.shape != shape or self._out.device != disp.device:
            self._out = torch.empty(shape, dtype=disp.dtype, device=disp.device)
        return self._out


def _all_gather_async(disp: torch.Tensor, world: int, out: torch.Tensor):
    if disp.is_cuda and dist.get_backend() == "nccl":
        return dist.all_gather_into_tensor(out, disp, async_op=True)
    return dist.all_gather(list(out.chunk(world, dim=0)), disp, async_op=True)


def all_gather_disparity(disp: torch.Tensor, world: int, out: torch.Tensor | None = None) -> torch.Tensor:
    """One all-gather of the whole shard (rank-major), RCCL/xGMI on GPU, gloo on CPU."""
    if out is None:
        out = torch.empty((world * disp.shape[0],) + tuple(disp.shape[1:]), dtype=disp.dtype, device=disp.device)
    if disp.is_cuda and dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(out, disp.contiguous())
    else:  # gloo lacks all_gather_into_tensor on older builds
        parts = list(out.chunk(world, dim=0))
        dist.all_gather(parts, disp.contiguous())
    return out


def gather_to_rank0(disp: torch.Tensor, world: int, rank: int):
    """Point-cloud style output: only rank 0 receives the full set."""
    parts = [torch.empty_like(disp) for _ in range(world)] if rank == 0 else None
    dist.gather(disp.contiguous(), parts, dst=0)
    return torch.cat(parts, 0) if rank == 0 else None


def gather_clouds_to_rank0(cloud: torch.Tensor, world: int, rank: int):
    """Every rank's point-cloud shard [B,H,W,6] -> [world*B,H,W,6] on rank 0 (None elsewhere); one collective.
    RCCL has no gather primitive over torch's all_gather_into_tensor path, so on GPU this is an all-gather whose
    result only rank 0 keeps (xGMI is point-to-point: the other ranks' receive traffic rides idle links)."""
    if world == 1:
        return cloud
    if cloud.is_cuda and dist.get_backend() == "nccl":
        out = torch.empty((world * cloud.shape[0],) + tuple(cloud.shape[1:]), dtype=cloud.dtype, device=cloud.device)
        dist.all_gather_into_tensor(out, cloud.contiguous())
        return out if rank == 0 else None
    return gather_to_rank0(cloud, world, rank)


class H2DPrefetcher:
    """Multi-buffered host->device input staging on a copy stream.

    ``prefetch(host_tensors)`` enqueues the pinned-host -> device copies of a FUTURE step on a side stream (the
    copy engine); ``next()`` hands out the oldest prefetched slot and makes the current stream wait for its copies.
    A slot is only overwritten once the compute stream has passed the step that read it (event recorded by the
    following ``next``).  Every step still copies its own inputs; only the overlap changes.

    Issue order matters on this hardware: streams share the GPU_MAX_HW_QUEUES = 4 hardware queues, and a copy's
    stream-ordering barrier sits in its queue behind whatever was enqueued there before it.  Copied "just in time"
    (``load``: copy step t, then run step t), the copy of step t lands behind the previous step's all-gather, which
    waits for the previous frame, and frame t then waits for the copy: the copy runs between frames.  Prefetched one
    step ahead (``prefetch`` of step t+1 BEFORE step t is enqueued; 3 slots), the copy only waits for the frame two
    steps back and runs under the current one (profiles/dp_overlap_r04.txt).
    """

    def __init__(self, host_tensors, device, slots: int = 3, stream=None):
        """``stream``: the copy stream to use (e.g. ``NativeStereoEngine.copy_stream``, so the data-parallel step
        adds no stream of its own); default a new stream."""
        self.device = torch.device(device)
        self.stream = stream if stream is not None else torch.cuda.Stream(self.device)
        self.slots = slots
        self.bufs = [[torch.empty_like(h, device=self.device) for h in host_tensors] for _ in range(slots)]
        # The caching allocator hands out blocks whose previous owner may still have work pending on
        # the allocating (current) stream; the copy stream writes them, so it first waits for that
        # stream (without this, a recycled block can be overwritten under a not-yet-run read).
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        self.freed = [None] * slots  # compute-stream event after the step that consumed the slot
        self.ready = [None] * slots  # copy-stream event after the slot's copies
        self._issued = 0  # slots handed to prefetch so far
        self._taken = 0  # slots handed out by next so far
        self._last = None

    def prefetch(self, host_tensors):
        """Enqueue the copies of a future step (at most ``slots - 1`` ahead of the consumer)."""
        if self._issued - self._taken >= self.slots - 1:
            raise RuntimeError("H2DPrefetcher: prefetch queue full (call next() first)")
        slot = self._issued % self.slots
        self._issued += 1
        with torch.cuda.stream(self.stream):
            if self.freed[slot] is not None:
                self.stream.wait_event(self.freed[slot])
            for d, h in zip(self.bufs[slot], host_tensors):
                d.copy_(h, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
            self.ready[slot] = ev

    def next(self):
        """Device buffers of the oldest prefetched step, ordered before the current stream's next work."""
        if self._taken >= self._issued:
            raise RuntimeError("H2DPrefetcher: next() without a prefetched step")
        cs = torch.cuda.current_stream(self.device)
        if self._last is not None:  # the previous slot is consumed by everything queued so far
            ev = torch.cuda.Event()
            ev.record(cs)
            self.freed[self._last] = ev
        slot = self._taken % self.slots
        self._taken += 1
        cs.wait_event(self.ready[slot])
        self._last = slot
        return self.bufs[slot]

    def load(self, host_tensors):
        """Just-in-time form: copy this step's inputs and hand them out."""
        self.prefetch(host_tensors)
        return self.next()


def _native_plan_load(path: str) -> int:
    """Merge a plan file into this process's tactic table (libstereo_amd.so, no device needed)."""
    from stereoalgorithms_amd import _native as N
    return int(N.dev().sa_conv_plan_load(str(path).encode()))


def build_engine_shared_plan(make_engine, world: int, rank: int, load_plan=None):
    """Build one engine per rank so that EVERY rank launches the tactics rank 0 tuned (ranks that
    tune independently pick different kernels on noisy timings, and the job's step time is the slowest rank's).

    Rank 0 builds first -- timing each conv shape -- and exports the entries its engine actually launched
    (``plan_export``, from the process plan: this works with plan files disabled too) while the other ranks wait in
    the broadcast of those bytes.  Each merges them into its own process tactic table (``load_plan``, default the
    native ``sa_conv_plan_load``), PINS the table (a stale plan file at the rank's own plan path can no longer override
    the broadcast entries when its engine loads it), and builds, finding every shape planned.  Bytes travel
    over the process group, not a shared file system, so this works across nodes.

    Returns ``(engine, digests)``: ``digests[r]`` is rank r's ``tactics_digest`` -- the (key, cfg, splitk) its frame
    graph launches -- or None when the engine cannot report one.  All equal = identical kernels on every rank."""
    import os
    import tempfile

    def digest_of(eng):
        d = getattr(eng, "tactics_digest", None)
        return d if isinstance(d, str) and d else None

    def export_bytes(eng):
        exp = getattr(eng, "plan_export", None)
        if exp is not None:
            fd, tmp = tempfile.mkstemp(suffix=".plan")
            os.close(fd)
            try:
                if exp(tmp) == 0:
                    with open(tmp, "rb") as f:
                        return f.read()
            finally:
                os.unlink(tmp)
        path = getattr(eng, "plan_path", "") or ""  # engines without an export: their plan file
        with open(path, "rb") if path and os.path.exists(path) else _empty() as f:
            return f.read()

    if world <= 1:
        eng = make_engine()
        return eng, [digest_of(eng)]
    box = [None]
    if rank == 0:
        eng = make_engine()
        box = [export_bytes(eng)]
    dist.broadcast_object_list(box, src=0)
    if rank != 0:
        data = box[0]
        if data:
            fd, tmp = tempfile.mkstemp(suffix=".plan")
            try:
                with os.fdopen(fd, "wb") as f:
                    f.write(data)
                (load_plan or _native_plan_load)(tmp)
            finally:
                os.unlink(tmp)
            if load_plan is None:
                _native_plan_pin(True)
        try:
            eng = make_engine()
        finally:
            if data and load_plan is None:
                _native_plan_pin(False)
    digests = [None] * world
    dist.all_gather_object(digests, digest_of(eng))
    return eng, digests


def _native_plan_pin(on: bool) -> None:
    from stereoalgorithms_amd import _native as N
    N.dev().sa_conv_plan_pin(1 if on else 0)


class _empty:
    """Context manager standing in for an absent plan file (read() -> b'')."""

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def read(self):
        return b""
