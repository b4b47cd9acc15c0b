"""Python handle on the native StereoEngine (csrc/runtime/engine.cpp).

One engine = one model on one GPU with a static memory plan and a captured whole-frame hipGraph.
``run`` works on torch CUDA tensors and launches on the current torch stream, so it composes with
torch.distributed (RCCL) collectives in the data-parallel path (``parallel.dp``).
"""
from __future__ import annotations

import ctypes as C
import sys

import numpy as np
import torch

from .. import _native as N

MODEL_PRESETS = (
    "raftstereo-sceneflow", "raftstereo-realtime",
    "crestereo-iter2", "crestereo-iter5", "crestereo-iter10",
    "hitnet-d400", "hitnet-xl", "fastacvnet-plus",
)


class _NativeHandle:
    """Owner of the native engine handle.  The engine holds one reference and every host_buffers() view holds
    another, so the native engine (whose pinned staging those views alias) is destroyed when the LAST of them goes:
    close() with views outstanding defers the free instead of leaving the views dangling."""

    def __init__(self, lib, h):
        self.lib, self.h = lib, h

    def destroy(self):
        if self.h:
            self.lib.sa_engine_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.destroy()
        except Exception:
            pass


class NativeStereoEngine:
    def __init__(self, model: str = "", weights: str | None = None, height: int = 480, width: int = 640,
                 batch: int = 1, iters: int = -1, device: int = 0, use_graph: bool = True, seed: int = 0):
        lib = N.require_native()
        self._lib = lib
        self.height, self.width, self.batch = height, width, batch
        self.device = torch.device("cuda", device)
        h = lib.sa_engine_create(model.encode(), (weights or "").encode(), height, width, batch, iters, device,
                                 int(use_graph), seed)
        if not h:
            raise RuntimeError(f"engine creation failed: {lib.sa_last_error().decode()}")
        self._h = h
        self._owner = _NativeHandle(lib, h)
        self.model = model
        self.has_q = False

    @property
    def _live(self):
        """The native handle; a closed engine raises instead of passing NULL to the C API (which would crash)."""
        if not getattr(self, "_h", None):
            raise RuntimeError("engine is closed")
        return self._h

    def close(self):
        """Release the engine.  The native engine is destroyed now unless host_buffers() views are still alive, in
        which case it goes with the last of them (the engine object itself is unusable either way)."""
        if getattr(self, "_h", None):
            self._h = None
            owner, self._owner = self._owner, None
            if sys.getrefcount(owner) <= 2:  # only this frame's reference: no views outstanding
                owner.destroy()

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def stage_times(self) -> list[tuple[str, float]]:
        """Per-stage device ms of the last frame (engine created with SA_STAGE_TIMES=1), e.g.
        [("encoders+corr", 1.2), ("gru_iterations", 11.0), ("network", 0.1), ("reproject", 0.05)]."""
        ms = (C.c_float * 16)()
        names = (C.c_char_p * 16)()
        n = self._lib.sa_engine_stage_times(self._live, ms, names, 16)
        if n < 0:
            raise RuntimeError(f"stage_times failed: {self._lib.sa_last_error().decode()}")
        return [(names[i].decode(), float(ms[i])) for i in range(n)]

    @property
    def device_bytes(self) -> int:
        return int(self._lib.sa_engine_device_bytes(self._live))

    @property
    def copy_stream(self) -> torch.cuda.ExternalStream:
        """The engine's side stream as a torch stream: idle outside graph capture, so callers stage their input
        copies there (parallel.dp.H2DPrefetcher) instead of creating a stream of their own.  The stream dies with
        the engine: free pinned host tensors that were copied on it BEFORE close() (torch's pinned-host allocator
        records an event on every stream that used a block when the block is freed)."""
        return torch.cuda.ExternalStream(self._lib.sa_engine_copy_stream(self._live), device=self.device)

    @property
    def main_stream(self) -> torch.cuda.ExternalStream:
        """The engine's own stream (where its frame graphs are captured and replayed) as a torch stream.  A caller
        that makes it current (``torch.cuda.set_stream``) runs frames without the cross-stream event pair a foreign
        caller stream needs, and adds no stream of its own: the data-parallel step then uses the engine stream, its
        copy stream and RCCL's stream (parallel.dp, bench.py)."""
        return torch.cuda.ExternalStream(self._lib.sa_engine_stream(self._live), device=self.device)

    @property
    def plan_path(self) -> str:
        """Tuned-plan cache file of this engine ('' when disabled: SA_PLAN_CACHE set, SA_PLAN_DIR='')."""
        return self._lib.sa_engine_plan_path(self._live).decode()

    @property
    def tactics_digest(self) -> str:
        """Digest of the tactics this engine's frame graph launches, from the process plan (not a file): the shapes it
        consulted with their (cfg, splitk) and the library build id.  Equal digests = identical kernels."""
        return self._lib.sa_engine_tactics_digest(self._live).decode()

    def plan_export(self, path: str) -> int:
        """Write this engine's plan entries to ``path`` (0 or errno): what a DP job's rank 0 broadcasts."""
        return int(self._lib.sa_engine_plan_export(self._live, str(path).encode()))

    @property
    def tuned_shapes(self) -> int:
        """Conv shapes this engine had to time at build (0 when its plan file covered everything)."""
        return int(self._lib.sa_engine_tuned_shapes(self._live))

    @property
    def plan_status(self) -> dict:
        """Tuned-plan cache at build: path, entries the file held (-1 absent, -2 written by another library build, -3
        not consulted), ``state`` (utils.plan.plan_state: absent / foreign-build / empty / loaded / not-consulted),
        save result (0 ok, errno of a failed write, -1 not attempted), the library build id and ``tactics``, the
        digest of the plan's tactic choices (utils.plan.tactic_digest: equal digests = identical kernels)."""
        from stereoalgorithms_amd.utils.plan import plan_state, tactic_digest
        ld, sv = C.c_int(0), C.c_int(0)
        self._lib.sa_engine_plan_status(self._live, C.byref(ld), C.byref(sv))
        return {"path": self.plan_path, "loaded": ld.value, "state": plan_state(ld.value), "saved": sv.value,
                "tuned_shapes": self.tuned_shapes, "build": self._lib.sa_plan_build_id().decode(),
                "tactics": tactic_digest(self.plan_path), "launched": self.tactics_digest}

    def nonzero_splitk_counters(self) -> int:
        """Diagnostic: split-K tile counters left non-zero (0 after every correctly ordered frame)."""
        return int(self._lib.sa_engine_nonzero_splitk_counters(self._live))

    def set_Q(self, Q):
        q = np.ascontiguousarray(np.asarray(Q, dtype=np.float32).reshape(16))
        N.check(self._lib.sa_engine_set_q(self._live, q.ctypes.data_as(C.c_void_p)), "set_Q")
        self.has_q = True

    def set_rectify_maps(self, map_left: np.ndarray, map_right: np.ndarray):
        ml = np.ascontiguousarray(map_left, dtype=np.float32)
        mr = np.ascontiguousarray(map_right, dtype=np.float32)
        assert ml.shape == (self.height, self.width, 2) and mr.shape == ml.shape
        N.check(self._lib.sa_engine_set_rectify_maps(self._live, ml.ctypes.data_as(C.c_void_p),
                                                     mr.ctypes.data_as(C.c_void_p)), "set_rectify_maps")

    def run(self, left: torch.Tensor, right: torch.Tensor, cloud: bool = False, rectify: bool = False,
            out: torch.Tensor | None = None, rectified: bool = False, cloud_out: torch.Tensor | None = None):
        """left/right: uint8 BGR [B,H,W,3] CUDA tensors -> disparity fp32 [B,H,W] (+cloud [B,H,W,6], written into
        ``cloud_out`` when given).  The cloud needs set_Q(); it is reprojected inside the frame graph."""
        b, h, w = self.batch, self.height, self.width
        assert left.shape == (b, h, w, 3) and left.dtype == torch.uint8 and left.is_cuda
        if cloud and not self.has_q:
            raise RuntimeError("point cloud requested but no Q matrix set (set_Q)")
        left, right = left.contiguous(), right.contiguous()
        disp = out if out is not None else torch.empty(b, h, w, dtype=torch.float32, device=left.device)
        pc = None
        if cloud:
            pc = cloud_out if cloud_out is not None else torch.empty(b, h, w, 6, dtype=torch.float32, device=left.device)
            assert pc.shape == (b, h, w, 6) and pc.dtype == torch.float32 and pc.is_contiguous()
        rl = torch.empty_like(left) if (rectify and rectified) else None
        rr = torch.empty_like(right) if (rectify and rectified) else None
        stream = C.c_void_p(torch.cuda.current_stream(left.device).cuda_stream)
        N.check(self._lib.sa_engine_run_device(
            self._live, C.c_void_p(left.data_ptr()), C.c_void_p(right.data_ptr()), C.c_void_p(disp.data_ptr()),
            C.c_void_p(pc.data_ptr() if pc is not None else 0), int(rectify), stream,
            C.c_void_p(rl.data_ptr() if rl is not None else 0), C.c_void_p(rr.data_ptr() if rr is not None else 0)),
            "engine run")
        res = [disp]
        if cloud:
            res.append(pc)
        if rectify and rectified:
            res += [rl, rr]
        return res[0] if len(res) == 1 else tuple(res)

    def host_buffers(self) -> dict:
        """The engine's pinned host staging as numpy views (valid while the engine lives, overwritten by the next
        run_host): ``left`` / ``right`` u8 [B,H,W,3], ``disp`` fp32 [B,H,W], ``cloud`` fp32 [B,H,W,6].  Passing them to
        run_host (inputs filled in place, ``out`` / ``cloud_out``) skips the pageable <-> pinned copies."""
        b, h, w = self.batch, self.height, self.width
        ptrs = [C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()]
        self._lib.sa_engine_host_buffers(self._live, *[C.byref(p) for p in ptrs])

        def view(p, shape, ctype, dtype):
            n = int(np.prod(shape))
            arr = (ctype * n).from_address(p.value)
            arr._sa_owner = self._owner  # the numpy view's base keeps the native engine alive (see close)
            return np.ctypeslib.as_array(arr).view(dtype).reshape(shape)
        return {"left": view(ptrs[0], (b, h, w, 3), C.c_uint8, np.uint8),
                "right": view(ptrs[1], (b, h, w, 3), C.c_uint8, np.uint8),
                "disp": view(ptrs[2], (b, h, w), C.c_float, np.float32),
                "cloud": view(ptrs[3], (b, h, w, 6), C.c_float, np.float32)}

    def host_times(self) -> dict:
        """Timing split of the last run_host in ms (device-side entries need SA_HOST_TIMES=1 at creation; h2d is -1
        when the frame graph read the inputs itself over PCIe, zero-copy inputs, and graph includes that read)."""
        t = (C.c_float * 8)()
        n = self._lib.sa_engine_host_times(self._live, t, 8)
        keys = ("total", "input_copies", "enqueue", "wait_and_output_copies", "h2d", "graph", "d2h")
        return {k: round(float(t[i]), 4) for i, k in enumerate(keys[:n])}

    def run_host(self, left: np.ndarray, right: np.ndarray, cloud: bool = True, rectify: bool = False,
                 out: np.ndarray | None = None, cloud_out: np.ndarray | None = None):
        """The reference's timed region: host BGR in, host disparity (+cloud) out.  ``out`` / ``cloud_out``: caller
        arrays to write (the reference's caller-allocated point cloud, RAFTStereo/test/main.cpp:20), e.g. the
        engine's own pinned buffers from host_buffers(); fresh arrays otherwise.

        Caller arrays passed on two consecutive frames are mapped into the GPU and stay mapped until another array is
        passed for that role or the engine is closed (sa_engine_run_host): keep them alive that long.  Arrays this
        wrapper would create per call -- fresh outputs, contiguous / uint8 copies of the inputs -- never reach the
        engine: they go through its pinned staging (a freed temporary re-allocated at the same address would
        otherwise hit a stale mapping)."""
        b, h, w = self.batch, self.height, self.width
        hb = None
        ins = []
        for name, img in (("left", left), ("right", right)):
            a = np.asarray(img)
            if a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"] and a.size == b * h * w * 3:
                ins.append(a.reshape(b, h, w, 3))
            else:  # a temporary would be made: stage it in the pinned buffer instead
                hb = hb if hb is not None else self.host_buffers()
                hb[name][...] = np.asarray(a, dtype=np.uint8).reshape(b, h, w, 3)
                ins.append(hb[name])
        left, right = ins
        fresh_out = out is None or (cloud and cloud_out is None)
        if fresh_out:
            hb = hb if hb is not None else self.host_buffers()
        disp = out if out is not None else hb["disp"]
        assert disp.shape == (b, h, w) and disp.dtype == np.float32 and disp.flags["C_CONTIGUOUS"]
        pc = None
        if cloud:
            pc = cloud_out if cloud_out is not None else hb["cloud"]
            assert pc.shape == (b, h, w, 6) and pc.dtype == np.float32 and pc.flags["C_CONTIGUOUS"]
        N.check(self._lib.sa_engine_run_host(self._live, left.ctypes.data_as(C.c_void_p), right.ctypes.data_as(C.c_void_p),
                                             disp.ctypes.data_as(C.c_void_p),
                                             pc.ctypes.data_as(C.c_void_p) if pc is not None else None,
                                             int(rectify)), "engine run_host")
        if out is None:
            disp = disp.copy()
        if cloud and cloud_out is None:
            pc = pc.copy()
        if hb is not None:  # inputs staged in the pinned buffers are overwritten by the next call
            left = left.copy() if left is hb["left"] else left
            right = right.copy() if right is hb["right"] else right
        return (disp, pc, left, right) if cloud else (disp, left, right)

    def low_res_flow(self) -> int:
        n = C.c_int(0)
        self._lib.sa_engine_aux_output(self._live, C.byref(n))
        return n.value
