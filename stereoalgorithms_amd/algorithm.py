"""Python face of the reference's per-model facade (RAFTStereo/src/RAFTStereoAlgorithm.cpp and siblings), over the
native ``sa::StereoAlgorithm`` (csrc/api/algorithm.cpp) through the flat C API:

    from stereoalgorithms_amd.algorithm import StereoAlgorithm
    with StereoAlgorithm("raftstereo-realtime", "StereoCalibration.yml", gpu=0) as alg:
        disparity, cloud = alg.run(left_bgr, right_bgr)      # numpy u8 [H, W, 3] in, fp32 [H, W] / [H, W, 6] out

Initialize reads the OpenCV-format calibration YAML, builds the engine and uploads the rectification maps and Q
once; ``run`` is the reference's timed region (rectify on the GPU, network, reprojection, copies back).  Like the
reference, the input arrays receive their rectified versions when ``rectify`` is set.  ``model`` is a preset name,
a ``.safetensors`` weights file or ``preset@weights`` (sa/algorithm.h).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N


class StereoAlgorithm:
    def __init__(self, model: str, calibration: str, gpu: int = 0, default_preset: str = ""):
        lib = N.require_native()
        self._lib = lib
        h = lib.sa_algorithm_create(model.encode(), gpu, calibration.encode(), default_preset.encode())
        if not h:
            raise RuntimeError(f"StereoAlgorithm initialize failed: {lib.sa_last_error().decode()}")
        self._h = h
        r, c = C.c_int(0), C.c_int(0)
        N.check(lib.sa_algorithm_frame_size(h, C.byref(r), C.byref(c)), "sa_algorithm_frame_size")
        self.height, self.width = r.value, c.value

    def run(self, left: np.ndarray, right: np.ndarray, rectify: bool = True, cloud: bool = True):
        """left / right: u8 BGR [H, W, 3] C-contiguous (rectified in place when ``rectify``).  Returns (disparity
        fp32 [H, W], point cloud fp32 [H, W, 6] or None)."""
        if self._h is None:
            raise RuntimeError("StereoAlgorithm is released")
        shape = (self.height, self.width, 3)
        for name, img in (("left", left), ("right", right)):
            if img.dtype != np.uint8 or img.shape != shape or not img.flags["C_CONTIGUOUS"] or not img.flags["WRITEABLE"]:
                raise ValueError(f"{name}: expected a writeable C-contiguous uint8 array of shape {shape}")
        disp = np.empty((self.height, self.width), np.float32)
        pc = np.empty((self.height, self.width, 6), np.float32) if cloud else None
        rc = self._lib.sa_algorithm_run(self._h, left.ctypes.data_as(C.c_void_p), right.ctypes.data_as(C.c_void_p),
                                        self.height, self.width, disp.ctypes.data_as(C.c_void_p),
                                        pc.ctypes.data_as(C.c_void_p) if pc is not None else None, int(rectify))
        if rc != 0:
            raise RuntimeError(f"StereoAlgorithm run failed: {self._lib.sa_last_error().decode()}")
        return disp, pc

    @property
    def last_ms(self) -> float:
        """Wall time of the last run's timed region (ms)."""
        if self._h is None:
            raise RuntimeError("StereoAlgorithm is released")
        return float(self._lib.sa_algorithm_last_ms(self._h))

    def close(self):
        if getattr(self, "_h", None):
            self._lib.sa_algorithm_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass
