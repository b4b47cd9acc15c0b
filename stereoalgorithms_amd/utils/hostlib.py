"""ctypes bindings for libstereo_host.so (CPU only): calibration files, rectification math,
image I/O, colour maps, point clouds.  Importable without a GPU or torch.

Reference parity: ReadObjectYml / RectifyImage (RAFTStereo/src/RAFTStereoAlgorithm.cpp:79-126),
Stereo_Calibration.cpp:162-179 (stereoRectify + YAML), demo output (RAFTStereo/test/main.cpp:31-39,
CREStereo/test/main.cpp:7-24).
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

LIBDIR = Path(__file__).resolve().parent.parent / "lib"
_lib = None

_d = C.POINTER(C.c_double)
_f = C.POINTER(C.c_float)
_u8 = C.POINTER(C.c_uint8)
_i = C.POINTER(C.c_int)

MAT_KEYS = ("intrinsic_left", "distCoeffs_left", "intrinsic_right", "distCoeffs_right", "R", "T", "R_L", "R_R",
            "P1", "P2", "Q")


def lib():
    global _lib
    if _lib is None:
        path = LIBDIR / "libstereo_host.so"
        if not path.exists():
            raise RuntimeError(f"{path} not built — run `python -m stereoalgorithms_amd._build`")
        L = C.CDLL(str(path))
        sig = {
            "sa_host_version": (C.c_char_p, []),
            "sa_host_free": (None, [C.c_void_p]),
            "sa_imread": (C.c_void_p, [C.c_char_p, C.c_int, _i, _i, _i]),
            "sa_imwrite": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
            "sa_heatmap": (C.c_int, [_f, C.c_int, C.c_int, _u8]),
            "sa_colormap_jet": (C.c_int, [_u8, C.c_int, _u8]),
            "sa_bgr2gray": (C.c_int, [_u8, C.c_int, C.c_int, _u8]),
            "sa_write_pointcloud": (C.c_int, [C.c_char_p, _f, C.c_long]),
            "sa_calib_new": (C.c_void_p, []),
            "sa_calib_load": (C.c_void_p, [C.c_char_p]),
            "sa_calib_free": (None, [C.c_void_p]),
            "sa_calib_save": (C.c_int, [C.c_void_p, C.c_char_p]),
            "sa_calib_get": (C.c_int, [C.c_void_p, C.c_char_p, _d, C.c_int, _i, _i]),
            "sa_calib_set": (C.c_int, [C.c_void_p, C.c_char_p, _d, C.c_int, C.c_int]),
            "sa_calib_get_roi": (C.c_int, [C.c_void_p, _i]),
            "sa_calib_set_roi": (C.c_int, [C.c_void_p, _i]),
            "sa_calib_rectify_maps": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _f, _f, C.c_int]),
            "sa_calib_stereo_rectify": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_int]),
            "sa_undistort_points": (C.c_int, [_d, _d, C.c_int, _d, _d, C.c_int, C.c_int, _d, C.c_int, _d]),
            "sa_project_points": (C.c_int, [_d, C.c_int, _d, _d, _d, _d, C.c_int, _d]),
            "sa_rodrigues": (C.c_int, [_d, _d]),
            "sa_rodrigues_inv": (C.c_int, [_d, _d]),
            "sa_remap_u8_cpu": (C.c_int, [_u8, C.c_int, C.c_int, C.c_int, _f, _u8]),
            "sa_reproject_cpu": (C.c_int, [_f, C.c_int, C.c_int, _d, _f]),
            "sa_find_chessboard": (C.c_int, [_u8, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _d]),
            "sa_stereo_calibrate_images": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_double, C.c_int, C.c_void_p,
                                                     _d]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name, None)
            if fn is not None:
                fn.restype, fn.argtypes = res, args
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t) if a is not None else None


def _f64(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float64)


# ------------------------------------------------------------------------------------------ images
def imread(path, grayscale: bool = False) -> np.ndarray | None:
    """cv::imread: HxWx3 BGR uint8 (or HxW grey)."""
    h, w, c = C.c_int(), C.c_int(), C.c_int()
    ptr = lib().sa_imread(str(path).encode(), int(grayscale), C.byref(h), C.byref(w), C.byref(c))
    if not ptr:
        return None
    n = h.value * w.value * c.value
    out = np.frombuffer((C.c_uint8 * n).from_address(ptr), dtype=np.uint8).copy()
    lib().sa_host_free(ptr)
    return out.reshape(h.value, w.value, c.value) if c.value > 1 else out.reshape(h.value, w.value)


def imwrite(path, img: np.ndarray, quality: int = 95) -> bool:
    img = np.ascontiguousarray(img)
    depth = {np.dtype(np.uint8): 0, np.dtype(np.float32): 5, np.dtype(np.float64): 6}[img.dtype]
    h, w = img.shape[:2]
    c = 1 if img.ndim == 2 else img.shape[2]
    return lib().sa_imwrite(str(path).encode(), img.ctypes.data_as(C.c_void_p), h, w, c, depth, quality) == 0


def heatmap(disp: np.ndarray) -> np.ndarray:
    disp = np.ascontiguousarray(disp, dtype=np.float32)
    out = np.empty(disp.shape + (3,), np.uint8)
    lib().sa_heatmap(_p(disp, _f), disp.shape[0], disp.shape[1], _p(out, _u8))
    return out


def colormap_jet(u8: np.ndarray) -> np.ndarray:
    u8 = np.ascontiguousarray(u8, dtype=np.uint8)
    out = np.empty(u8.shape + (3,), np.uint8)
    lib().sa_colormap_jet(_p(u8, _u8), u8.size, _p(out, _u8))
    return out


def bgr2gray(img: np.ndarray) -> np.ndarray:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    out = np.empty(img.shape[:2], np.uint8)
    lib().sa_bgr2gray(_p(img, _u8), img.shape[0], img.shape[1], _p(out, _u8))
    return out


def write_pointcloud(path, cloud: np.ndarray) -> bool:
    cloud = np.ascontiguousarray(cloud, dtype=np.float32).reshape(-1, 6)
    return lib().sa_write_pointcloud(str(path).encode(), _p(cloud, _f), cloud.shape[0]) == 0


# ------------------------------------------------------------------------------------ calibration
class Calibration:
    """The reference's CalibrationParam (RAFTStereo/include/TRTRAFTStereo.h:30-43) backed by the
    native FileStorage reader/writer."""

    def __init__(self, path=None):
        L = lib()
        self._h = L.sa_calib_load(str(path).encode()) if path is not None else L.sa_calib_new()
        if not self._h:
            raise FileNotFoundError(f"cannot read calibration file {path}")

    def __del__(self):
        if getattr(self, "_h", None):
            lib().sa_calib_free(self._h)
            self._h = None

    def __getitem__(self, key: str) -> np.ndarray | None:
        buf = np.zeros(64, np.float64)
        r, c = C.c_int(), C.c_int()
        n = lib().sa_calib_get(self._h, key.encode(), _p(buf, _d), 64, C.byref(r), C.byref(c))
        if n < 0:
            raise KeyError(key)
        return None if n == 0 else buf[:n].reshape(r.value, c.value).copy()

    def __setitem__(self, key: str, value):
        v = _f64(np.atleast_2d(value))
        if lib().sa_calib_set(self._h, key.encode(), _p(v, _d), v.shape[0], v.shape[1]) != 0:
            raise KeyError(key)

    @property
    def rois(self):
        out = np.zeros(8, np.int32)
        has = lib().sa_calib_get_roi(self._h, _p(out, _i))
        return (tuple(out[:4]), tuple(out[4:])) if has else None

    @rois.setter
    def rois(self, v):
        a = np.ascontiguousarray(np.concatenate([np.asarray(v[0]), np.asarray(v[1])]), dtype=np.int32)
        lib().sa_calib_set_roi(self._h, _p(a, _i))

    def save(self, path):
        if lib().sa_calib_save(self._h, str(path).encode()) != 0:
            raise IOError(f"cannot write {path}")

    def stereo_rectify(self, width=640, height=480, alpha=-1.0, zero_disparity=True):
        if lib().sa_calib_stereo_rectify(self._h, width, height, alpha, int(zero_disparity)) != 0:
            raise ValueError("stereo_rectify needs R and T")

    def rectify_maps(self, width=640, height=480, quantize=True):
        """(map_left, map_right) float32 [H, W, 2] for cv::remap / the HIP remap kernel."""
        ml = np.empty((height, width, 2), np.float32)
        mr = np.empty_like(ml)
        if lib().sa_calib_rectify_maps(self._h, width, height, _p(ml, _f), _p(mr, _f), int(quantize)) != 0:
            raise ValueError("calibration lacks intrinsics")
        return ml, mr

    def Q(self):
        return self["Q"]


def undistort_points(pts, K, D=None, R=None, P=None):
    pts = _f64(np.asarray(pts).reshape(-1, 2))
    K, D, R, P = _f64(K), _f64(D), _f64(R), _f64(P)
    out = np.empty_like(pts)
    nd = 0 if D is None else D.size
    pr, pc = (P.shape if P is not None else (0, 0))
    lib().sa_undistort_points(_p(K, _d), _p(D, _d), nd, _p(R, _d), _p(P, _d), pr, pc, _p(pts, _d), pts.shape[0],
                              _p(out, _d))
    return out


def project_points(obj, rvec, tvec, K, D=None):
    obj = _f64(np.asarray(obj).reshape(-1, 3))
    out = np.empty((obj.shape[0], 2), np.float64)
    D = _f64(D)
    lib().sa_project_points(_p(obj, _d), obj.shape[0], _p(_f64(rvec), _d), _p(_f64(tvec), _d), _p(_f64(K), _d),
                            _p(D, _d), 0 if D is None else D.size, _p(out, _d))
    return out


def rodrigues(v):
    v = _f64(v)
    if v.size == 3:
        out = np.empty(9, np.float64)
        lib().sa_rodrigues(_p(v, _d), _p(out, _d))
        return out.reshape(3, 3)
    out = np.empty(3, np.float64)
    lib().sa_rodrigues_inv(_p(v, _d), _p(out, _d))
    return out


def remap(img: np.ndarray, map_xy: np.ndarray) -> np.ndarray:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    c = 1 if img.ndim == 2 else img.shape[2]
    out = np.empty_like(img)
    m = np.ascontiguousarray(map_xy, dtype=np.float32)
    lib().sa_remap_u8_cpu(_p(img, _u8), img.shape[0], img.shape[1], c, _p(m, _f), _p(out, _u8))
    return out


def reproject(disp: np.ndarray, Q) -> np.ndarray:
    disp = np.ascontiguousarray(disp, dtype=np.float32)
    out = np.empty(disp.shape + (3,), np.float32)
    lib().sa_reproject_cpu(_p(disp, _f), disp.shape[0], disp.shape[1], _p(_f64(Q), _d), _p(out, _f))
    return out


# ------------------------------------------------------------------ calibration tool
def find_chessboard(gray: np.ndarray, cols: int = 11, rows: int = 8, subpix: bool = True) -> np.ndarray | None:
    """Inner chessboard corners [cols*rows, 2] (row-major from the top-left) or None."""
    g = np.ascontiguousarray(gray, dtype=np.uint8)
    out = np.zeros((cols * rows, 2), np.float64)
    ok = lib().sa_find_chessboard(_p(g, _u8), g.shape[0], g.shape[1], cols, rows, int(subpix), _p(out, _d))
    return out if ok else None


def stereo_calibrate_images(paths, cols: int = 11, rows: int = 8, square: float = 25.0, subpix: bool = True):
    """The Stereo_Calibration pipeline over alternating left/right image paths.
    Returns (Calibration, used_pairs, (rms_left, rms_right, rms_stereo))."""
    cal = Calibration()
    rms = np.zeros(3, np.float64)
    n = lib().sa_stereo_calibrate_images("\n".join(str(p) for p in paths).encode(), cols, rows, float(square),
                                        int(subpix), cal._h, _p(rms, _d))
    if n < 0:
        raise RuntimeError(f"stereo calibration failed ({n})")
    return cal, n, tuple(rms.tolist())
