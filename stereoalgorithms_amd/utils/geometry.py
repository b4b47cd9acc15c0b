"""Stereo geometry in numpy (reference implementations + helpers).

These mirror the OpenCV calls the reference makes on the CPU every frame
(``cv::initUndistortRectifyMap`` + ``cv::remap``, RAFTStereo/src/RAFTStereoAlgorithm.cpp:113-126) and the
reprojection of its GPU kernels (``cv::reprojectImageTo3D`` semantics,
RAFTStereo/src/stereo_preprocess.cu:41-68).  OpenCV is not available here, so the formulas are
re-derived; the production path computes the maps once natively (csrc/geometry) and remaps on the
GPU (csrc/kernels/prepost.hip).  These numpy versions are the test oracles.
"""
from __future__ import annotations

import numpy as np


def _dist(D) -> np.ndarray:
    d = np.zeros(14, np.float64)
    D = np.asarray(D, np.float64).ravel()
    d[: min(len(D), 14)] = D[:14]
    return d


def distort_normalized(x, y, D):
    """Apply OpenCV's radial/tangential/rational/thin-prism distortion to normalised coords."""
    k1, k2, p1, p2, k3, k4, k5, k6, s1, s2, s3, s4 = _dist(D)[:12]
    x2, y2 = x * x, y * y
    r2 = x2 + y2
    _2xy = 2 * x * y
    kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2)
    xd = x * kr + p1 * _2xy + p2 * (r2 + 2 * x2) + s1 * r2 + s2 * r2 * r2
    yd = y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy + s3 * r2 + s4 * r2 * r2
    return xd, yd


def init_undistort_rectify_map(K, D, R, P, size) -> np.ndarray:
    """cv::initUndistortRectifyMap -> float map [H, W, 2] (x, y) in source pixel coordinates."""
    K = np.asarray(K, np.float64).reshape(3, 3)
    R = np.eye(3) if R is None or np.size(R) == 0 else np.asarray(R, np.float64).reshape(3, 3)
    P = np.asarray(P, np.float64)
    newK = P.reshape(3, -1)[:, :3]
    iR = np.linalg.inv(newK @ R)
    w, h = size
    jj, ii = np.meshgrid(np.arange(w, dtype=np.float64), np.arange(h, dtype=np.float64))
    _x = jj * iR[0, 0] + ii * iR[0, 1] + iR[0, 2]
    _y = jj * iR[1, 0] + ii * iR[1, 1] + iR[1, 2]
    _w = jj * iR[2, 0] + ii * iR[2, 1] + iR[2, 2]
    x, y = _x / _w, _y / _w
    xd, yd = distort_normalized(x, y, D)
    fx, fy, u0, v0 = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    return np.stack([fx * xd + u0, fy * yd + v0], -1).astype(np.float32)


def _remap_weights(ax_i: np.ndarray, ay_i: np.ndarray) -> np.ndarray:
    """OpenCV INTER_LINEAR fixed-point coefficients (sum 32768) for 1/32 sub-pixel indices."""
    ax, ay = ax_i / 32.0, ay_i / 32.0
    wf = np.stack([(1 - ax) * (1 - ay), ax * (1 - ay), (1 - ax) * ay, ax * ay], -1)
    wi = np.rint(wf * 32768).astype(np.int64)
    diff = wi.sum(-1) - 32768
    big = np.argmax(wi, -1)
    small = np.argmin(wi, -1)
    idx = np.where(diff < 0, big, small)
    np.put_along_axis(wi, idx[..., None], np.take_along_axis(wi, idx[..., None], -1) - diff[..., None], -1)
    return wi


def remap_bilinear_u8(src: np.ndarray, maps: np.ndarray) -> np.ndarray:
    """cv::remap(src, dst, map, INTER_LINEAR, BORDER_CONSTANT=0) with CV_16SC2 quantisation."""
    hs, ws = src.shape[:2]
    iu = np.rint(maps[..., 0].astype(np.float64) * 32).astype(np.int64)
    iv = np.rint(maps[..., 1].astype(np.float64) * 32).astype(np.int64)
    x0, y0 = iu >> 5, iv >> 5
    wi = _remap_weights(iu & 31, iv & 31)
    acc = np.zeros(maps.shape[:2] + (src.shape[2],), np.int64)
    for j, (dx, dy) in enumerate(((0, 0), (1, 0), (0, 1), (1, 1))):
        xx, yy = x0 + dx, y0 + dy
        ok = (xx >= 0) & (xx < ws) & (yy >= 0) & (yy < hs)
        px = src[np.clip(yy, 0, hs - 1), np.clip(xx, 0, ws - 1)].astype(np.int64)
        acc += np.where(ok[..., None], px * wi[..., j:j + 1], 0)
    return np.clip((acc + (1 << 14)) >> 15, 0, 255).astype(np.uint8)


def reproject_image_to_3d(disp: np.ndarray, Q) -> np.ndarray:
    """[H,W] disparity -> [H,W,3] XYZ using the full 4x4 Q (homogeneous divide)."""
    Q = np.asarray(Q, np.float64).reshape(4, 4)
    h, w = disp.shape
    jj, ii = np.meshgrid(np.arange(w, dtype=np.float64), np.arange(h, dtype=np.float64))
    v = np.stack([jj, ii, disp.astype(np.float64), np.ones_like(jj)], -1) @ Q.T
    with np.errstate(divide="ignore", invalid="ignore"):
        return (v[..., :3] / v[..., 3:4]).astype(np.float32)


def reproject_cloud_torch(disp, left_bgr, Q):
    """Batched XYZRGB point cloud [B,H,W,6] fp32 of disparity [B,H,W] with the full 4x4 Q, colours from the left
    BGR u8 image as RGB -- the contract of the reprojection kernel (csrc/kernels/prepost.hip) and of the
    reference's reprojectImageTo3D kernels (RAFTStereo/src/stereo_preprocess.cu:41-68).  torch, any device."""
    import torch
    q = torch.as_tensor(np.asarray(Q, np.float32).reshape(4, 4), device=disp.device)
    b, h, w = disp.shape
    c = torch.arange(w, device=disp.device, dtype=torch.float32).view(1, 1, w).expand(b, h, w)
    r = torch.arange(h, device=disp.device, dtype=torch.float32).view(1, h, 1).expand(b, h, w)
    d = disp.float()
    comp = [q[i, 0] * c + q[i, 1] * r + q[i, 2] * d + q[i, 3] for i in range(4)]
    xyz = torch.stack([comp[0] / comp[3], comp[1] / comp[3], comp[2] / comp[3]], -1)
    return torch.cat([xyz, left_bgr.flip(-1).float()], -1).contiguous()


def rectify_maps_from_calib(calib: dict, size=(640, 480)):
    """Left/right maps from a StereoCalibration.yml dict (keys of the reference)."""
    ml = init_undistort_rectify_map(calib["intrinsic_left"], calib["distCoeffs_left"], calib["R_L"], calib["P1"], size)
    mr = init_undistort_rectify_map(calib["intrinsic_right"], calib["distCoeffs_right"], calib["R_R"], calib["P2"], size)
    return ml, mr
