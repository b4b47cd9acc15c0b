"""Synthetic rectified stereo pairs (no datasets are available offline).

A multi-scale random texture is rendered for the left view and warped with a known smooth
disparity field (right(x) = left(x + d(x))), giving BGR uint8 pairs of the reference's input shape
(640x480) for the demos, tests and benchmarks.
"""
from __future__ import annotations

import numpy as np


def _texture(rng, h, w):
    img = np.zeros((h, w, 3), np.float64)
    for s in (4, 8, 16, 32, 64):
        gh, gw = h // s + 2, w // s + 2
        g = rng.random((gh, gw, 3))
        yi = np.linspace(0, gh - 1.001, h)
        xi = np.linspace(0, gw - 1.001, w)
        y0, x0 = yi.astype(int), xi.astype(int)
        fy, fx = (yi - y0)[:, None, None], (xi - x0)[None, :, None]
        a = g[y0][:, x0]
        b = g[y0][:, x0 + 1]
        c = g[y0 + 1][:, x0]
        d = g[y0 + 1][:, x0 + 1]
        img += (a * (1 - fx) * (1 - fy) + b * fx * (1 - fy) + c * (1 - fx) * fy + d * fx * fy) * (s / 64.0) ** 0.5
    img -= img.min()
    img /= img.max() + 1e-9
    return img


def stereo_pair(h=480, w=640, max_disp=48.0, seed=0):
    """Returns (left_bgr u8 [h,w,3], right_bgr u8 [h,w,3], disparity f32 [h,w])."""
    rng = np.random.default_rng(seed)
    pad = int(max_disp) + 2
    tex = _texture(rng, h, w + pad)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    disp = 0.25 * max_disp + 0.6 * max_disp * (0.5 + 0.5 * np.sin(xx / w * 3.1 + yy / h * 2.3)) * (yy / h)
    left = tex[:, :w]
    xs = xx + disp  # right(x) = left(x + d)?  right view sees the point at x - d: right(x) = L(x + d)
    x0 = np.clip(np.floor(xs).astype(int), 0, w + pad - 2)
    fx = (xs - np.floor(xs))[..., None]
    right = tex[yy.astype(int), x0] * (1 - fx) + tex[yy.astype(int), x0 + 1] * fx
    to_u8 = lambda a: (np.clip(a, 0, 1) * 255).astype(np.uint8)[..., ::-1].copy()  # RGB->BGR
    return to_u8(left), to_u8(right), disp.astype(np.float32)


def batch_pairs(n, h=480, w=640, seed=0):
    ls, rs = [], []
    for i in range(n):
        l, r, _ = stereo_pair(h, w, seed=seed + i)
        ls.append(l)
        rs.append(r)
    return np.stack(ls), np.stack(rs)
