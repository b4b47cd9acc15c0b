#!/usr/bin/env python3
"""Split side-by-side stereo captures into left/right images (reference
Stereo_Calibration/process_image.py:16-26: 1280x480 frames -> left<i>.jpg / right<i>.jpg of 640x480).

    python3 tools/split_stereo.py Stereo_Raw/ left_right_image/ [--width-left 640]

Images are read and written with the framework's own baseline JPEG/PNG codec (no OpenCV); the
left half is columns [0, W/2), the right half [W/2, W).  Files are processed in sorted name order
(the reference used os.listdir order, which is unspecified) and numbered from 0.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def split_pair(img, width_left=None):
    w = img.shape[1]
    wl = width_left or w // 2
    if not 0 < wl < w:
        raise ValueError(f"bad split column {wl} for width {w}")
    return img[:, :wl].copy(), img[:, wl:].copy()


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("src_dir")
    p.add_argument("dst_dir")
    p.add_argument("--width-left", type=int, default=None, help="split column (default: half the width)")
    p.add_argument("--quality", type=int, default=95)
    a = p.parse_args(argv)
    from stereoalgorithms_amd.utils import hostlib as H
    os.makedirs(a.dst_dir, exist_ok=True)
    exts = (".jpg", ".jpeg", ".png")
    names = sorted(n for n in os.listdir(a.src_dir) if n.lower().endswith(exts))
    i = 0
    for n in names:
        img = H.imread(os.path.join(a.src_dir, n))
        if img is None:
            print(f"skip unreadable {n}")
            continue
        left, right = split_pair(img, a.width_left)
        H.imwrite(os.path.join(a.dst_dir, f"left{i}.jpg"), left, a.quality)
        H.imwrite(os.path.join(a.dst_dir, f"right{i}.jpg"), right, a.quality)
        i += 1
    print(f"split {i} image(s) into {a.dst_dir}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
