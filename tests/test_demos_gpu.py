"""End-to-end runs of the reference's "tests" — its demo executables — and of the C ABI they call
(/root/reference/RAFTStereo/test/main.cpp:8-39, CREStereo/test/main.cpp:55-72,
FastACVNet_plus/test/main.cpp:42).  Headless, on the reference's own fixture pair and calibration."""
import json
import math
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "stereoalgorithms_amd", "bin")
LIB = os.path.join(ROOT, "stereoalgorithms_amd", "lib")
FX = os.path.join(ROOT, "tests", "fixtures")
H, W = 480, 640

DEMOS = ["raft_stereo_demo", "HitNet_demo", "crestereo_demo", "fastacvnet_plus_demo"]


def _jpeg_size(path):
    """(width, height) from the SOF0 marker."""
    b = open(path, "rb").read()
    i = 2
    while i < len(b):
        assert b[i] == 0xFF
        m, ln = b[i + 1], (b[i + 2] << 8) | b[i + 3]
        if m in (0xC0, 0xC1):
            return (b[i + 7] << 8) | b[i + 8], (b[i + 5] << 8) | b[i + 6]
        i += 2 + ln
    raise AssertionError("no SOF")


@pytest.mark.gpu
@pytest.mark.parametrize("demo", DEMOS)
def test_demo_writes_outputs(demo, tmp_path):
    r = subprocess.run([os.path.join(BIN, demo), "--left", os.path.join(FX, "left0.jpg"),
                        "--right", os.path.join(FX, "right0.jpg"), "--calib", os.path.join(FX, "StereoCalibration.yml"),
                        "--frames", "3", "--out", str(tmp_path)], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "Algorithm_V1.0" in r.stdout and "mean" in r.stdout
    for f in ("disparity.jpg", "heatmap.jpg"):
        assert _jpeg_size(tmp_path / f) == (W, H), f
    lines = (tmp_path / "pointcloud.txt").read_text().splitlines()
    assert len(lines) == H * W
    nfin = 0
    for ln in lines[:: 97]:
        v = ln.split()
        assert len(v) == 6
        xyz = [float(t) for t in v[:3]]
        rgb = [float(t) for t in v[3:]]
        assert all(0 <= c <= 255 for c in rgb)
        nfin += all(math.isfinite(t) for t in xyz)
    assert nfin > 0


@pytest.mark.gpu
def test_demo_stream_list(tmp_path):
    """--list: several pairs streamed through the host frame pipeline (decode / write threads beside the engine)."""
    lst = tmp_path / "pairs.txt"
    lst.write_text("".join(f"{os.path.join(FX, 'left0.jpg')} {os.path.join(FX, 'right0.jpg')}\n" for _ in range(4)))
    r = subprocess.run([os.path.join(BIN, "raft_stereo_demo"), "--model", "raftstereo-realtime", "--list", str(lst),
                        "--save-all", "--calib", os.path.join(FX, "StereoCalibration.yml"), "--out", str(tmp_path)],
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "stream frames 4" in r.stdout
    for i in range(4):
        assert _jpeg_size(tmp_path / f"disparity_{i}.jpg") == (W, H)
    assert _jpeg_size(tmp_path / "heatmap.jpg") == (W, H)
    assert len((tmp_path / "pointcloud.txt").read_text().splitlines()) == H * W


@pytest.mark.gpu
def test_c_abi_contract():
    r = subprocess.run([os.path.join(BIN, "abi_check"), LIB, os.path.join(FX, "left0.jpg"), os.path.join(FX, "right0.jpg"),
                        os.path.join(FX, "StereoCalibration.yml"), "2"], capture_output=True, text=True, timeout=110)
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(recs) == 4, r.stdout + r.stderr[-2000:]
    for rec in recs:
        assert rec["ok"], rec
        assert rec["missing_calib_null"] and rec["version_ok"] and rec["plain_entry_rectify_semantics"]
        assert rec["finite"] == H * W and rec["bad_xyz"] == 0
    assert r.returncode == 0
