"""CPU tests of the native host library (libstereo_host.so): calibration YAML, rectification math,
image codecs, colour maps, point-cloud output.  Reference files: tests/fixtures (copied from the
reference's */test and Stereo_Calibration directories)."""
import math

import numpy as np
import pytest

from stereoalgorithms_amd.utils import hostlib as H

FIX = "tests/fixtures"


@pytest.fixture(scope="module")
def calib():
    return H.Calibration(f"{FIX}/StereoCalibration.yml")


def test_yaml_roundtrip_is_byte_identical(calib, tmp_path):
    # OpenCV FileStorage formatting (%.16e, "1." for integral values, 71-column wrapping)
    out = tmp_path / "c.yml"
    calib.save(out)
    assert out.read_text() == open(f"{FIX}/StereoCalibration.yml").read()


def test_yaml_reader_values(calib):
    K = calib["intrinsic_left"]
    assert K.shape == (3, 3) and abs(K[0, 0] - 517.86623547729778) < 1e-12 and K[2, 2] == 1
    assert calib["distCoeffs_left"].shape == (1, 5)
    assert calib["T"].shape == (3, 1) and abs(calib["T"][0, 0] + 60.101825472125526) < 1e-12
    assert calib.rois == ((0, 0, 640, 480), (0, 0, 640, 480))


def test_yaml_rational_model_file():
    # StereoCalibration_new.yml: hand-formatted data, 1x8 rational distortion, negative Q[14]
    c = H.Calibration(f"{FIX}/StereoCalibration_new.yml")
    d = c["distCoeffs_left"]
    assert d.shape == (1, 8) and abs(d[0, 5] - 1.2095338665) < 1e-12
    assert c["Q"][3, 2] < 0


def test_missing_keys_are_empty(tmp_path):
    p = tmp_path / "partial.yml"
    p.write_text("%YAML:1.0\n---\nQ: !!opencv-matrix\n   rows: 1\n   cols: 2\n   dt: d\n   data: [ 1., 2. ]\n")
    c = H.Calibration(p)
    assert c["intrinsic_left"] is None
    assert np.array_equal(c["Q"], [[1.0, 2.0]])


def test_stereo_rectify_matches_reference_file(calib):
    """cv::stereoRectify(CALIB_ZERO_DISPARITY, alpha=0) as run by Stereo_Calibration.cpp:162 reproduces
    the R_L/R_R/P1/P2/Q stored in the reference's calibration file.  Tolerance: the image corners
    of this lens do not converge in undistortPoints' 5 fixed-point steps, so f/c move by ~0.1%
    between OpenCV builds (documented in csrc/host/camera.cpp)."""
    ref = {k: calib[k] for k in ("R_L", "R_R", "P1", "P2", "Q")}
    c = H.Calibration(f"{FIX}/StereoCalibration.yml")
    c.stereo_rectify(640, 480, alpha=0.0, zero_disparity=True)
    assert np.abs(c["R_L"] - ref["R_L"]).max() < 1e-6
    assert np.abs(c["R_R"] - ref["R_R"]).max() < 1e-6
    for k in ("P1", "P2"):
        assert np.allclose(c[k], ref[k], rtol=2e-3, atol=0.6)
    # Q structure: [1 0 0 -cx; 0 1 0 -cy; 0 0 0 f; 0 0 -1/Tx (cx-cx')/Tx]
    Q = c["Q"]
    assert np.isclose(Q[3, 2], ref["Q"][3, 2], rtol=1e-6) and Q[3, 3] == 0.0
    assert np.isclose(Q[2, 3], c["P1"][0, 0])
    # rectified rotations are consistent with the stereo extrinsics: R_R R R_L^T = I
    assert np.abs(c["R_R"] @ calib["R"] @ c["R_L"].T - np.eye(3)).max() < 1e-12


def _np_rectify_map(K, D, R, P, w, h):
    """numpy re-derivation of OpenCV's initUndistortRectifyMap model (5 coeffs)."""
    k1, k2, p1, p2, k3 = D.ravel()[:5]
    iR = np.linalg.inv(P[:3, :3] @ R)
    jj, ii = np.meshgrid(np.arange(w), np.arange(h))
    X = iR @ np.stack([jj.ravel(), ii.ravel(), np.ones(w * h)])
    x, y = X[0] / X[2], X[1] / X[2]
    r2 = x * x + y * y
    kr = 1 + k1 * r2 + k2 * r2 ** 2 + k3 * r2 ** 3
    xd = x * kr + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * kr + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    u = K[0, 0] * xd + K[0, 2]
    v = K[1, 1] * yd + K[1, 2]
    return np.stack([u, v], -1).reshape(h, w, 2)


def test_rectify_map_matches_numpy_model(calib):
    ml, mr = calib.rectify_maps(640, 480, quantize=False)
    ref_l = _np_rectify_map(calib["intrinsic_left"], calib["distCoeffs_left"], calib["R_L"], calib["P1"], 640, 480)
    ref_r = _np_rectify_map(calib["intrinsic_right"], calib["distCoeffs_right"], calib["R_R"], calib["P2"], 640,
                            480)
    assert np.abs(ml - ref_l).max() < 1e-3 and np.abs(mr - ref_r).max() < 1e-3
    q, _ = calib.rectify_maps(640, 480, quantize=True)  # CV_16SC2: 1/32-pixel grid
    assert np.allclose(q * 32, np.round(q * 32)) and np.abs(q - ml).max() <= 1 / 64 + 1e-4


def test_rectify_map_rational_model():
    c = H.Calibration(f"{FIX}/StereoCalibration_new.yml")
    ml, mr = c.rectify_maps(640, 480, quantize=False)
    assert np.isfinite(ml).all() and np.isfinite(mr).all()


def test_project_undistort_roundtrip(calib):
    K, D = calib["intrinsic_left"], calib["distCoeffs_left"]
    rng = np.random.default_rng(0)
    obj = np.concatenate([rng.uniform(-0.3, 0.3, (50, 2)), np.ones((50, 1))], 1)
    img = H.project_points(obj, np.zeros(3), np.zeros(3), K, D)
    und = H.undistort_points(img, K, D)
    assert np.abs(und - obj[:, :2]).max() < 1e-6


def test_rodrigues_roundtrip():
    r = np.array([0.1, -0.2, 0.3])
    R = H.rodrigues(r)
    assert np.allclose(R @ R.T, np.eye(3), atol=1e-12)
    th = np.linalg.norm(r)
    k = r / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    assert np.allclose(R, np.eye(3) + math.sin(th) * Kx + (1 - math.cos(th)) * Kx @ Kx)
    assert np.allclose(H.rodrigues(R), r)


def test_remap_identity_and_shift():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (40, 50, 3), dtype=np.uint8)
    ys, xs = np.mgrid[0:40, 0:50].astype(np.float32)
    assert np.array_equal(H.remap(img, np.stack([xs, ys], -1)), img)
    out = H.remap(img, np.stack([xs + 2, ys], -1))
    assert np.array_equal(out[:, :48], img[:, 2:]) and (out[:, 48:] == 0).all()
    half = H.remap(img, np.stack([xs + 0.5, ys], -1)).astype(int)
    expect = (img[:, :-1].astype(int) + img[:, 1:]) / 2
    assert np.abs(half[:, :-1] - expect).max() <= 1


def test_reproject_cpu_matches_formula(calib):
    Q = calib["Q"]
    d = np.full((4, 5), 30.0, np.float32)
    xyz = H.reproject(d, Q)
    c, r = 3, 2
    X = Q @ np.array([c, r, 30.0, 1.0])
    assert np.allclose(xyz[r, c], X[:3] / X[3], rtol=1e-5)


def test_jpeg_decoder_matches_pil():
    from PIL import Image
    ours = H.imread(f"{FIX}/left0.jpg")
    ref = np.asarray(Image.open(f"{FIX}/left0.jpg").convert("RGB"))[..., ::-1]
    assert ours.shape == (480, 640, 3)
    diff = np.abs(ours.astype(int) - ref.astype(int))
    assert diff.max() == 0  # ISLOW IDCT + fancy upsampling + libjpeg YCbCr tables: bit-exact


def test_jpeg_encoder_roundtrip(tmp_path):
    from PIL import Image
    img = H.imread(f"{FIX}/right0.jpg")
    p = tmp_path / "o.jpg"
    assert H.imwrite(p, img)
    back = np.asarray(Image.open(p).convert("RGB"))[..., ::-1].astype(float)
    psnr = 10 * np.log10(255 ** 2 / ((back - img) ** 2).mean())
    assert psnr > 34
    assert np.array_equal(H.imread(p), np.asarray(Image.open(p).convert("RGB"))[..., ::-1]) or \
        np.abs(H.imread(p).astype(int) - back).max() <= 2


def test_grey_float_jpeg_like_opencv(tmp_path):
    # cv::imwrite of a CV_32FC1 disparity saturates to u8 (RAFTStereo/test/main.cpp:31)
    from PIL import Image
    d = np.linspace(-10, 300, 64 * 48, dtype=np.float32).reshape(48, 64)
    p = tmp_path / "disparity.jpg"
    assert H.imwrite(p, d)
    back = np.asarray(Image.open(p))
    assert back.ndim == 2 and back.shape == (48, 64)
    expect = np.clip(np.rint(d), 0, 255)
    assert np.abs(back.astype(float) - expect).mean() < 1.5


def test_png_roundtrip_lossless(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, (33, 47, 3), dtype=np.uint8)
    p = tmp_path / "x.png"
    assert H.imwrite(p, img)
    assert np.array_equal(np.asarray(Image.open(p))[..., ::-1], img)
    assert np.array_equal(H.imread(p), img)
    ref_png = "/root/reference/CREStereo/test/test/left.png"
    import os
    if os.path.exists(ref_png):
        assert np.array_equal(H.imread(ref_png), np.asarray(Image.open(ref_png).convert("RGB"))[..., ::-1])


def test_jet_colormap_and_heatmap():
    lut = H.colormap_jet(np.arange(256, dtype=np.uint8))
    # MATLAB jet(64) interpolated to 256 (OpenCV COLORMAP_JET): dark blue -> cyan -> yellow -> dark red
    assert tuple(lut[0]) == (143, 0, 0) and tuple(lut[255]) == (0, 0, 128)
    assert lut[128, 1] > 200  # green in the middle
    d = np.linspace(0, 50, 100, dtype=np.float32).reshape(10, 10)
    hm = H.heatmap(d)
    assert hm.shape == (10, 10, 3) and tuple(hm[0, 0]) == tuple(lut[0]) and tuple(hm[-1, -1]) == tuple(lut[255])


def test_pointcloud_txt_format(tmp_path):
    cloud = np.array([[1.5, -2.0, 1000.25, 10, 20, 30], [np.inf, 0, 1e-7, 255, 0, 1]], np.float32)
    p = tmp_path / "pointcloud.txt"
    H.write_pointcloud(p, cloud)
    lines = p.read_text().splitlines()
    assert lines == ["1.5 -2 1000.25 10 20 30", "inf 0 1e-07 255 0 1"]


def test_bgr2gray_matches_opencv_coefficients():
    px = np.array([[[10, 200, 30], [255, 255, 255]]], np.uint8)
    g = H.bgr2gray(px)
    p = px.astype(np.int64)
    expect = (p[..., 0] * 1868 + p[..., 1] * 9617 + p[..., 2] * 4899 + 8192) >> 14
    assert np.array_equal(g, expect)
