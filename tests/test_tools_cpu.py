"""CPU tests of the capture-side tools: side-by-side splitter (reference
Stereo_Calibration/process_image.py) and the V4L2 capture app's argument / error handling
(reference usb_test.py; no camera exists here, so only the paths that need none are exercised)."""
import os
import re
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))


def _host():
    from stereoalgorithms_amd.utils import hostlib as H
    try:
        H.lib()
    except Exception as e:  # pragma: no cover
        pytest.skip(f"host library not built: {e}")
    return H


def test_split_stereo_halves(tmp_path):
    H = _host()
    import split_stereo
    src = tmp_path / "raw"
    src.mkdir()
    yy, xx = np.mgrid[0:48, 0:128]
    frames = []
    for i in range(3):  # smooth gradients (JPEG-friendly), different ramps on the two halves
        f = np.stack([(xx + 20 * i) % 128, yy * 2 + 10 * i, np.where(xx < 64, 40, 200) + 0 * yy], -1)
        frames.append(f.astype(np.uint8))
    for i, f in enumerate(frames):
        assert H.imwrite(src / f"{i:02d}.png", f)
    dst = tmp_path / "lr"
    assert split_stereo.main([str(src), str(dst)]) == 0
    for i, f in enumerate(frames):
        l, r = H.imread(dst / f"left{i}.jpg"), H.imread(dst / f"right{i}.jpg")
        assert l.shape == (48, 64, 3) and r.shape == (48, 64, 3)
        # JPEG q95 round trip: small error, halves not swapped
        assert np.abs(l.astype(int) - f[:, :64]).mean() < 3
        assert np.abs(r.astype(int) - f[:, 64:]).mean() < 3
        assert np.abs(l.astype(int) - f[:, 64:]).mean() > 30


def test_split_pair_exact_and_bad_column():
    import split_stereo
    img = np.arange(4 * 10 * 3, dtype=np.uint8).reshape(4, 10, 3)
    l, r = split_stereo.split_pair(img)
    assert np.array_equal(np.concatenate([l, r], 1), img) and l.shape[1] == 5
    l, r = split_stereo.split_pair(img, 3)
    assert l.shape[1] == 3 and r.shape[1] == 7
    with pytest.raises(ValueError):
        split_stereo.split_pair(img, 10)


def test_stereo_capture_cli():
    exe = ROOT / "stereoalgorithms_amd" / "bin" / "stereo_capture"
    if not exe.exists():
        pytest.skip("capture app not built")
    r = subprocess.run([str(exe), "--help"], capture_output=True, text=True, timeout=30)
    assert r.returncode == 0 and "--device" in r.stdout
    r = subprocess.run([str(exe), "--device", "/dev/does-not-exist"], capture_output=True, text=True, timeout=30)
    assert r.returncode == 1 and "cannot open" in r.stderr
    r = subprocess.run([str(exe), "--bogus"], capture_output=True, text=True, timeout=30)
    assert r.returncode == 2


def test_cmake_configures(tmp_path):
    """The CMake build (for C++ users, as the reference's) configures; SA_TEST_CMAKE_BUILD=1 also
    builds every target (~1 min on 8 cores)."""
    import shutil
    if not shutil.which("cmake") or not Path("/opt/rocm/llvm/bin/clang++").exists():
        pytest.skip("cmake / ROCm toolchain not available")
    b = tmp_path / "cmb"
    r = subprocess.run(["cmake", "-S", str(ROOT), "-B", str(b)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    if os.environ.get("SA_TEST_CMAKE_BUILD") == "1":
        r = subprocess.run(["cmake", "--build", str(b), "-j", "8"], capture_output=True, text=True, timeout=1800)
        assert r.returncode == 0, r.stdout[-3000:]
        for t in ("libstereo_amd.so", "libRAFTStereo.so", "raft_stereo_demo", "Stereo_Calibration"):
            assert (b / t).exists()


def test_host_sanitizers(tmp_path):
    """Host code under ASan + UBSan: calibration YAML, rectification, codecs,
    heat-map, point cloud, chessboard detection and a short stereo calibration on the fixtures."""
    import shutil
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    r = subprocess.run(["bash", str(ROOT / "tools" / "sanitize" / "run.sh"), str(tmp_path)], capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "host_check ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr


def test_hostcopy_pool_tsan(tmp_path):
    """The timed-region copy pool (csrc/runtime/hostcopy.cpp) under ThreadSanitizer: 100k back-to-back run() calls
    with 1-5 tiny tasks each.  The round-2 pool lost a task when a worker woke late for a finished run (a hang
    under this stress); claims now carry the run's generation."""
    import shutil
    if not shutil.which("g++") or not os.path.exists("/opt/rocm/lib/libamdhip64.so"):
        pytest.skip("g++ / HIP runtime not available")
    r = subprocess.run(["bash", str(ROOT / "tools" / "sanitize" / "hostcopy_tsan.sh"), str(tmp_path), "100000"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "hostcopy_stress: 100000 runs x 3 workers ok" in r.stdout
    assert "ThreadSanitizer" not in r.stderr


def test_frame_pipeline_tsan(tmp_path):
    """The host frame pipeline (csrc/host/pipeline.cpp: loader thread -> engine thread -> writer thread with
    recycled frames) under ThreadSanitizer: order and content through recycled buffers, and clean shutdown after a
    failing Infer, a throwing Source / Sink and a frame cap."""
    import shutil
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    r = subprocess.run(["bash", str(ROOT / "tools" / "sanitize" / "pipeline_tsan.sh"), str(tmp_path), "400"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "pipeline_stress: 400 rounds ok" in r.stdout
    assert "ThreadSanitizer" not in r.stderr


def test_timeline_critical_chain(tmp_path):
    """tools/timeline.py on a synthetic two-frame trace: frame cut at the preprocess marker, busy / idle union,
    iterations at the marker kernel and the critical chain (latest-ending predecessor) with its launch gaps."""
    hdr = "Kernel_Name,Start_Timestamp,End_Timestamp,Grid_Size_X,Workgroup_Size_X\n"
    rows = []
    for f in range(3):
        t = f * 1_000_000
        rows += [("preprocess_kernel", t, t + 1000), ("enc_kernel", t + 1000, t + 5000),
                 ("side_kernel", t + 1200, t + 2000)]  # a concurrent branch, off the chain
        for it in range(3):
            b = t + 6000 + it * 10000
            rows += [("motion_encoder_kernel", b, b + 3000), ("gru_kernel", b + 3000, b + 8000)]
    csv = tmp_path / "x_kernel_trace.csv"
    csv.write_text(hdr + "".join(f"{n},{s},{e},256,256\n" for n, s, e in rows))
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "timeline.py"), str(csv), "--iter-marker",
                        "motion_encoder", "--chain", "5"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    out = r.stdout
    assert "3 iterations" in out
    # frame: 0..34000 ns span, idle = the 1000 ns before iteration 0 plus 2000 ns between iterations
    m = re.search(r"span\s+([\d.]+) us, busy\s+([\d.]+) us", out)
    assert m and abs(float(m.group(1)) - 34.0) < 1e-6 and abs(float(m.group(2)) - 29.0) < 1e-6, out
    chain = out[out.index("critical chain"):]
    # the concurrent branch is off the chain; the chain accounts for the whole span (kernels + launch gaps)
    assert "side_kernel" not in chain, out
    m = re.search(r"([\d.]+) us in kernels \+ ([\d.]+) us of launch gaps = ([\d.]+) us", chain)
    assert m and abs(float(m.group(1)) - 29.0) < 1e-6 and abs(float(m.group(3)) - 34.0) < 1e-6, chain


def test_pmc_summary_busy_fraction(tmp_path):
    """tools/pmc_summary.py: per-dispatch counters summed over rows, medians per (kernel, grid), and the MFMA busy
    fraction at the held clock = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)."""
    csv = tmp_path / "run_counter_collection.csv"
    rows = ["Dispatch_Id,Kernel_Name,Grid_Size,Counter_Name,Counter_Value"]
    for d in range(3):
        # two rows per counter and dispatch (e.g. per XCD slices) are summed
        rows += [f"{d},conv_igemm_kernel<256>,614400,SQ_VALU_MFMA_BUSY_CYCLES,{1.0e8}",
                 f"{d},conv_igemm_kernel<256>,614400,SQ_VALU_MFMA_BUSY_CYCLES,{1.0e8}",
                 f"{d},conv_igemm_kernel<256>,614400,GRBM_GUI_ACTIVE,{4.0e6}",
                 f"{d},other_kernel,256,GRBM_GUI_ACTIVE,{1.0e3}"]
    csv.write_text("\n".join(rows) + "\n")
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "pmc_summary.py"), str(csv), "--match", "conv_igemm"],
                         capture_output=True, text=True, check=True).stdout
    assert "other_kernel" not in out
    assert "SQ_VALU_MFMA_BUSY_CYCLES         2e+08" in out
    # 2e8 / (4e6 / 8 * 1024) = 0.390625
    assert "held clock, busy / (GRBM_GUI_ACTIVE / 8 x 1024): 0.391" in out


def test_bench_regress_gate(tmp_path):
    """tools/bench_regress.py: a > tol slower preset (or lower throughput) fails the gate, faster ones pass; the
    baseline may be a driver BENCH_rNN.json (bench line inside run.stdout_tail) or a plain bench log."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]

    def line(fps, sf_ms, sf_net):
        return json.dumps({"metric": "m", "value": fps, "latency_b1": {
            "raftstereo-sceneflow": {"latency_ms_mean": sf_ms,
                                     "device_stages_ms": {"encoders+corr": 1.0, "gru_iterations": sf_net - 1.0,
                                                          "reproject": 0.16}}}})

    base = tmp_path / "BENCH_r01.json"
    base.write_text(json.dumps({"parsed": {}, "run": {"stdout_tail": "noise\n" + line(100.0, 8.0, 7.0) + "\n"}}))

    def gate(text):
        f = tmp_path / "fresh.log"
        f.write_text("warmup...\n" + text + "\n")
        r = subprocess.run([sys.executable, str(root / "tools" / "bench_regress.py"), str(f), "--baseline", str(base)],
                           capture_output=True, text=True)
        return r.returncode, r.stdout

    rc, out = gate(line(101.0, 7.9, 6.9))
    assert rc == 0 and "0 regression(s)" in out
    rc, out = gate(line(95.0, 7.9, 6.9))  # throughput -5 %
    assert rc == 1 and "REGRESSION" in out
    rc, out = gate(line(100.0, 8.4, 7.0))  # latency +5 %
    assert rc == 1 and "raftstereo-sceneflow latency" in out
    rc, out = gate(line(100.0, 8.1, 7.1))  # +1.25 % / +1.4 %: within the 3 % tolerance
    assert rc == 0


def test_timeline_cross_queue_links(tmp_path):
    """tools/timeline.py splits the critical chain's links by hardware queue (rocprofv3 Queue_Id): a chain that
    hops queues twice per frame reports those hops and their gaps apart from the same-queue links."""
    hdr = "Kernel_Name,Start_Timestamp,End_Timestamp,Grid_Size_X,Workgroup_Size_X,Queue_Id\n"
    rows = []
    for f in range(3):
        t = f * 1_000_000
        rows += [("preprocess_kernel", t, t + 1000, 2), ("a_kernel", t + 2000, t + 5000, 2),
                 ("b_kernel", t + 15000, t + 20000, 4),   # 10 us cross-queue gap
                 ("c_kernel", t + 21000, t + 25000, 4),   # 1 us same-queue gap
                 ("d_kernel", t + 37000, t + 40000, 2)]   # 12 us cross-queue gap
    csv = tmp_path / "q_kernel_trace.csv"
    csv.write_text(hdr + "".join(f"{n},{s},{e},256,256,{q}\n" for n, s, e, q in rows))
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "timeline.py"), str(csv), "--chain", "5"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    m = re.search(r"links: (\d+) same-queue \(([\d.]+) us of gaps\), (\d+) cross-queue \(([\d.]+) us", r.stdout)
    assert m, r.stdout
    assert (int(m.group(1)), int(m.group(3))) == (2, 2), r.stdout
    assert abs(float(m.group(2)) - 2.0) < 1e-6 and abs(float(m.group(4)) - 22.0) < 1e-6, r.stdout
