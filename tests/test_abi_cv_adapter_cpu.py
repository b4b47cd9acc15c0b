"""cv::Mat overloads of the per-model C ABI (csrc/include/abi/cv_adapter.h).

OpenCV is not installed here, so reference-style application code ("pass cv::Mat to RunRAFTStereo") is compiled
against a minimal cv::Mat mock (tests/fixtures/mock_opencv) and linked with stand-ins of the extern "C" exports
that record what they receive: the inputs must arrive as zero-copy views (same data pointer, rows, cols, row
stride, type) and the disparity must come back in the caller's cv::Mat.  All four ABI headers are included in one
translation unit to check the overloads coexist.  Parity with a real cv::Mat is unpinned.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

APP = r"""
#include "abi/RAFTStereoAlgorithm.h"
#include "abi/HitNetAlgorithm.h"
#include "abi/CREStereoAlgorithm.h"
#include "abi/FastACVNet_plus_Algorithm.h"
#include <cstdio>
#include <vector>

// stand-ins for the libraries' C exports: record the views, produce a disparity of the input's size
static const void* g_left = nullptr;
static size_t g_step = 0;
static int g_rows = 0, g_cols = 0, g_type = -1, g_calls = 0;
static int fake_run(sa::Mat& l, sa::Mat& r, float* pc, sa::Mat& d, float base) {
  g_left = l.data, g_step = l.step, g_rows = l.rows, g_cols = l.cols, g_type = l.type();
  ++g_calls;
  if (r.rows != l.rows || pc == nullptr) return -1;
  d.create(l.rows, l.cols, sa::SA_32FC1);
  for (int y = 0; y < d.rows; ++y)
    for (int x = 0; x < d.cols; ++x) d.at<float>(y, x) = base + y * 1000.f + x;
  return 0;
}
extern "C" int RunRAFTStereo(void*, sa::Mat& l, sa::Mat& r, float* pc, sa::Mat& d) { return fake_run(l, r, pc, d, 1.f); }
extern "C" int RunHitNet(void*, sa::Mat& l, sa::Mat& r, float* pc, sa::Mat& d) { return fake_run(l, r, pc, d, 2.f); }
extern "C" int RunCREStereo(void*, sa::Mat& l, sa::Mat& r, float* pc, sa::Mat& d) { return fake_run(l, r, pc, d, 3.f); }
extern "C" int RunCREStereo_RectifyImage(void*, sa::Mat& l, sa::Mat& r, float* pc, sa::Mat& d) { return fake_run(l, r, pc, d, 4.f); }
extern "C" int RunFastACVNet_plus(void*, sa::Mat& l, sa::Mat& r, float* pc, sa::Mat& d) { return fake_run(l, r, pc, d, 5.f); }
extern "C" int RunFastACVNet_plus_RectifyImage(void*, sa::Mat& l, sa::Mat& r, float* pc, sa::Mat& d) { return fake_run(l, r, pc, d, 6.f); }

int main() {
  const int H = 6, W = 10, stride = W * 3 + 16;  // padded rows: a ROI-like cv::Mat
  std::vector<unsigned char> lbuf(H * stride, 7), rbuf(H * stride, 9);
  cv::Mat left(H, W, CV_8UC3, lbuf.data(), stride), right(H, W, CV_8UC3, rbuf.data(), stride), disp;
  std::vector<float> pc(H * W * 6);
  int fails = 0;
  float base = 1.f;
  using Fn = int (*)(void*, cv::Mat&, cv::Mat&, float*, cv::Mat&);  // the reference's signature
  Fn fns[] = {&RunRAFTStereo, &RunHitNet, &RunCREStereo, &RunCREStereo_RectifyImage, &RunFastACVNet_plus,
              &RunFastACVNet_plus_RectifyImage};
  for (Fn f : fns) {
    const int rc = f(nullptr, left, right, pc.data(), disp);
    const bool view_ok = g_left == lbuf.data() && g_step == (size_t)stride && g_rows == H && g_cols == W &&
                         g_type == CV_8UC3;
    const bool out_ok = disp.rows == H && disp.cols == W && disp.type() == CV_32FC1 &&
                        ((float*)disp.ptr(5))[7] == base + 5007.f && ((float*)disp.ptr(0))[0] == base;
    std::printf("rc %d view %d out %d\n", rc, (int)view_ok, (int)out_ok);
    fails += rc != 0 || !view_ok || !out_ok;
    base += 1.f;
  }
  std::printf("calls %d fails %d\n", g_calls, fails);
  return fails == 0 && g_calls == 6 ? 0 : 1;
}
"""


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_cv_mat_overloads(tmp_path):
    src = tmp_path / "app.cpp"
    src.write_text(APP)
    exe = tmp_path / "app"
    cmd = ["g++", "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(ROOT, "csrc", "include"),
           "-I", os.path.join(ROOT, "tests", "fixtures", "mock_opencv"), str(src), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_headers_without_opencv_are_unchanged(tmp_path):
    """Without OpenCV on the include path the headers declare only the sa::Mat C ABI."""
    src = tmp_path / "plain.cpp"
    src.write_text('#include "abi/RAFTStereoAlgorithm.h"\n#ifdef SA_CV_ADAPTER_CORE\n#error adapter active\n#endif\n'
                   'int main() { return 0; }\n')
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", os.path.join(ROOT, "csrc", "include"), str(src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
