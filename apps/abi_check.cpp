// abi_check — executes the reference-compatible C ABI of all four model libraries end to end and prints
// one JSON line per library (tests/test_demos_gpu.py).  The reference's only "tests" are its demos
// (RAFTStereo/test/main.cpp:8-39, CREStereo/test/main.cpp:55-72), which call Initialize -> Run* -> Release;
// this checks the observable contract of those calls:
//   * Initialize returns NULL for a missing calibration file (documented deviation: the reference returns
//     a handle that is not initialised, RAFTStereoAlgorithm.cpp:133-138);
//   * RunRAFTStereo / RunHitNet rectify the caller's images in place (RAFTStereoAlgorithm.cpp:57-72);
//     RunCREStereo / RunFastACVNet_plus do not, their _RectifyImage variants do
//     (CREStereoAlgorithm.cpp:59-91);
//   * disparity comes back as an H x W CV_32FC1 Mat, pointcloud as H*W*6 floats whose XYZ are finite where
//     the disparity is positive, and Version returns "<Model>Algorithm_V1.0".
// All four libraries export the same symbol names, so each is dlopen'ed RTLD_LOCAL and resolved by dlsym.
//
//   abi_check <lib_dir> <left.jpg> <right.jpg> <StereoCalibration.yml> [frames]
#include <dlfcn.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "sa/imgio.h"
#include "sa/mat.h"

typedef void* (*init_fn)(char*, int, char*);
typedef int (*run_fn)(void*, sa::Mat&, sa::Mat&, float*, sa::Mat&);
typedef const char* (*ver_fn)(void*);
typedef int (*rel_fn)(void*);

struct LibSpec {
  const char* lib;
  const char* run;           // plain Run entry
  const char* run_rectify;   // _RectifyImage entry (nullptr: the plain entry rectifies)
  bool plain_rectifies;
  const char* version;
};

static bool same(const sa::Mat& a, const sa::Mat& b) {
  return a.rows == b.rows && a.cols == b.cols && std::memcmp(a.data, b.data, a.step * a.rows) == 0;
}

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: abi_check <lib_dir> <left> <right> <calib.yml> [frames]\n");
    return 2;
  }
  const std::string dir = argv[1], calib = argv[4];
  const int frames = argc > 5 ? std::atoi(argv[5]) : 2;
  const sa::Mat L = sa::imread(argv[2]), R = sa::imread(argv[3]);
  if (L.empty() || R.empty()) {
    std::fprintf(stderr, "cannot read inputs\n");
    return 2;
  }
  const LibSpec specs[] = {
      {"libRAFTStereo.so", "RunRAFTStereo", nullptr, true, "RAFTStereoAlgorithm_V1.0"},
      {"libHitNet.so", "RunHitNet", nullptr, true, "HitNetAlgorithm_V1.0"},
      {"libCREStereo.so", "RunCREStereo", "RunCREStereo_RectifyImage", false, "CREStereoAlgorithm_V1.0"},
      {"libFastACVNet_plus.so", "RunFastACVNet_plus", "RunFastACVNet_plus_RectifyImage", false,
       "FastACVNet_plus_Algorithm_V1.0"},
  };
  int failures = 0;
  for (const LibSpec& s : specs) {
    const std::string path = dir + "/" + s.lib;
    void* so = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!so) {
      std::printf("{\"lib\": \"%s\", \"ok\": false, \"error\": \"dlopen: %s\"}\n", s.lib, dlerror());
      ++failures;
      continue;
    }
    auto init = (init_fn)dlsym(so, "Initialize");
    auto run = (run_fn)dlsym(so, s.run);
    auto runr = s.run_rectify ? (run_fn)dlsym(so, s.run_rectify) : nullptr;
    auto ver = (ver_fn)dlsym(so, "Version");
    auto rel = (rel_fn)dlsym(so, "Release");
    std::string err;
    bool missing_null = false, version_ok = false, plain_rect_ok = false, rect_ok = true, shapes_ok = false;
    long finite_disp = 0, positive = 0, bad_xyz = 0;
    double mean_disp = 0;
    if (!init || !run || !ver || !rel || (s.run_rectify && !runr)) {
      err = "missing symbol";
    } else {
      missing_null = init((char*)"", 0, (char*)"/nonexistent/StereoCalibration.yml") == nullptr;
      void* h = init((char*)"", 0, (char*)calib.c_str());
      if (!h) {
        err = "Initialize failed";
      } else {
        version_ok = std::strcmp(ver(h), s.version) == 0;
        std::vector<float> pc((size_t)L.rows * L.cols * 6, NAN);
        sa::Mat disp, l1, r1;
        int rc = 0;
        for (int f = 0; f < frames && rc == 0; ++f) {
          l1 = L.clone();
          r1 = R.clone();
          rc = run(h, l1, r1, pc.data(), disp);
        }
        // plain entry: rectifies in place for RAFT / HitNet, leaves the inputs untouched otherwise
        plain_rect_ok = rc == 0 && (s.plain_rectifies ? (!same(l1, L) && !same(r1, R)) : (same(l1, L) && same(r1, R)));
        if (rc == 0 && runr) {
          sa::Mat l2 = L.clone(), r2 = R.clone(), d2;
          rc = runr(h, l2, r2, pc.data(), d2);
          rect_ok = rc == 0 && !same(l2, L) && !same(r2, R) && d2.rows == L.rows && d2.cols == L.cols;
        }
        if (rc != 0) err = "Run returned " + std::to_string(rc);
        shapes_ok = disp.rows == L.rows && disp.cols == L.cols && disp.type() == sa::SA_32FC1;
        if (shapes_ok) {
          for (int y = 0; y < disp.rows; ++y)
            for (int x = 0; x < disp.cols; ++x) {
              const float d = disp.ptr<float>(y)[x];
              if (!std::isfinite(d)) continue;
              ++finite_disp;
              mean_disp += d;
              if (d > 0) {
                ++positive;
                const float* p = &pc[((size_t)y * disp.cols + x) * 6];
                if (!std::isfinite(p[0]) || !std::isfinite(p[1]) || !std::isfinite(p[2])) ++bad_xyz;
              }
            }
          mean_disp /= std::max<long>(1, finite_disp);
        }
        rel(h);
      }
    }
    const bool ok = err.empty() && missing_null && version_ok && plain_rect_ok && rect_ok && shapes_ok &&
                    finite_disp == (long)L.rows * L.cols && bad_xyz == 0;
    failures += !ok;
    std::printf("{\"lib\": \"%s\", \"ok\": %s, \"error\": \"%s\", \"missing_calib_null\": %s, \"version_ok\": %s, "
                "\"plain_entry_rectify_semantics\": %s, \"rectify_entry_ok\": %s, \"shape_ok\": %s, "
                "\"finite\": %ld, \"positive\": %ld, \"bad_xyz\": %ld, \"mean_disparity\": %.4f}\n",
                s.lib, ok ? "true" : "false", err.c_str(), missing_null ? "true" : "false",
                version_ok ? "true" : "false", plain_rect_ok ? "true" : "false", rect_ok ? "true" : "false",
                shapes_ok ? "true" : "false", finite_disp, positive, bad_xyz, mean_disp);
    std::fflush(stdout);
    dlclose(so);
  }
  return failures ? 1 : 0;
}
