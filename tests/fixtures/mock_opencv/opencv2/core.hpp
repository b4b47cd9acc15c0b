// Minimal stand-in for OpenCV's cv::Mat (just the members abi/cv_adapter.h touches, with OpenCV's shapes: a
// MStep row stride convertible to size_t, CV_MAKETYPE type codes, owning create()).  Test fixture only:
// tests/test_abi_cv_adapter_cpu.py compiles the ABI headers against it because OpenCV is not installed.
#pragma once
#include <cstddef>
#include <memory>
#include <vector>

#define CV_8U 0
#define CV_32F 5
#define CV_MAKETYPE(depth, cn) ((depth) + (((cn) - 1) << 3))
#define CV_8UC3 CV_MAKETYPE(CV_8U, 3)
#define CV_32FC1 CV_MAKETYPE(CV_32F, 1)

namespace cv {
class Mat {
 public:
  struct MStep {
    size_t p[2] = {0, 0};
    operator size_t() const { return p[0]; }
  };
  int rows = 0, cols = 0;
  unsigned char* data = nullptr;
  MStep step;

  Mat() = default;
  Mat(int r, int c, int type) { create(r, c, type); }
  Mat(int r, int c, int type, void* ext, size_t stride) : rows(r), cols(c), data((unsigned char*)ext), type_(type) {
    step.p[0] = stride;
  }
  void create(int r, int c, int type) {
    if (r == rows && c == cols && type == type_ && buf_) return;
    rows = r, cols = c, type_ = type;
    step.p[0] = (size_t)c * elemSize();
    buf_ = std::make_shared<std::vector<unsigned char>>(step.p[0] * r);
    data = buf_->data();
  }
  int type() const { return type_; }
  size_t elemSize() const { return (size_t)(((type_ >> 3) + 1) * ((type_ & 7) == CV_32F ? 4 : 1)); }
  bool empty() const { return data == nullptr || rows == 0; }
  unsigned char* ptr(int r) { return data + (size_t)r * step.p[0]; }

 private:
  int type_ = 0;
  std::shared_ptr<std::vector<unsigned char>> buf_;
};
}  // namespace cv
