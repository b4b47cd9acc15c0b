// Minimal dense image/matrix container with OpenCV-compatible type codes.
//
// The reference's C ABI passes `cv::Mat&` (RAFTStereo/include/RAFTStereoAlgorithm.h:24-39) and its
// facades read `cv::FileStorage` matrices (RAFTStereo/src/RAFTStereoAlgorithm.cpp:79-95).  OpenCV is
// not part of this stack, so `sa::Mat` provides the subset those call sites rely on: rows / cols /
// type() / data / step, CV_8UC3 / CV_32FC1 / CV_64FC1 semantics, shared ownership on copy and
// clone() for a deep copy.  Type codes equal OpenCV's CV_MAKETYPE values so files and FFI callers
// agree on them.
#pragma once
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <vector>

namespace sa {

enum MatDepth { SA_8U = 0, SA_8S = 1, SA_16U = 2, SA_16S = 3, SA_32S = 4, SA_32F = 5, SA_64F = 6 };
constexpr int sa_maketype(int depth, int cn) { return depth + ((cn - 1) << 3); }
enum MatType : int {
  SA_8UC1 = sa_maketype(SA_8U, 1),
  SA_8UC3 = sa_maketype(SA_8U, 3),
  SA_16SC2 = sa_maketype(SA_16S, 2),
  SA_32FC1 = sa_maketype(SA_32F, 1),
  SA_32FC2 = sa_maketype(SA_32F, 2),
  SA_32FC3 = sa_maketype(SA_32F, 3),
  SA_32FC6 = sa_maketype(SA_32F, 6),
  SA_64FC1 = sa_maketype(SA_64F, 1),
};

inline int depth_size(int depth) {
  static const int sz[] = {1, 1, 2, 2, 4, 4, 8};
  return sz[depth & 7];
}

class Mat {
 public:
  int rows = 0, cols = 0;
  uint8_t* data = nullptr;
  size_t step = 0;  // bytes per row

  Mat() = default;
  Mat(int r, int c, int type) { create(r, c, type); }
  Mat(int r, int c, int type, double fill) {
    create(r, c, type);
    setTo(fill);
  }
  // non-owning view over caller memory (like cv::Mat(rows, cols, type, data))
  Mat(int r, int c, int type, void* ext, size_t step_bytes = 0)
      : rows(r), cols(c), data(static_cast<uint8_t*>(ext)), type_(type) {
    step = step_bytes ? step_bytes : (size_t)c * elemSize();
  }

  void create(int r, int c, int type) {
    if (r == rows && c == cols && type == type_ && buf_ && buf_.use_count() == 1) return;
    rows = r;
    cols = c;
    type_ = type;
    step = (size_t)c * elemSize();
    buf_ = std::make_shared<std::vector<uint8_t>>(step * (size_t)r);
    data = buf_->data();
  }
  int type() const { return type_; }
  int depth() const { return type_ & 7; }
  int channels() const { return (type_ >> 3) + 1; }
  size_t elemSize1() const { return (size_t)depth_size(depth()); }
  size_t elemSize() const { return elemSize1() * channels(); }
  size_t total() const { return (size_t)rows * cols; }
  bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
  bool isContinuous() const { return step == (size_t)cols * elemSize(); }

  template <typename T>
  T* ptr(int r = 0) {
    return reinterpret_cast<T*>(data + (size_t)r * step);
  }
  template <typename T>
  const T* ptr(int r = 0) const {
    return reinterpret_cast<const T*>(data + (size_t)r * step);
  }
  template <typename T>
  T& at(int r, int c) {
    return ptr<T>(r)[c];
  }
  template <typename T>
  const T& at(int r, int c) const {
    return ptr<T>(r)[c];
  }
  // element i of a continuous single-channel matrix (row-major)
  double get(int i) const {
    const int r = i / cols, c = i % cols;
    switch (depth()) {
      case SA_8U: return at<uint8_t>(r, c);
      case SA_16S: return at<int16_t>(r, c);
      case SA_32S: return at<int32_t>(r, c);
      case SA_32F: return at<float>(r, c);
      case SA_64F: return at<double>(r, c);
      default: throw std::runtime_error("Mat::get: unsupported depth");
    }
  }

  Mat clone() const {
    Mat m(rows, cols, type_);
    for (int r = 0; r < rows; ++r) std::memcpy(m.data + r * m.step, data + r * step, (size_t)cols * elemSize());
    return m;
  }
  void copyTo(Mat& dst) const {
    if (dst.rows != rows || dst.cols != cols || dst.type() != type_) dst.create(rows, cols, type_);
    for (int r = 0; r < rows; ++r) std::memcpy(dst.data + r * dst.step, data + r * step, (size_t)cols * elemSize());
  }
  void setTo(double v) {
    for (int r = 0; r < rows; ++r)
      for (int c = 0; c < cols * channels(); ++c) {
        switch (depth()) {
          case SA_8U: ptr<uint8_t>(r)[c] = (uint8_t)v; break;
          case SA_16S: ptr<int16_t>(r)[c] = (int16_t)v; break;
          case SA_32S: ptr<int32_t>(r)[c] = (int32_t)v; break;
          case SA_32F: ptr<float>(r)[c] = (float)v; break;
          case SA_64F: ptr<double>(r)[c] = v; break;
          default: break;
        }
      }
  }
  // single-channel conversion to double / float (returns a new continuous matrix)
  Mat toF64() const {
    Mat m(rows, cols, sa_maketype(SA_64F, channels()));
    for (int r = 0; r < rows; ++r)
      for (int c = 0; c < cols * channels(); ++c) m.ptr<double>(r)[c] = elem(r, c);
    return m;
  }
  Mat toF32() const {
    Mat m(rows, cols, sa_maketype(SA_32F, channels()));
    for (int r = 0; r < rows; ++r)
      for (int c = 0; c < cols * channels(); ++c) m.ptr<float>(r)[c] = (float)elem(r, c);
    return m;
  }
  static Mat eye(int n) {
    Mat m(n, n, SA_64FC1, 0.0);
    for (int i = 0; i < n; ++i) m.at<double>(i, i) = 1.0;
    return m;
  }

 private:
  double elem(int r, int c) const {  // c indexes channels-interleaved columns
    switch (depth()) {
      case SA_8U: return ptr<uint8_t>(r)[c];
      case SA_8S: return ptr<int8_t>(r)[c];
      case SA_16U: return ptr<uint16_t>(r)[c];
      case SA_16S: return ptr<int16_t>(r)[c];
      case SA_32S: return ptr<int32_t>(r)[c];
      case SA_32F: return ptr<float>(r)[c];
      case SA_64F: return ptr<double>(r)[c];
      default: return 0.0;
    }
  }
  int type_ = 0;
  std::shared_ptr<std::vector<uint8_t>> buf_;
};

}  // namespace sa
