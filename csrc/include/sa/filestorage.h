// OpenCV-FileStorage-compatible YAML (subset) for calibration files.
//
// Reads / writes the `%YAML:1.0` + `!!opencv-matrix` format produced by the reference calibration
// tool (Stereo_Calibration/Stereo_Calibration.cpp:165-179) and consumed by every facade
// (RAFTStereo/src/RAFTStereoAlgorithm.cpp:79-95): top-level `key: !!opencv-matrix` maps with
// rows / cols / dt / data, flow sequences (`validROIL: [ 0, 0, 640, 480 ]`) and scalars.  The
// writer reproduces OpenCV's number formatting ("%.16e", integral values as "1.") and its
// 71-column flow wrapping so files round-trip byte-for-byte.  Also reads the OpenCV XML
// `<imagelist>` used by Stereo_Calibration/stereo_calib.xml.
#pragma once
#include <map>
#include <string>
#include <vector>

#include "sa/mat.h"

namespace sa {

struct FsNode {
  enum Kind { kNone, kScalar, kSeq, kMat } kind = kNone;
  std::string scalar;              // kScalar
  std::vector<std::string> seq;    // kSeq (raw item tokens)
  Mat mat;                         // kMat
  bool empty() const { return kind == kNone; }
  double real() const;
  int integer() const { return (int)real(); }
  std::string str() const { return scalar; }
  std::vector<double> reals() const;
};

class FileStorage {
 public:
  enum Mode { READ = 0, WRITE = 1 };
  FileStorage() = default;
  FileStorage(const std::string& path, int mode) { open(path, mode); }
  ~FileStorage() { release(); }
  bool open(const std::string& path, int mode);
  bool isOpened() const { return opened_; }
  void release();

  // READ: missing keys give an empty node (the reference leaves the Mat empty)
  FsNode operator[](const std::string& key) const;
  std::vector<std::string> keys() const { return order_; }
  static FileStorage from_string(const std::string& text);

  // WRITE
  void write(const std::string& key, const Mat& m);
  void write(const std::string& key, double v);
  void write(const std::string& key, int v);
  void write(const std::string& key, const std::string& s);
  void write_seq(const std::string& key, const std::vector<int>& v);
  std::string text() const { return out_; }

 private:
  void parse(const std::string& text);
  bool opened_ = false;
  int mode_ = READ;
  std::string path_, out_;
  std::map<std::string, FsNode> nodes_;
  std::vector<std::string> order_;
};

// OpenCV's icvDoubleToString formatting
std::string fs_format_double(double v);
// <imagelist> of an OpenCV XML file (Stereo_Calibration.cpp:53-66 readStringList)
bool read_string_list(const std::string& path, std::vector<std::string>& out);

}  // namespace sa
