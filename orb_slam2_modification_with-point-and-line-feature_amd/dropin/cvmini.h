// Minimal stand-ins for the OpenCV / opencv_contrib / Eigen types that appear
// in the reference's hot-path signatures (ORBextractor.h:51-85,
// LineExtractor.h:25-30, ORBmatcher.h, LineMatcher.h, Optimizer.h:121,234).
// They exist so that the drop-in classes in this directory compile with the
// reference's exact method signatures and can be linked and tested here,
// where OpenCV and Eigen are absent. A maintainer integrating into the
// reference deletes this header and includes OpenCV / Eigen instead: the
// field layouts of KeyPoint (28 B) and KeyLine (68 B) are those of OpenCV 3.4
// and opencv_contrib 3.4, which is what the static_asserts in the .cc files
// check against the C ABI (include/orbpl.h).
#pragma once
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <vector>

namespace cv {

enum { CV_8U = 0, CV_8UC1 = 0, CV_32F = 5 };

struct Point2f {
  float x = 0, y = 0;
};

struct KeyPoint {           // cv::KeyPoint field order (OpenCV 3.4)
  Point2f pt;
  float size = 0, angle = -1, response = 0;
  int octave = 0, class_id = -1;
};

// Row-major 2-D array of u8 or f32 with shared storage, like cv::Mat.
class Mat {
 public:
  int rows = 0, cols = 0;
  size_t step = 0;          // bytes per row
  uint8_t* data = nullptr;

  Mat() = default;
  Mat(int r, int c, int type) { create(r, c, type); }
  Mat(int r, int c, int type, void* ext, size_t st = 0)
      : rows(r), cols(c), step(st ? st : (size_t)c * esize(type)), data((uint8_t*)ext), type_(type) {}

  static size_t esize(int type) { return type == CV_32F ? 4 : 1; }
  static Mat eye(int r, int c, int type) {
    Mat m(r, c, type);
    for (int i = 0; i < r && i < c; i++) {
      if (type == CV_32F) m.at<float>(i, i) = 1.f;
      else m.at<uint8_t>(i, i) = 1;
    }
    return m;
  }
  int type() const { return type_; }
  bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
  void create(int r, int c, int type) {
    if (r == rows && c == cols && type == type_ && store_) return;
    rows = r;
    cols = c;
    type_ = type;
    step = (size_t)c * esize(type);
    store_ = std::make_shared<std::vector<uint8_t>>((size_t)r * step, 0);
    data = store_->data();
  }
  void release() { *this = Mat(); }
  Mat clone() const {
    Mat m(rows, cols, type_);
    for (int i = 0; i < rows; i++) std::memcpy(m.data + i * m.step, data + i * step, m.step);
    return m;
  }
  void copyTo(Mat& o) const { o = clone(); }
  Mat rowRange(int a, int b) const {
    Mat m = *this;
    m.rows = b - a;
    m.data = data + (size_t)a * step;
    return m;
  }
  Mat row(int i) const { return rowRange(i, i + 1); }
  template <class T> T* ptr(int r = 0) { return reinterpret_cast<T*>(data + (size_t)r * step); }
  template <class T> const T* ptr(int r = 0) const {
    return reinterpret_cast<const T*>(data + (size_t)r * step);
  }
  template <class T> T& at(int r, int c) { return ptr<T>(r)[c]; }
  template <class T> const T& at(int r, int c) const { return ptr<T>(r)[c]; }
  bool isContinuous() const { return step == (size_t)cols * esize(type_); }

 private:
  int type_ = CV_8U;
  std::shared_ptr<std::vector<uint8_t>> store_;
};

// _InputArray / _OutputArray reduced to what the hot path uses
class InputArray {
 public:
  InputArray(const Mat& m) : m_(&m) {}   // NOLINT: implicit, as in OpenCV
  Mat getMat() const { return *m_; }
  bool empty() const { return m_->empty(); }

 private:
  const Mat* m_;
};

class OutputArray {
 public:
  OutputArray(Mat& m) : m_(&m) {}        // NOLINT
  void create(int r, int c, int type) { m_->create(r, c, type); }
  Mat& getMatRef() { return *m_; }
  void release() { m_->release(); }

 private:
  Mat* m_;
};

namespace line_descriptor {
struct KeyLine {            // opencv_contrib 3.4 line_descriptor::KeyLine
  float angle = 0;
  int class_id = 0;
  int octave = 0;
  Point2f pt;
  float response = 0, size = 0;
  float startPointX = 0, startPointY = 0, endPointX = 0, endPointY = 0;
  float sPointInOctaveX = 0, sPointInOctaveY = 0, ePointInOctaveX = 0, ePointInOctaveY = 0;
  float lineLength = 0;
  int numOfPixels = 0;
};
}  // namespace line_descriptor

}  // namespace cv

namespace Eigen {
struct Vector3d {
  double v[3] = {0, 0, 0};
  Vector3d() = default;
  Vector3d(double a, double b, double c) : v{a, b, c} {}
  double& operator[](int i) { return v[i]; }
  double operator[](int i) const { return v[i]; }
};
}  // namespace Eigen
