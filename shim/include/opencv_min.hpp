// opencv_min.hpp -- the slice of OpenCV 3.2's core API that the ORB-SLAM2 hot-path classes touch
// (cv::Mat, cv::KeyPoint, cv::Point2f, cv::InputArray/OutputArray), so the shim classes keep the
// reference's signatures (include/ORBextractor.h:77, include/ORBmatcher.h:50,114,116) without
// OpenCV, which this image does not have.  A maintainer building inside ORB-SLAM2 deletes this
// header and includes <opencv2/core/core.hpp> instead: every use below is source-compatible.
//
// Mat is a reference-counted 2-D buffer (CV_8U / CV_32F / CV_64F, one channel): shallow copies
// share data exactly like cv::Mat, clone()/copyTo() deep-copy, row()/rowRange() are views.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <vector>

#ifndef CV_8U
#define CV_8U 0
#define CV_32F 5
#define CV_64F 6
#define CV_8UC1 CV_8U
#define CV_32FC1 CV_32F
#define CV_64FC1 CV_64F
#endif

namespace cv {

typedef unsigned char uchar;

// cv::Point_<T> with OpenCV's typedefs, so signatures mangle as they do against the real header
template <class T>
struct Point_ {
  T x = T(), y = T();
  Point_() = default;
  Point_(T x_, T y_) : x(x_), y(y_) {}
};
typedef Point_<int> Point2i;
typedef Point_<float> Point2f;
typedef Point2i Point;

// cv::KeyPoint: 28 bytes, field order pt, size, angle, response, octave, class_id
class KeyPoint {
 public:
  Point2f pt;
  float size = 0.f;
  float angle = -1.f;
  float response = 0.f;
  int octave = 0;
  int class_id = -1;
  KeyPoint() = default;
  KeyPoint(float x, float y, float size_, float angle_ = -1.f, float response_ = 0.f, int octave_ = 0,
           int class_id_ = -1)
      : pt(x, y), size(size_), angle(angle_), response(response_), octave(octave_), class_id(class_id_) {}
};

inline size_t elem_size(int type) {
  switch (type) {
    case CV_8U: return 1;
    case CV_32F: return 4;
    case CV_64F: return 8;
  }
  throw std::invalid_argument("opencv_min: unsupported Mat type");
}

class Mat {
 public:
  int rows = 0, cols = 0;
  uchar* data = nullptr;
  size_t step = 0;  // bytes per row

  Mat() = default;
  Mat(int r, int c, int type) { create(r, c, type); }
  // wraps external memory (no ownership), like cv::Mat(rows, cols, type, data, step)
  Mat(int r, int c, int type, void* ext, size_t step_ = 0)
      : rows(r), cols(c), data(static_cast<uchar*>(ext)), type_(type) {
    step = step_ ? step_ : (size_t)c * elem_size(type);
  }

  void create(int r, int c, int type) {
    if (buf_ && buf_.use_count() == 1 && rows == r && cols == c && type_ == type) return;
    rows = r;
    cols = c;
    type_ = type;
    step = (size_t)c * elem_size(type);
    buf_ = std::make_shared<std::vector<uchar>>((size_t)r * step);
    data = buf_->data();
  }
  void release() {
    buf_.reset();
    data = nullptr;
    rows = cols = 0;
    step = 0;
  }
  bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
  int type() const { return type_; }
  size_t elemSize() const { return elem_size(type_); }
  bool isContinuous() const { return step == (size_t)cols * elem_size(type_); }

  Mat rowRange(int r0, int r1) const {
    if (r0 < 0 || r1 > rows || r0 > r1) throw std::out_of_range("opencv_min: rowRange");
    Mat m(*this);
    m.rows = r1 - r0;
    m.data = data + (size_t)r0 * step;
    return m;
  }
  Mat row(int r) const { return rowRange(r, r + 1); }
  Mat clone() const {
    Mat m(rows, cols, type_);
    const size_t rb = (size_t)cols * elem_size(type_);
    for (int r = 0; r < rows; r++) std::memcpy(m.data + (size_t)r * m.step, data + (size_t)r * step, rb);
    return m;
  }
  void copyTo(Mat& dst) const {
    if (dst.data == data) return;
    dst.create(rows, cols, type_);
    const size_t rb = (size_t)cols * elem_size(type_);
    for (int r = 0; r < rows; r++) std::memcpy(dst.data + (size_t)r * dst.step, data + (size_t)r * step, rb);
  }
  template <class T> T* ptr(int r = 0) { return reinterpret_cast<T*>(data + (size_t)r * step); }
  template <class T> const T* ptr(int r = 0) const { return reinterpret_cast<const T*>(data + (size_t)r * step); }
  template <class T> T& at(int r, int c) { return ptr<T>(r)[c]; }
  template <class T> const T& at(int r, int c) const { return ptr<T>(r)[c]; }

 private:
  int type_ = CV_8U;
  std::shared_ptr<std::vector<uchar>> buf_;
};

// cv::_InputArray / cv::_OutputArray over a Mat (the only kind the reference passes here)
class _InputArray {
 public:
  _InputArray(const Mat& m) : m_(&m) {}  // NOLINT: implicit like OpenCV
  Mat getMat() const { return *m_; }
  bool empty() const { return m_->empty(); }

 private:
  const Mat* m_;
};
typedef const _InputArray& InputArray;

class _OutputArray {
 public:
  _OutputArray(Mat& m) : m_(&m) {}  // NOLINT: implicit like OpenCV
  void create(int r, int c, int type) const { m_->create(r, c, type); }
  void release() const { m_->release(); }
  Mat& getMatRef() const { return *m_; }
  bool empty() const { return m_->empty(); }

 private:
  Mat* m_;
};
typedef const _OutputArray& OutputArray;

}  // namespace cv
