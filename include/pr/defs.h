// pr/defs.h -- types of the drop-in facade (reference: src/defs.h:21-41,209-211).
//
// With Eigen available (and PR_NO_EIGEN undefined) the pr:: types ARE the reference's Eigen
// typedefs, so exec/icp_test.cpp-style callers compile unchanged.  Without Eigen (this image
// has none) minimal layout-compatible PODs stand in: Vector3f = 3 packed floats, Vector2f = 2,
// Matrix3f / Isometry3f column-major, IntPair = std::pair<int,int> -- exactly the memory the
// C-ABI (include/picp_c.h) reads.
#pragma once
#include <cmath>
#include <algorithm>
#include <cstring>
#include <utility>
#include <vector>

#if !defined(PR_NO_EIGEN) && __has_include(<Eigen/Core>)
#include <Eigen/Core>
#include <Eigen/Geometry>
#include <Eigen/StdVector>
#define PR_HAVE_EIGEN 1
namespace pr {
typedef Eigen::Vector2f Vector2f;
typedef Eigen::Vector3f Vector3f;
typedef Eigen::Matrix3f Matrix3f;
typedef Eigen::Isometry3f Isometry3f;
typedef std::vector<Eigen::Vector3f, Eigen::aligned_allocator<Eigen::Vector3f> > Vector3fVector;
typedef std::vector<Eigen::Vector2f, Eigen::aligned_allocator<Eigen::Vector2f> > Vector2fVector;
inline const float* data16(const Isometry3f& T) { return T.matrix().data(); }
inline Isometry3f iso_from16(const float* p) {
  Isometry3f T;
  std::memcpy(T.matrix().data(), p, 16 * sizeof(float));
  return T;
}
inline const float* data9(const Matrix3f& K) { return K.data(); }
}  // namespace pr
#else
#define PR_HAVE_EIGEN 0
// the reference's classes carry Eigen's aligned operator new (src/picp_solver.h:23,
// src/camera.h:14); the POD stand-ins need no over-alignment
#ifndef EIGEN_MAKE_ALIGNED_OPERATOR_NEW
#define EIGEN_MAKE_ALIGNED_OPERATOR_NEW
#endif
namespace pr {

struct Vector2f {
  float v[2] = {0.f, 0.f};
  Vector2f() = default;
  Vector2f(float x, float y) : v{x, y} {}
  float& x() { return v[0]; }
  float& y() { return v[1]; }
  float x() const { return v[0]; }
  float y() const { return v[1]; }
  float& operator[](int i) { return v[i]; }
  float operator[](int i) const { return v[i]; }
  const float* data() const { return v; }
};

struct Vector3f {
  float v[3] = {0.f, 0.f, 0.f};
  Vector3f() = default;
  Vector3f(float x, float y, float z) : v{x, y, z} {}
  float& x() { return v[0]; }
  float& y() { return v[1]; }
  float& z() { return v[2]; }
  float x() const { return v[0]; }
  float y() const { return v[1]; }
  float z() const { return v[2]; }
  float& operator[](int i) { return v[i]; }
  float operator[](int i) const { return v[i]; }
  float norm() const { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
  Vector3f operator-(const Vector3f& o) const { return {v[0] - o.v[0], v[1] - o.v[1], v[2] - o.v[2]}; }
  Vector3f operator*(float s) const { return {v[0] * s, v[1] * s, v[2] * s}; }
  const float* data() const { return v; }
};

// column-major 3x3 (Eigen::Matrix3f layout)
struct Matrix3f {
  float m[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  static Matrix3f Identity() { return Matrix3f(); }
  float& operator()(int r, int c) { return m[c * 3 + r]; }
  float operator()(int r, int c) const { return m[c * 3 + r]; }
  Vector3f operator*(const Vector3f& p) const {
    Vector3f o;
    for (int i = 0; i < 3; ++i) o[i] = ((*this)(i, 0) * p[0] + (*this)(i, 1) * p[1]) + (*this)(i, 2) * p[2];
    return o;
  }
  Matrix3f operator*(const Matrix3f& B) const {
    Matrix3f C;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) C(i, j) = ((*this)(i, 0) * B(0, j) + (*this)(i, 1) * B(1, j)) + (*this)(i, 2) * B(2, j);
    return C;
  }
  Matrix3f transpose() const {
    Matrix3f T;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) T(i, j) = (*this)(j, i);
    return T;
  }
  const float* data() const { return m; }
};

// rigid transform, column-major 4x4 (Eigen::Isometry3f memory)
struct Isometry3f {
  float m[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  static Isometry3f Identity() { return Isometry3f(); }
  float& operator()(int r, int c) { return m[c * 4 + r]; }
  float operator()(int r, int c) const { return m[c * 4 + r]; }
  Matrix3f linear() const {
    Matrix3f R;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) R(i, j) = (*this)(i, j);
    return R;
  }
  Matrix3f rotation() const { return linear(); }
  void setLinear(const Matrix3f& R) {
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) (*this)(i, j) = R(i, j);
  }
  Vector3f translation() const { return {m[12], m[13], m[14]}; }
  void setTranslation(const Vector3f& t) {
    m[12] = t[0];
    m[13] = t[1];
    m[14] = t[2];
  }
  Vector3f operator*(const Vector3f& p) const {  // linear()*p + translation()
    Vector3f o;
    for (int i = 0; i < 3; ++i) o[i] = (((*this)(i, 0) * p[0] + (*this)(i, 1) * p[1]) + (*this)(i, 2) * p[2]) + (*this)(i, 3);
    return o;
  }
  Isometry3f operator*(const Isometry3f& B) const {
    Isometry3f C;
    C.setLinear(linear() * B.linear());
    Vector3f t = linear() * B.translation();
    C.setTranslation({t[0] + m[12], t[1] + m[13], t[2] + m[14]});
    return C;
  }
  // the Eigen calls the reference makes on poses (src/cam.cpp:185,220; exec/icp_test.cpp:115)
  const Isometry3f& matrix() const { return *this; }
  bool isApprox(const Isometry3f& o, float prec = 1e-5f) const {  // Eigen's Frobenius-norm rule
    double d = 0, a = 0, b = 0;
    for (int i = 0; i < 16; ++i) {
      d += (double)(m[i] - o.m[i]) * (m[i] - o.m[i]);
      a += (double)m[i] * m[i];
      b += (double)o.m[i] * o.m[i];
    }
    return std::sqrt(d) <= prec * std::sqrt(std::min(a, b));
  }
  Isometry3f inverse() const {
    Isometry3f I;
    Matrix3f Rt = linear().transpose();
    I.setLinear(Rt);
    Vector3f t = Rt * translation();
    I.setTranslation({-t[0], -t[1], -t[2]});
    return I;
  }
  const float* data() const { return m; }
};

typedef std::vector<Vector3f> Vector3fVector;
typedef std::vector<Vector2f> Vector2fVector;
inline const float* data16(const Isometry3f& T) { return T.m; }
inline Isometry3f iso_from16(const float* p) {
  Isometry3f T;
  std::memcpy(T.m, p, 16 * sizeof(float));
  return T;
}
inline const float* data9(const Matrix3f& K) { return K.m; }
static_assert(sizeof(Vector3f) == 12 && sizeof(Vector2f) == 8, "packed vector layout");
static_assert(sizeof(Isometry3f) == 64 && sizeof(Matrix3f) == 36, "matrix layout");
}  // namespace pr
#endif

namespace pr {
typedef std::pair<int, int> IntPair;          // src/defs.h:209 (first = image, second = world)
typedef std::vector<IntPair> IntPairVector;   // src/defs.h:211
static_assert(sizeof(IntPair) == 8, "IntPair must be two packed int32");
}  // namespace pr
