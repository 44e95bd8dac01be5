// pr/triangulation.h -- Cam::triangulatePoints' arithmetic (reference src/cam.cpp:94-140:
// P_k = K * inverse(T_k)(0:3,0:4), cv::triangulatePoints + convertPointsFromHomogeneous) on the
// GPU through the C-ABI.  T1/T2 are camera-in-world poses, as in the reference.
#pragma once
#include <vector>

#include "picp_c.h"
#include "pr/defs.h"

namespace pr {

// Returns a PICP_* status; out receives one point per input pair (no cheirality check, as
// in the reference).
inline int triangulatePoints(const Matrix3f& K, const Isometry3f& T1, const Isometry3f& T2,
                             const Vector2fVector& points1, const Vector2fVector& points2,
                             Vector3fVector& out, int device = 0) {
  if (points1.size() != points2.size()) return PICP_ERR_ARG;
  float P1[12], P2[12];
  int rc = picp_projection_matrix(data9(K), data16(T1), P1);
  if (rc) return rc;
  rc = picp_projection_matrix(data9(K), data16(T2), P2);
  if (rc) return rc;
  out.resize(points1.size());
  if (points1.empty()) return PICP_OK;
  return picp_triangulate(device, P1, P2, reinterpret_cast<const float*>(points1.data()),
                          reinterpret_cast<const float*>(points2.data()), (int64_t)points1.size(),
                          reinterpret_cast<float*>(out.data()));
}

}  // namespace pr
