// pr/camera.h -- drop-in pr::Camera (reference: src/camera.h:13-57, src/camera.cpp:1-37).
//
// A value type holding image size, K and the world-in-camera pose, with the reference's
// host-side projectPoint/projectPoints.  The PICP hot path never calls these: the kernels
// project on the device (02-visualodometry_amd/csrc/picp_kernels.hip).
#pragma once
#include "pr/defs.h"

namespace pr {

class Camera {
 public:
  EIGEN_MAKE_ALIGNED_OPERATOR_NEW
  Camera(int rows = 100, int cols = 100, const Matrix3f& camera_matrix = Matrix3f::Identity(),
         const Isometry3f& world_in_camera_pose = Isometry3f::Identity())
      : _rows(rows), _cols(cols), _camera_matrix(camera_matrix), _world_in_camera_pose(world_in_camera_pose) {}

  // src/camera.h:24-36
  inline bool projectPoint(Vector2f& image_point, const Vector3f& world_point) const {
    Vector3f camera_point = _world_in_camera_pose * world_point;
    if (camera_point.z() <= 0) return false;
    Vector3f projected_point = _camera_matrix * camera_point;
    const float iz = (float)(1.0 / (double)projected_point.z());
    image_point = Vector2f(projected_point.x() * iz, projected_point.y() * iz);
    if (image_point.x() < 0 || image_point.x() > _cols - 1) return false;
    if (image_point.y() < 0 || image_point.y() > _rows - 1) return false;
    return true;
  }

  // src/camera.cpp:14-35 (invalid points are (-1,-1) when keep_indices)
  int projectPoints(Vector2fVector& image_points, const Vector3fVector& world_points,
                    bool keep_indices = false) const {
    image_points.resize(world_points.size());
    int num_image_points = 0, num_points_inside = 0;
    for (size_t i = 0; i < world_points.size(); i++) {
      Vector2f& image_point = image_points[num_image_points];
      bool is_inside = projectPoint(image_point, world_points[i]);
      if (is_inside)
        num_points_inside++;
      else
        image_point = Vector2f(-1, -1);
      if (keep_indices || is_inside) num_image_points++;
    }
    image_points.resize(num_image_points);
    return num_points_inside;
  }

  inline const Isometry3f& worldInCameraPose() const { return _world_in_camera_pose; }
  inline void setWorldInCameraPose(const Isometry3f& pose) { _world_in_camera_pose = pose; }
  inline const Matrix3f& cameraMatrix() const { return _camera_matrix; }
  // not in the reference (its _rows/_cols are protected): needed to marshal the camera
  inline int rows() const { return _rows; }
  inline int cols() const { return _cols; }

 protected:
  int _rows;
  int _cols;
  Matrix3f _camera_matrix;
  Isometry3f _world_in_camera_pose;
};

}  // namespace pr
