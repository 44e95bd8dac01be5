// Test scaffold written from the reference's INTERFACE (src/cam.h:17-158, src/cam.cpp:10-232):
// a class that holds pr::Camera and pr::PICPSolver BY VALUE, assigns them in its constructor and
// re-initialises the solver from by-value point vectors, as Cam does.  It reaches the solver only
// through `#include "picp_solver.h"` / `"camera.h"`, i.e. through include/ref_src/'s shims
// copied into this tree -- the transitive include path of src/cam.h:6-7.
#pragma once
#include <vector>

#include "camera.h"
#include "defs.h"
#include "picp_solver.h"

struct TestDataPoint {  // the coordinates part of Data_Point (src/data_point.h)
  float u, v;
};
struct TestWorldPoint {  // the coordinates part of World_Point (src/data_point.h)
  float x, y, z;
};

class CamLike {
 public:
  EIGEN_MAKE_ALIGNED_OPERATOR_NEW
  explicit CamLike(const pr::Matrix3f& K);
  // src/cam.cpp:179-189: pack the by-value arguments into members, init, threshold 1000
  void initOneRound(std::vector<TestWorldPoint> world_points, std::vector<TestDataPoint> img_points);
  // src/cam.cpp:191-224: five rounds without outliers, then copy the solver's camera back
  bool oneRound(pr::IntPairVector correspondences);
  pr::Isometry3f getPose() const { return picp_cam.worldInCameraPose(); }
  void setPose(const pr::Isometry3f& pose) { picp_cam.setWorldInCameraPose(pose); }
  int numInliers() const { return picp_solver.numInliers(); }

 private:
  pr::Matrix3f K_eig;
  pr::Vector3fVector _world_points_picp;
  pr::Vector2fVector _image_points_picp;
  pr::Camera picp_cam;
  pr::PICPSolver picp_solver;
};
