// Test scaffold (see cam_like.h): the by-value member patterns of the reference's src/cam.cpp.
#include "cam_like.h"

#include <iostream>

CamLike::CamLike(const pr::Matrix3f& K) : K_eig(K) {
  // src/cam.cpp:33-34: assignment of temporaries to by-value members
  picp_cam = pr::Camera(480, 640, K_eig, pr::Isometry3f::Identity());
  picp_solver = pr::PICPSolver();
}

void CamLike::initOneRound(std::vector<TestWorldPoint> world_points, std::vector<TestDataPoint> img_points) {
  _world_points_picp.clear();
  for (const auto& w : world_points) _world_points_picp.emplace_back(w.x, w.y, w.z);  // extract_V3fV
  _image_points_picp.clear();
  for (const auto& d : img_points) _image_points_picp.emplace_back(d.u, d.v);  // extract_V2fV
  picp_solver.init(picp_cam, _world_points_picp, _image_points_picp);
  picp_solver.setKernelThreshold(1000.0f);
  if (!picp_cam.worldInCameraPose().isApprox(picp_solver.camera().worldInCameraPose()))
    std::cerr << "CamLike::initOneRound: camera poses are different" << std::endl;
}

bool CamLike::oneRound(pr::IntPairVector correspondences) {
  bool ok = true;
  for (int i = 0; i < 5; i++) ok = picp_solver.oneRound(correspondences, false) && ok;
  picp_cam = picp_solver.camera();
  return ok && picp_cam.worldInCameraPose().isApprox(picp_solver.camera().worldInCameraPose());
}
