// pr/picp_solver.h -- drop-in pr::PICPSolver (reference: src/picp_solver.h:21-82,
// src/picp_solver.cpp:8-105) over the C-ABI of libpicp_amd.so (include/picp_c.h).
//
// Same names, argument meaning and return values as the reference.  The reference's own sources
// (exec/icp_test.cpp, src/cam.cpp, src/my_utilities.cpp) reach the solver through
// `#include "picp_solver.h"` / `"camera.h"` inside src/; include/ref_src/ holds the two one-line
// headers that replace those files, so every caller compiles against this class unchanged
// (INTEGRATION.md §2).  Differences, all deliberate:
//   * init() COPIES world/image points to device memory (the reference keeps raw pointers to
//     them, src/picp_solver.cpp:21-22, and icp_test passes temporaries: use-after-free).
//   * linearize + damped LDLT + update run on the GPU (picp_kernels.hip); oneRound() is one
//     device round trip.  solve() runs the whole exec/icp_test.cpp:88-107 loop on the device.
//   * copies get their own device handle with copies of the points (picp_clone); moves hand the
//     handle over.  The reference's implicit copy shares the caller's arrays instead.
//   * errors from the device are reported on std::cerr and make oneRound() return false;
//     lastStatus() gives the C-ABI status code.
// Header-only: no C++ types cross the library boundary.
#pragma once
#include <cstdint>
#include <iostream>

#include "picp_c.h"
#include "pr/camera.h"
#include "pr/defs.h"

namespace pr {

class PICPSolver {
 public:
  EIGEN_MAKE_ALIGNED_OPERATOR_NEW

  //! src/picp_solver.cpp:8-15 (no handle yet: the device state is created by the first init)
  PICPSolver() : PICPSolver(0) {}
  explicit PICPSolver(int device) : _device(device) {
    _kernel_thereshold = 1000;  // src/picp_solver.cpp:14
    _damping = 1;               // :11
    _min_num_inliers = 0;       // :12
  }
  ~PICPSolver() { picp_destroy(_h); }

  // Value semantics like the reference class, whose implicit copy copies every member
  // (src/picp_solver.h:72-81); src/cam.cpp:34 assigns `picp_solver = PICPSolver();` to a by-value
  // member.  A move hands the device handle over; a copy gets its own handle holding copies of
  // the points, correspondences and pose (picp_clone), so it keeps solving the same problem as
  // the reference's copy (which shares the caller's arrays) does.
  PICPSolver(PICPSolver&& o) noexcept { take(o); }
  PICPSolver& operator=(PICPSolver&& o) noexcept {
    if (this != &o) {
      picp_destroy(_h);
      _h = nullptr;
      take(o);
    }
    return *this;
  }
  PICPSolver(const PICPSolver& o) { copy_from(o); }
  PICPSolver& operator=(const PICPSolver& o) {
    if (this != &o) {
      picp_t* keep = _h;
      _h = nullptr;
      copy_from(o);
      picp_destroy(keep);
    }
    return *this;
  }

  //! src/picp_solver.h:32-34
  void init(const Camera& camera, const Vector3fVector& world_points, const Vector2fVector& image_points) {
    _camera = camera;
    if (!_h && !check(picp_create(&_h, _device, camera.rows(), camera.cols(), data9(camera.cameraMatrix())), "picp_create"))
      return;
    check(picp_set_camera(_h, camera.rows(), camera.cols(), data9(camera.cameraMatrix())), "picp_set_camera");
    check(picp_set_points(_h, reinterpret_cast<const float*>(world_points.data()), (int64_t)world_points.size(),
                          reinterpret_cast<const float*>(image_points.data()), (int64_t)image_points.size()),
          "picp_set_points");
    check(picp_set_pose(_h, data16(camera.worldInCameraPose())), "picp_set_pose");
  }

  inline float kernelThreshold() const { return _kernel_thereshold; }
  inline void setKernelThreshold(float kernel_threshold) { _kernel_thereshold = kernel_threshold; }

  //! the camera whose pose holds the current estimate (src/picp_solver.h:44)
  const Camera& camera() const { return _camera; }
  const float chiInliers() const { return _stats.chi_in; }
  const float chiOutliers() const { return _stats.chi_out; }
  const int numInliers() const { return _stats.n_in; }

  //! src/picp_solver.cpp:93-105 -- false when n_in < min_inliers (pose unchanged)
  bool oneRound(const IntPairVector& correspondences, bool keep_outliers) {
    if (!_h) return false;
    if (!check(picp_set_correspondences(_h, reinterpret_cast<const int32_t*>(correspondences.data()),
                                        (int64_t)correspondences.size()),
               "picp_set_correspondences"))
      return false;
    _status = picp_one_round(_h, _kernel_thereshold, _damping, _min_num_inliers, keep_outliers ? 1 : 0, &_stats);
    if (_status == PICP_TOO_FEW_INLIERS) {
      std::cerr << "too few inliers, skipping" << std::endl;  // src/picp_solver.cpp:98
      return false;
    }
    if (_status != PICP_OK) {
      std::cerr << "picp_one_round: " << picp_last_error() << std::endl;
      return false;
    }
    pull_pose();
    return true;
  }

  // ---- extensions (not in the reference) ----
  //! exec/icp_test.cpp:88-107 fused on the device; returns the number of oneRound calls
  int solve(const IntPairVector& correspondences, int max_rounds = 50, float conv_eps = 1e-5f,
            bool keep_outliers = false, bool* converged = nullptr) {
    if (!_h) return 0;
    if (!check(picp_set_correspondences(_h, reinterpret_cast<const int32_t*>(correspondences.data()),
                                        (int64_t)correspondences.size()),
               "picp_set_correspondences"))
      return 0;
    picp_params p;
    picp_params_default(&p);
    p.threshold = _kernel_thereshold;
    p.damping = _damping;
    p.min_inliers = _min_num_inliers;
    p.keep_outliers = keep_outliers ? 1 : 0;
    p.max_rounds = max_rounds;
    p.conv_eps = conv_eps;
    if (!check(picp_solve(_h, &p, &_stats), "picp_solve")) return 0;
    pull_pose();
    if (converged) *converged = _stats.converged != 0;
    return _stats.rounds;
  }
  void setDamping(float d) { _damping = d; }
  void setMinNumInliers(int n) { _min_num_inliers = n; }
  int lastStatus() const { return _status; }
  const picp_stats& stats() const { return _stats; }

 protected:
  bool check(int rc, const char* what) {
    _status = rc;
    if (rc != PICP_OK) {
      std::cerr << what << ": " << picp_last_error() << std::endl;
      return false;
    }
    return true;
  }
  void pull_pose() {
    float T[16];
    if (picp_get_pose(_h, T) == PICP_OK) _camera.setWorldInCameraPose(iso_from16(T));
  }
  void copy_state(const PICPSolver& o) {
    _device = o._device;
    _camera = o._camera;
    _kernel_thereshold = o._kernel_thereshold;
    _damping = o._damping;
    _min_num_inliers = o._min_num_inliers;
    _stats = o._stats;
    _status = o._status;
  }
  void take(PICPSolver& o) {
    copy_state(o);
    _h = o._h;
    o._h = nullptr;
  }
  void copy_from(const PICPSolver& o) {
    copy_state(o);
    if (o._h) check(picp_clone(o._h, &_h), "picp_clone");
  }

  int _device;
  picp_t* _h = nullptr;
  Camera _camera;                //< this will hold our state
  float _kernel_thereshold;      //< threshold for the kernel
  float _damping;                //< damping, to slow the solution
  int _min_num_inliers;          //< if less inliers than this value, the solver stops
  picp_stats _stats = {0.f, 0.f, 0, 1, 0, 0, 0, 0};
  int _status = PICP_OK;
};

}  // namespace pr
