// Test scaffold: every way the reference's sources use pr::PICPSolver / pr::Camera, written from
// the interface (src/picp_solver.h:21-82, src/camera.h:13-57), compiled against the facade
// through include/ref_src/'s shims and linked with libpicp_amd.so only.
//
//   dropin_main <problem.bin> <out.txt>
//
// problem.bin: int32 n_world, n_image, m; float T_wc[16] (column-major world-in-camera prior);
// float K[9] (column-major); float world[3 n_world]; float image[2 n_image]; int32 pairs[2 m].
// out.txt: one line per pattern, "<name> <rounds> <n_in> <16 floats of the pose>".
// Exit status: 0 ok, 2 when a solver reported an error (e.g. no GPU), 1 on bad input.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <iostream>
#include <limits>
#include <utility>
#include <vector>

#include "../src/cam_like.h"

namespace {

struct Problem {
  pr::Isometry3f prior;
  pr::Matrix3f K;
  std::vector<float> world, image;
  pr::IntPairVector corr;
};

bool load(const char* path, Problem& p) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  int32_t hdr[3];
  bool ok = std::fread(hdr, sizeof(hdr), 1, f) == 1 && hdr[0] >= 0 && hdr[1] >= 0 && hdr[2] >= 0;
  float T[16], K[9];
  ok = ok && std::fread(T, sizeof(T), 1, f) == 1 && std::fread(K, sizeof(K), 1, f) == 1;
  if (ok) {
    p.prior = pr::iso_from16(T);
    for (int c = 0; c < 3; ++c)
      for (int r = 0; r < 3; ++r) p.K(r, c) = K[c * 3 + r];
    p.world.resize(3 * (size_t)hdr[0]);
    p.image.resize(2 * (size_t)hdr[1]);
    std::vector<int32_t> pairs(2 * (size_t)hdr[2]);
    ok = std::fread(p.world.data(), sizeof(float), p.world.size(), f) == p.world.size() &&
         std::fread(p.image.data(), sizeof(float), p.image.size(), f) == p.image.size() &&
         std::fread(pairs.data(), sizeof(int32_t), pairs.size(), f) == pairs.size();
    for (int32_t k = 0; ok && k < hdr[2]; ++k) p.corr.emplace_back(pairs[2 * k], pairs[2 * k + 1]);
  }
  std::fclose(f);
  return ok;
}

// extract_V3fV / extract_V2fV (src/my_utilities.cpp:209-223): fresh vectors returned by value,
// so the caller's init() arguments are temporaries (exec/icp_test.cpp:81-85)
pr::Vector3fVector extract_V3fV(const std::vector<float>& w) {
  pr::Vector3fVector v;
  for (size_t i = 0; i + 2 < w.size(); i += 3) v.emplace_back(w[i], w[i + 1], w[i + 2]);
  return v;
}
pr::Vector2fVector extract_V2fV(const std::vector<float>& im) {
  pr::Vector2fVector v;
  for (size_t i = 0; i + 1 < im.size(); i += 2) v.emplace_back(im[i], im[i + 1]);
  return v;
}

void emit(FILE* out, const char* name, int rounds, int n_in, const pr::Isometry3f& T) {
  std::fprintf(out, "%s %d %d", name, rounds, n_in);
  const float* d = pr::data16(T);
  for (int i = 0; i < 16; ++i) std::fprintf(out, " %.9g", d[i]);
  std::fprintf(out, "\n");
}

int g_failures = 0;

// exec/icp_test.cpp:78-117: one frame of the loop -- float chi, relative 1e-5, <= 50 rounds;
// returns the camera-in-world estimate (worldInCameraPose().inverse())
pr::Isometry3f icp_frame(pr::Camera& picp_cam, pr::PICPSolver& picp_solver, const Problem& p,
                         const pr::Isometry3f& previous_pose, int* rounds) {
  picp_cam.setWorldInCameraPose(previous_pose.inverse());
  picp_solver.init(picp_cam, extract_V3fV(p.world), extract_V2fV(p.image));  // temporaries
  picp_solver.setKernelThreshold(3000.0f);
  float prevError = std::numeric_limits<float>::max();
  int j = 0;
  for (; j < 50; j++) {
    if (!picp_solver.oneRound(p.corr, false)) {
      std::cerr << "Solver iteration " << j << " failed." << std::endl;
      ++g_failures;
      break;
    }
    const float currentError = picp_solver.chiInliers();
    const float rel = (prevError > 1e-10) ? std::abs(prevError - currentError) / prevError : 0.0f;
    if (rel < 0.00001f) {
      ++j;
      break;
    }
    prevError = currentError;
  }
  *rounds = j;
  return picp_solver.camera().worldInCameraPose().inverse();
}

// src/my_utilities.cpp:263-313: a local solver, threshold 100, outliers kept (robust weights),
// double chi, relative 0.05
pr::Isometry3f local_solver_round(const pr::Isometry3f& last_pose_estimate, pr::Camera& pr_cam,
                                  const pr::Vector3fVector& world_points,
                                  const pr::Vector2fVector& image_points,
                                  const pr::IntPairVector& correspondences, int* rounds, int* n_in) {
  *rounds = 0;
  *n_in = 0;
  if (correspondences.size() < 10) return last_pose_estimate;
  pr::PICPSolver solver;
  pr_cam.setWorldInCameraPose(last_pose_estimate);
  solver.init(pr_cam, world_points, image_points);
  solver.setKernelThreshold(100.0f);
  double prevError = std::numeric_limits<double>::max();
  int i = 0;
  for (; i < 50; ++i) {
    if (!solver.oneRound(correspondences, true)) {
      ++g_failures;
      break;
    }
    const double currentError = solver.chiInliers();
    const double rel = (prevError > 1e-10) ? std::abs(prevError - currentError) / prevError : 0.0;
    if (rel < 0.05) {
      ++i;
      break;
    }
    prevError = currentError;
  }
  *rounds = i;
  *n_in = solver.numInliers();
  return solver.camera().worldInCameraPose();
}

bool run_rounds(pr::PICPSolver& s, const pr::IntPairVector& corr, int n) {
  bool ok = true;
  for (int i = 0; i < n; ++i) ok = s.oneRound(corr, false) && ok;
  if (!ok) ++g_failures;
  return ok;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 3) {
    std::fprintf(stderr, "usage: %s <problem.bin> <out.txt>\n", argv[0]);
    return 1;
  }
  Problem p;
  if (!load(argv[1], p)) {
    std::fprintf(stderr, "bad problem file %s\n", argv[1]);
    return 1;
  }
  FILE* out = std::fopen(argv[2], "w");
  if (!out) return 1;

  // --- exec/icp_test.cpp:29-31,61-117: solver and camera outside the frame loop, re-init per
  //     frame with temporaries; frame 2 starts from frame 1's estimate ---
  {
    pr::Camera picp_cam(480, 640, p.K, pr::Isometry3f::Identity());
    pr::PICPSolver picp_solver;
    std::vector<pr::Isometry3f> poses;
    poses.push_back(p.prior.inverse());  // camera-in-world prior
    int rounds = 0;
    poses.push_back(icp_frame(picp_cam, picp_solver, p, poses.back(), &rounds));
    emit(out, "icp_frame1", rounds, picp_solver.numInliers(), poses.back());
    poses.push_back(icp_frame(picp_cam, picp_solver, p, poses.back(), &rounds));
    emit(out, "icp_frame2", rounds, picp_solver.numInliers(), poses.back());
  }

  // --- src/my_utilities.cpp:263-313: local solver, outliers kept, threshold 100 ---
  {
    pr::Camera pr_cam(480, 640, p.K, pr::Isometry3f::Identity());
    const pr::Vector3fVector W = extract_V3fV(p.world);
    const pr::Vector2fVector I = extract_V2fV(p.image);
    int rounds = 0, n_in = 0;
    pr::Isometry3f T = local_solver_round(p.prior, pr_cam, W, I, p.corr, &rounds, &n_in);
    emit(out, "local_keep_outliers", rounds, n_in, T);
  }

  // --- src/cam.cpp:10-34,179-224: by-value members, assignment in the constructor ---
  {
    CamLike cam(p.K);
    cam.setPose(p.prior);
    std::vector<TestWorldPoint> wp;
    for (size_t i = 0; i + 2 < p.world.size(); i += 3) wp.push_back({p.world[i], p.world[i + 1], p.world[i + 2]});
    std::vector<TestDataPoint> dp;
    for (size_t i = 0; i + 1 < p.image.size(); i += 2) dp.push_back({p.image[i], p.image[i + 1]});
    cam.initOneRound(wp, dp);
    if (!cam.oneRound(p.corr)) ++g_failures;
    emit(out, "cam_by_value", 5, cam.numInliers(), cam.getPose());
    CamLike cam2 = cam;  // copies the solver member (a new device handle with the same problem)
    if (!cam2.oneRound(p.corr)) ++g_failures;
    emit(out, "cam_copy_plus5", 10, cam2.numInliers(), cam2.getPose());
  }

  // --- value semantics: copy construction, copy assignment, moves, vector growth ---
  {
    pr::Camera c(480, 640, p.K, p.prior);
    pr::PICPSolver a;
    a.init(c, extract_V3fV(p.world), extract_V2fV(p.image));
    a.setKernelThreshold(3000.0f);
    run_rounds(a, p.corr, 2);
    pr::PICPSolver b(a);  // copy after 2 rounds
    run_rounds(a, p.corr, 3);
    run_rounds(b, p.corr, 3);
    emit(out, "copy_src_5", 5, a.numInliers(), a.camera().worldInCameraPose());
    emit(out, "copy_dst_5", 5, b.numInliers(), b.camera().worldInCameraPose());
    pr::PICPSolver d;
    d = b;  // copy assignment into an uninitialised solver
    pr::PICPSolver m(std::move(b));  // move: b's handle is handed over
    run_rounds(m, p.corr, 1);
    run_rounds(d, p.corr, 1);
    emit(out, "moved_6", 6, m.numInliers(), m.camera().worldInCameraPose());
    emit(out, "assigned_6", 6, d.numInliers(), d.camera().worldInCameraPose());
    std::vector<pr::PICPSolver> pool;
    for (int i = 0; i < 3; ++i) pool.push_back(a);  // growth moves the elements (noexcept move)
    run_rounds(pool[0], p.corr, 1);
    emit(out, "vector_6", 6, pool[0].numInliers(), pool[0].camera().worldInCameraPose());
    pool[2] = std::move(pool[0]);
    run_rounds(pool[2], p.corr, 1);
    emit(out, "vector_moved_7", 7, pool[2].numInliers(), pool[2].camera().worldInCameraPose());
    // a default-constructed solver that was never init'ed: oneRound fails cleanly
    pr::PICPSolver fresh;
    if (fresh.oneRound(p.corr, false)) std::fprintf(stderr, "uninitialised solver ran a round\n");
  }
  std::fclose(out);
  return g_failures ? 2 : 0;
}
