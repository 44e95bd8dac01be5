// icp_test -- the reference's published pipeline (exec/icp_test.cpp:17-215) driven through the
// drop-in pr:: facade, i.e. on the MI355X PICP + triangulation kernels.
//
//   icp_test [data_dir=./data] [out_dir=./output] [--fused | --vo] [--gt-bootstrap] [--frames N]
//            [--device D]
//
// Per frame, as the reference: match the next frame's descriptors to the map
// (match_points, src/my_utilities.h:70-120), PICP from the previous pose (threshold 3000, <= 50
// rounds, relative chi convergence 1e-5), match current<->next, keep the matches not already
// tied to the map (add_new_world_points, src/my_utilities.cpp:413-434) and triangulate them
// between the previous and the new pose (src/cam.cpp:94-140).  Then scale-align the trajectory
// (Umeyama scale, src/my_utilities.cpp:459-478) and write output/*.txt like the reference.
//
// The bootstrap pose of frame 1 is cv::findEssentialMat(RANSAC) + cv::recoverPose
// (src/cam.cpp:37-91) on the GPU (picp_essential_batch, OpenCV's RANSAC subsets replayed);
// --gt-bootstrap substitutes the ground-truth relative pose normalised to unit translation.  --fused runs
// the icp loop as one device solve (pr::PICPSolver::solve) instead of host-driven oneRound().
// Descriptor matching runs on the GPU matcher (picp_match).  --vo runs the whole per-frame loop
// device-resident (picp_vo_*: match, PICP, match, select, triangulate, append on the GPU) and
// then writes the same outputs.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <limits>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

#include "pr/picp_solver.h"
#include "pr/triangulation.h"

namespace {

constexpr int kDesc = 10;
constexpr float kDistanceThreshold = 0.2f;  // src/my_utilities.h:44
constexpr float kRatioThreshold = 0.8f;     // src/my_utilities.h:46

struct DataPoint {
  int id_meas = 0, id_real = 0;
  float u = 0, v = 0;
  float desc[kDesc] = {};
};
struct WorldPoint {
  float xyz[3] = {};
  float desc[kDesc] = {};
  int id_meas = -1, id_real = -1;
};
struct Measurement {
  int seq = -1;
  float gt[3] = {}, odom[3] = {};
  std::vector<DataPoint> points;
};

// src/my_utilities.cpp:35-112 (whitespace tokens; malformed lines skipped with a message)
bool read_measurement(const std::string& path, Measurement& m) {
  std::ifstream f(path);
  if (!f) {
    std::cerr << "Error opening file " << path << std::endl;
    return false;
  }
  std::string line;
  while (std::getline(f, line)) {
    std::istringstream ss(line);
    std::vector<std::string> tok;
    for (std::string t; ss >> t;) tok.push_back(t);
    if (tok.empty()) continue;
    if (tok[0] == "seq:" && tok.size() >= 2) {
      m.seq = std::stoi(tok[1]);
    } else if (tok[0] == "gt_pose:" && tok.size() >= 4) {
      for (int k = 0; k < 3; ++k) m.gt[k] = std::stof(tok[1 + k]);
    } else if (tok[0] == "odom_pose:" && tok.size() >= 4) {
      for (int k = 0; k < 3; ++k) m.odom[k] = std::stof(tok[1 + k]);
    } else if (tok[0] == "point" && tok.size() >= 5 + kDesc) {
      DataPoint d;
      d.id_meas = std::stoi(tok[1]);
      d.id_real = std::stoi(tok[2]);
      d.u = std::stof(tok[3]);
      d.v = std::stof(tok[4]);
      for (int k = 0; k < kDesc; ++k) d.desc[k] = std::stof(tok[5 + k]);
      m.points.push_back(d);
    } else {
      std::cerr << "Invalid line in file " << path << ": " << line << std::endl;
    }
  }
  return true;
}

int g_device = 0;

// src/my_utilities.h:70-120 on the GPU matcher (picp_match): nearest descriptor, absolute
// threshold and Lowe ratio, bit-identical to the reference's scan.
// corr.first = index in set 1, corr.second = index in set 2.
template <class A, class B>
void match_points(const std::vector<A>& p1, const std::vector<B>& p2, pr::IntPairVector& corr) {
  if (p1.empty()) return;
  std::vector<float> d1(p1.size() * kDesc), d2(std::max<size_t>(p2.size(), 1) * kDesc);
  for (size_t i = 0; i < p1.size(); ++i) std::memcpy(&d1[i * kDesc], p1[i].desc, sizeof(p1[i].desc));
  for (size_t j = 0; j < p2.size(); ++j) std::memcpy(&d2[j * kDesc], p2[j].desc, sizeof(p2[j].desc));
  std::vector<int32_t> bi(p1.size()), acc(p1.size());
  std::vector<float> best(p1.size()), second(p1.size());
  if (picp_match(g_device, d1.data(), (int64_t)p1.size(), d2.data(), (int64_t)p2.size(), kDesc,
                 kDistanceThreshold, kRatioThreshold, bi.data(), best.data(), second.data(),
                 acc.data()) != PICP_OK) {
    std::cerr << "match_points failed: " << picp_last_error() << std::endl;
    std::exit(EXIT_FAILURE);
  }
  for (size_t i = 0; i < p1.size(); ++i)
    if (acc[i]) corr.emplace_back((int)i, bi[i]);
}

pr::Isometry3f planar_pose(const float p[3]) {  // augment_pose, src/my_utilities.cpp:245-260
  pr::Isometry3f T = pr::Isometry3f::Identity();
  const float c = std::cos(p[2]), s = std::sin(p[2]);
  T(0, 0) = c; T(0, 1) = -s;
  T(1, 0) = s; T(1, 1) = c;
  T(0, 3) = p[0];
  T(1, 3) = p[1];
  T(2, 3) = 0.f;
  return T;
}

pr::Isometry3f camera_mount() {  // data/camera.dat cam_transform
  pr::Isometry3f M = pr::Isometry3f::Identity();
  M(0, 0) = 0; M(0, 1) = 0; M(0, 2) = 1; M(0, 3) = 0.2f;
  M(1, 0) = -1; M(1, 1) = 0; M(1, 2) = 0;
  M(2, 0) = 0; M(2, 1) = -1; M(2, 2) = 0;
  return M;
}

pr::Isometry3f camera_to_image() {  // src/cam.cpp:18-26
  pr::Isometry3f T = pr::Isometry3f::Identity();
  T(0, 0) = 0; T(0, 1) = 0; T(0, 2) = 1;
  T(1, 0) = -1; T(1, 1) = 0; T(1, 2) = 0;
  T(2, 0) = 0; T(2, 1) = -1; T(2, 2) = 0;
  return T;
}

// Umeyama similarity scale of P -> Q (src/my_utilities.cpp:459-478 uses only this scale).
void sym3_eig(double A[3][3], double ev[3]) {
  for (int sweep = 0; sweep < 50; ++sweep) {
    const double off = A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[1][2] * A[1][2];
    if (off < 1e-30) break;
    for (int p = 0; p < 3; ++p)
      for (int q = p + 1; q < 3; ++q) {
        if (std::fabs(A[p][q]) < 1e-300) continue;
        const double th = (A[q][q] - A[p][p]) / (2 * A[p][q]);
        const double t = (th >= 0 ? 1 : -1) / (std::fabs(th) + std::sqrt(th * th + 1));
        const double c = 1 / std::sqrt(t * t + 1), s = t * c;
        for (int k = 0; k < 3; ++k) {
          const double akp = A[k][p], akq = A[k][q];
          A[k][p] = c * akp - s * akq;
          A[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < 3; ++k) {
          const double apk = A[p][k], aqk = A[q][k];
          A[p][k] = c * apk - s * aqk;
          A[q][k] = s * apk + c * aqk;
        }
      }
  }
  for (int i = 0; i < 3; ++i) ev[i] = A[i][i];
}

double umeyama_scale(const std::vector<pr::Vector3f>& P, const std::vector<pr::Vector3f>& Q) {
  const size_t n = P.size();
  double mp[3] = {0, 0, 0}, mq[3] = {0, 0, 0};
  for (size_t i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) {
      mp[k] += P[i][k] / (double)n;
      mq[k] += Q[i][k] / (double)n;
    }
  double varp = 0, S[3][3] = {};
  for (size_t i = 0; i < n; ++i) {
    double dp[3], dq[3];
    for (int k = 0; k < 3; ++k) {
      dp[k] = P[i][k] - mp[k];
      dq[k] = Q[i][k] - mq[k];
      varp += dp[k] * dp[k] / (double)n;
    }
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) S[r][c] += dq[r] * dp[c] / (double)n;
  }
  double StS[3][3] = {};
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      for (int k = 0; k < 3; ++k) StS[r][c] += S[k][r] * S[k][c];
  const double det = S[0][0] * (S[1][1] * S[2][2] - S[1][2] * S[2][1]) -
                     S[0][1] * (S[1][0] * S[2][2] - S[1][2] * S[2][0]) +
                     S[0][2] * (S[1][0] * S[2][1] - S[1][1] * S[2][0]);
  double ev[3];
  sym3_eig(StS, ev);
  double sv[3];
  for (int k = 0; k < 3; ++k) sv[k] = std::sqrt(std::max(0.0, ev[k]));
  std::sort(sv, sv + 3);
  const double trace = sv[2] + sv[1] + (det < 0 ? -sv[0] : sv[0]);
  return varp > 0 ? trace / varp : 1.0;
}

}  // namespace

int main(int argc, char** argv) {
  std::string data_dir = "./data", out_dir = "./output";
  bool fused = false, vo = false, gt_bootstrap = false;
  int n_meas = 121, device = 0, pos = 0;
  for (int a = 1; a < argc; ++a) {
    std::string s = argv[a];
    if (s == "--fused") fused = true;
    else if (s == "--vo") vo = true;
    else if (s == "--gt-bootstrap") gt_bootstrap = true;
    else if (s == "--frames" && a + 1 < argc) n_meas = std::atoi(argv[++a]);
    else if (s == "--device" && a + 1 < argc) device = std::atoi(argv[++a]);
    else if (pos == 0) { data_dir = s; ++pos; }
    else if (pos == 1) { out_dir = s; ++pos; }
  }
  g_device = device;
  std::vector<Measurement> meas(n_meas);
  for (int i = 0; i < n_meas; ++i) {
    char name[64];
    std::snprintf(name, sizeof(name), "/meas-%05d.dat", i);
    if (!read_measurement(data_dir + name, meas[i])) return EXIT_FAILURE;
  }

  pr::Matrix3f K = pr::Matrix3f::Identity();  // src/cam.cpp:14-16
  K(0, 0) = 180; K(0, 2) = 320; K(1, 1) = 180; K(1, 2) = 240;
  pr::Camera picp_cam(480, 640, K, pr::Isometry3f::Identity());
  pr::PICPSolver picp_solver(device);

  std::vector<WorldPoint> world;
  std::vector<pr::Isometry3f> poses, gt_poses;
  poses.push_back(pr::Isometry3f::Identity());

  auto triangulate = [&](const pr::Isometry3f& T1, const pr::Isometry3f& T2, const std::vector<DataPoint>& a,
                         const std::vector<DataPoint>& b, const pr::IntPairVector& pairs) {
    pr::Vector2fVector p1, p2;
    for (auto& c : pairs) {
      p1.push_back(pr::Vector2f(a[c.first].u, a[c.first].v));
      p2.push_back(pr::Vector2f(b[c.second].u, b[c.second].v));
    }
    if (p1.empty()) return;
    pr::Vector3fVector X;
    if (pr::triangulatePoints(K, T1, T2, p1, p2, X, device) != PICP_OK) {
      std::cerr << "triangulation failed: " << picp_last_error() << std::endl;
      std::exit(EXIT_FAILURE);
    }
    for (size_t i = 0; i < pairs.size(); ++i) {  // World_Point of the first image, src/cam.cpp:122-139
      WorldPoint w;
      for (int k = 0; k < 3; ++k) w.xyz[k] = X[i][k];
      std::memcpy(w.desc, a[pairs[i].first].desc, sizeof(w.desc));
      w.id_meas = a[pairs[i].first].id_meas;
      w.id_real = a[pairs[i].first].id_real;
      world.push_back(w);
    }
  };

  // bootstrap: Cam::computeEssentialAndRecoverPose on the matches of frames 0-1
  // (exec/icp_test.cpp:44-51, src/cam.cpp:37-91) -> picp_essential_batch; the pose of frame 1 is
  // Cam::getPose = [R | t]^-1 (unit baseline).  --gt-bootstrap: the gt relative pose normalised
  // to unit translation instead.
  pr::IntPairVector init_corr;
  match_points(meas[0].points, meas[1].points, init_corr);
  pr::Isometry3f T01 = pr::Isometry3f::Identity();
  if (gt_bootstrap) {
    const pr::Isometry3f M = camera_mount();
    T01 = (planar_pose(meas[0].gt) * M).inverse() * (planar_pose(meas[1].gt) * M);
    pr::Vector3f t01 = T01.translation();
    const float tn = t01.norm();
    T01(0, 3) = t01[0] / tn; T01(1, 3) = t01[1] / tn; T01(2, 3) = t01[2] / tn;
  } else {
    std::vector<float> p1, p2;
    for (auto& c : init_corr) {
      p1.push_back(meas[0].points[c.first].u);
      p1.push_back(meas[0].points[c.first].v);
      p2.push_back(meas[1].points[c.second].u);
      p2.push_back(meas[1].points[c.second].v);
    }
    const int64_t offs[2] = {0, (int64_t)init_corr.size()};
    float T16[16];
    int32_t inliers = 0, good = 0;
    if (picp_essential_batch(device, 1, offs, p1.data(), p2.data(), pr::data9(K), nullptr, T16, &inliers,
                             &good, nullptr) != PICP_OK) {
      std::cerr << "essential bootstrap failed: " << picp_last_error() << std::endl;
      return EXIT_FAILURE;
    }
    if (inliers == 0) {  // src/cam.cpp:58-61
      std::cerr << "Essential matrix computation failed!" << std::endl;
      return EXIT_FAILURE;
    }
    T01 = pr::iso_from16(T16);
  }
  long total_rounds = 0;
  double picp_ms = 0;
  if (vo) {
    // the whole loop below, device-resident: one VO segment over frames 0 .. n_meas-1 with the
    // bootstrap pair (Identity, T01) (picp_vo_*, include/picp_c.h)
    std::vector<int64_t> off(n_meas + 1, 0);
    for (int f = 0; f < n_meas; ++f) off[f + 1] = off[f] + (int64_t)meas[f].points.size();
    std::vector<float> uv((size_t)off[n_meas] * 2), desc((size_t)off[n_meas] * kDesc);
    for (int f = 0; f < n_meas; ++f)
      for (size_t i = 0; i < meas[f].points.size(); ++i) {
        const DataPoint& d = meas[f].points[i];
        uv[2 * (off[f] + i)] = d.u;
        uv[2 * (off[f] + i) + 1] = d.v;
        std::memcpy(&desc[(off[f] + i) * kDesc], d.desc, sizeof(d.desc));
      }
    picp_vo_t* seq = nullptr;
    if (picp_vo_create(&seq, device, 480, 640, pr::data9(K), n_meas, off.data(), uv.data(), desc.data(),
                       kDesc) != PICP_OK) {
      std::cerr << "picp_vo_create failed: " << picp_last_error() << std::endl;
      return EXIT_FAILURE;
    }
    float boot[32];
    std::memcpy(boot, pr::data16(pr::Isometry3f::Identity()), 16 * sizeof(float));
    std::memcpy(boot + 16, pr::data16(T01), 16 * sizeof(float));
    picp_params prm;
    picp_params_default(&prm);
    prm.threshold = 3000.0f;
    const int64_t first = 0;
    const int32_t steps = n_meas - 1;
    auto t0 = std::chrono::steady_clock::now();
    if (picp_vo_set_segments(seq, 1, &first, &steps, boot, &prm) != PICP_OK || picp_vo_run(seq) != PICP_OK) {
      std::cerr << "picp_vo run failed: " << picp_last_error() << std::endl;
      return EXIT_FAILURE;
    }
    picp_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::vector<float> P16((size_t)n_meas * 16);
    std::vector<picp_vo_step> rec(n_meas);
    int64_t mn = 0;
    if (picp_vo_get_poses(seq, P16.data()) != PICP_OK || picp_vo_get_steps(seq, rec.data()) != PICP_OK ||
        picp_vo_get_map(seq, 0, 0, nullptr, nullptr, &mn) != PICP_OK) {
      std::cerr << "picp_vo readback failed: " << picp_last_error() << std::endl;
      return EXIT_FAILURE;
    }
    std::vector<float> mxyz((size_t)std::max<int64_t>(mn, 1) * 3), mdesc((size_t)std::max<int64_t>(mn, 1) * kDesc);
    picp_vo_get_map(seq, 0, mn, mxyz.data(), mdesc.data(), &mn);
    picp_vo_destroy(seq);
    poses.clear();
    for (int f = 0; f < n_meas; ++f) {
      poses.push_back(pr::iso_from16(&P16[(size_t)f * 16]));
      gt_poses.push_back(planar_pose(meas[f].gt));
      total_rounds += f ? rec[f].rounds : 0;
    }
    // a map point carries the descriptor (and so the ids) of the observation it came from
    for (int64_t k = 0; k < mn; ++k) {
      WorldPoint w;
      std::memcpy(w.xyz, &mxyz[k * 3], sizeof(w.xyz));
      std::memcpy(w.desc, &mdesc[k * kDesc], sizeof(w.desc));
      for (int f = 0; f < n_meas && w.id_real < 0; ++f)
        for (auto& d : meas[f].points)
          if (std::memcmp(d.desc, w.desc, sizeof(w.desc)) == 0) {
            w.id_meas = d.id_meas;
            w.id_real = d.id_real;
            break;
          }
      world.push_back(w);
    }
  } else {
  triangulate(pr::Isometry3f::Identity(), T01, meas[0].points, meas[1].points, init_corr);
  for (int i = 0; i < n_meas - 1; i++) {
    gt_poses.push_back(planar_pose(meas[i].gt));
    const std::vector<DataPoint>& curr = meas[i].points;
    const std::vector<DataPoint>& next = meas[i + 1].points;
    pr::IntPairVector corr;  // (next image idx, world idx)
    match_points(next, world, corr);

    pr::Isometry3f previous_pose = poses.back();
    picp_cam.setWorldInCameraPose(previous_pose.inverse());
    pr::Vector3fVector wv;
    for (auto& w : world) wv.push_back(pr::Vector3f(w.xyz[0], w.xyz[1], w.xyz[2]));
    pr::Vector2fVector iv;
    for (auto& d : next) iv.push_back(pr::Vector2f(d.u, d.v));
    auto t0 = std::chrono::steady_clock::now();
    picp_solver.init(picp_cam, wv, iv);
    picp_solver.setKernelThreshold(3000.0f);
    if (fused) {
      total_rounds += picp_solver.solve(corr, 50, 0.00001f);
    } else {  // exec/icp_test.cpp:88-107 verbatim semantics, host-driven rounds
      float prev = std::numeric_limits<float>::max();
      for (int j = 0; j < 50; j++) {
        ++total_rounds;
        if (!picp_solver.oneRound(corr, false)) {
          std::cerr << "Solver iteration " << j << " failed." << std::endl;
          break;
        }
        const float cur = picp_solver.chiInliers();
        const float rel = (prev > 1e-10) ? std::abs(prev - cur) / prev : 0.0f;
        if (rel < 0.00001f) break;
        prev = cur;
      }
    }
    picp_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    pr::Isometry3f estimated_pose = picp_solver.camera().worldInCameraPose().inverse();
    poses.push_back(estimated_pose);

    pr::IntPairVector img_corr;  // (curr idx, next idx)
    match_points(curr, next, img_corr);
    pr::IntPairVector to_tri;    // add_new_world_points: next points not already matched to the map
    for (auto& c : img_corr) {
      bool found = false;
      for (auto& w : corr)
        if (next[c.second].id_meas == next[w.first].id_meas) { found = true; break; }
      if (!found) to_tri.push_back(c);
    }
    triangulate(previous_pose, estimated_pose, curr, next, to_tri);
  }
  gt_poses.push_back(planar_pose(meas[n_meas - 1].gt));
  }

  const pr::Isometry3f C2I = camera_to_image();
  std::vector<pr::Vector3f> P, Q;
  for (size_t j = 0; j < poses.size(); ++j) {
    poses[j] = C2I * poses[j];
    P.push_back(poses[j].translation());
    Q.push_back(gt_poses[j].translation());
  }
  const double scale = umeyama_scale(P, Q);

  std::ofstream ft(out_dir + "/estimated_trajectory.txt"), fs(out_dir + "/estimated_trajectory_scaled.txt"),
      fe(out_dir + "/errors.txt"), fw(out_dir + "/estimated_world_points.txt");
  if (!ft || !fs || !fe || !fw) {
    std::cerr << "Error: Unable to open output file." << std::endl;
    return EXIT_FAILURE;
  }
  const float pi = 3.14159265358979323846f;
  double sum_e = 0, sum_e2 = 0, max_e = 0, sum_yaw = 0, max_yaw = 0;
  for (size_t j = 0; j < poses.size(); ++j) {
    const pr::Isometry3f& g = gt_poses[j];
    const pr::Isometry3f& p = poses[j];
    const float angle_gt = std::atan2(g(1, 0), g(0, 0));
    const float angle = std::atan2(p(1, 0), p(0, 0)) + pi / 2.0f;
    pr::Vector3f t = p.translation();
    ft << j << " " << t[0] << " " << t[1] << " " << angle << "\n";
    pr::Vector3f ts = t * (float)scale;
    fs << j << " " << ts[0] << " " << ts[1] << " " << angle << "\n";
    const float e = (ts - g.translation()).norm();
    const float er = std::abs(angle - angle_gt);
    fe << j << " " << e << " " << er << "\n";
    float wrapped = std::fmod(er, 2 * pi);
    wrapped = std::min(wrapped, 2 * pi - wrapped);
    sum_e += e; sum_e2 += (double)e * e; max_e = std::max(max_e, (double)e);
    sum_yaw += wrapped; max_yaw = std::max(max_yaw, (double)wrapped);
  }
  for (int id = 0; id < 1000; id++)
    for (auto& w : world)
      if (w.id_real == id) {
        pr::Vector3f X = C2I * pr::Vector3f(w.xyz[0], w.xyz[1], w.xyz[2]) * (float)scale;
        fw << id << " " << X[0] << " " << X[1] << " " << X[2] << "\n";
        break;
      }
  const double n = (double)poses.size();
  std::printf("{\"frames\": %d, \"world_points\": %zu, \"scale\": %.6f, \"trans_err_mean\": %.6f, "
              "\"trans_err_rmse\": %.6f, \"trans_err_max\": %.6f, \"yaw_err_wrapped_mean\": %.6f, "
              "\"yaw_err_wrapped_max\": %.6f, \"picp_rounds\": %ld, \"picp_ms\": %.3f, \"fused\": %d, \"vo\": %d, "
              "\"bootstrap\": \"%s\"}\n",
              (int)n, world.size(), scale, sum_e / n, std::sqrt(sum_e2 / n), max_e, sum_yaw / n, max_yaw,
              total_rounds, picp_ms, fused ? 1 : 0, vo ? 1 : 0, gt_bootstrap ? "gt" : "essential");
  return 0;
}
