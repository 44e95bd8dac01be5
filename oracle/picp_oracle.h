/*
 * picp_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference PICP hot path (llepa/02-VisualOdometry) used as the
 * parity checker for the MI355X implementation.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library; the product path
 * (02-visualodometry_amd/) never links or calls it.
 *
 * The reference itself cannot be compiled here (it needs Eigen3 + OpenCV, neither is
 * installed), so this is a restatement, pinned by the known-answer tests
 * built from the reference's own noise-free data/ (tests/golden/).
 *
 * Conventions (identical to the C-ABI in include/picp_c.h):
 *   pose  T[16]  : 4x4 float, COLUMN-major (Eigen::Isometry3f memory layout),
 *                  T(i,j) = T[j*4+i]; this is the world-in-camera pose.
 *   K[9]         : 3x3 float, column-major (Eigen::Matrix3f layout).
 *   world[3*W]   : packed xyz (Vector3fVector layout, src/defs.h:22).
 *   image[2*I]   : packed uv  (Vector2fVector layout, src/defs.h:23).
 *   pairs[2*M]   : int32 (first = image index, second = world index) (IntPairVector,
 *                  src/defs.h:209-211, src/picp_solver.cpp:65-66).
 *   H[36]        : 6x6 column-major, both triangles.
 */
#ifndef PICP_ORACLE_H
#define PICP_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* accumulation modes of or_linearize */
#define OR_MODE_FAITHFUL 0 /* float32 sequential accumulation, float LDLT (the reference's own arithmetic) */
#define OR_MODE_F64      1 /* per-correspondence float32 math, float64 accumulation + float64 LDLT */

typedef struct {
  double H[36];
  double b[6];
  double chi_in;
  double chi_out;
  int32_t n_in;
  int32_t n_projected; /* correspondences that passed projectPoint (not in the reference API) */
} or_lin_t;

typedef struct {
  float chi_in;
  float chi_out;
  int32_t n_in;
  int32_t ok; /* oneRound's return value */
} or_stats_t;

/* src/camera.h:24-36 */
int or_project_point(const float T[16], const float K[9], int rows, int cols,
                     const float p[3], float img[2]);

/* src/picp_solver.cpp:26-54 ; J is 2x6 column-major (J(r,c) = J[c*2+r]) */
int or_error_and_jacobian(const float T[16], const float K[9], int rows, int cols,
                          const float p[3], const float z[2], float e[2], float J[12]);

/* src/picp_solver.cpp:56-91 */
void or_linearize(const float T[16], const float K[9], int rows, int cols,
                  const float* world, const float* image, const int32_t* pairs, int64_t m,
                  float threshold, int keep_outliers, int mode, or_lin_t* out);

/* Same as or_linearize but over already-gathered SoA arrays (x,y,z,u,v), i.e. pairs (i,i).
 * Used for the large synthetic configurations where the gather is the identity. */
void or_linearize_soa(const float T[16], const float K[9], int rows, int cols,
                      const float* x, const float* y, const float* z, const float* u,
                      const float* v, int64_t m, float threshold, int keep_outliers, int mode,
                      or_lin_t* out);

/* src/defs.h:100-136 */
void or_v2t_euler(const float v[6], float T[16]);

/* Eigen LDLT (diagonal pivoting) restatement, as used by src/picp_solver.cpp:102 */
void or_ldlt_solve6_f(const float A[36], const float rhs[6], float x[6]);
void or_ldlt_solve6_d(const double A[36], const double rhs[6], double x[6]);

/* src/picp_solver.cpp:93-105 ; updates T in place. returns oneRound's bool. */
int or_one_round(float T[16], const float K[9], int rows, int cols, const float* world,
                 const float* image, const int32_t* pairs, int64_t m, float threshold,
                 float damping, int min_inliers, int keep_outliers, int mode,
                 or_stats_t* stats);

/* The driver loop of exec/icp_test.cpp:88-107 (max_rounds, relative-chi convergence).
 * soa != 0 => world=(x,y,z) planes and image=(u,v) planes with pairs ignored (identity).
 * Returns rounds executed (oneRound calls); *converged set as icp_test's flag. */
int or_solve(float T[16], const float K[9], int rows, int cols, const float* world,
             const float* image, const int32_t* pairs, int64_t m, float threshold,
             float damping, int min_inliers, int keep_outliers, int mode, int max_rounds,
             float conv_eps, or_stats_t* last_stats, int* converged);

/* Same loop over SoA planes (x,y,z,u,v). */
int or_solve_soa(float T[16], const float K[9], int rows, int cols, const float* x,
                 const float* y, const float* z, const float* u, const float* v, int64_t m,
                 float threshold, float damping, int min_inliers, int keep_outliers, int mode,
                 int max_rounds, float conv_eps, or_stats_t* last_stats, int* converged);

/* Timing-only variants for the all-cores CPU baseline: the linearize is a chunked reduction
 * over `threads` OpenMP threads (contiguous chunks, combined in chunk order).  NOT a parity
 * oracle: the summation order differs from the reference's sequential one. */
void or_linearize_soa_mt(const float T[16], const float K[9], int rows, int cols,
                         const float* x, const float* y, const float* z, const float* u,
                         const float* v, int64_t m, float threshold, int keep_outliers, int mode,
                         int threads, or_lin_t* out);
int or_solve_soa_mt(float T[16], const float K[9], int rows, int cols, const float* x,
                    const float* y, const float* z, const float* u, const float* v, int64_t m,
                    float threshold, float damping, int min_inliers, int keep_outliers, int mode,
                    int max_rounds, float conv_eps, int threads, or_stats_t* last_stats,
                    int* converged);

/* Linear (DLT) triangulation, OpenCV cv::triangulatePoints + convertPointsFromHomogeneous
 * as called from src/cam.cpp:115-118.  P1,P2 are 3x4 ROW-major (cv::Mat layout).
 * uv1/uv2 packed float2, xyz_out packed float3.  Smallest right singular vector via a
 * cyclic Jacobi eigen-decomposition of A^T A in long double (independent of the GPU's
 * one-sided Jacobi SVD). */
void or_triangulate(const float P1[12], const float P2[12], const float* uv1, const float* uv2,
                    int64_t q, float* xyz_out);

/* P = K * inverse(T_camera_in_world)(0:3,0:4) as src/cam.cpp:109-112 (row-major out) */
void or_projection_matrix(const float K[9], const float T_cw[16], float P[12]);

/* match_points (src/my_utilities.h:70-120): for every descriptor of set 1 the nearest (squared
 * L2, float, summed over the dims in order) descriptor of set 2 and the second nearest, strict
 * '<' updates in index order; accepted iff best < dist_thr and best/second < ratio_thr
 * (DISTANCE_THRESHOLD 0.2, RATIO_THRESHOLD 0.8, src/my_utilities.h:44-46).  best_idx = -1 when
 * set 2 is empty.  Returns the number accepted. */
int64_t or_match_points(const float* d1, int64_t n1, const float* d2, int64_t n2, int dim,
                        float dist_thr, float ratio_thr, int32_t* best_idx, float* best_dist,
                        float* second_dist, int32_t* accepted);

/* The VO loop of exec/icp_test.cpp:36-136 over one segment of a sequence:
 * frames [f0, f0 + steps] of the packed observations (frame k = rows [frame_off[k],
 * frame_off[k+1]) of uv (float2) and desc (float[dim])).
 *   bootstrap (:40-58, with the pose pair given instead of computeEssentialAndRecoverPose):
 *     pairs = match(frame f0, frame f0+1); map = triangulate(T0, T1, pairs) (descriptor of f0).
 *   step t (:61-136): next = f0+t+1; corr = match(next, map); PICP from poses[t] (icp_test
 *     loop: threshold, <= max_rounds, relative-chi conv_eps, keep_outliers false);
 *     poses[t+1] = estimate; pairs = match(curr, next); add_new_world_points
 *     (src/my_utilities.cpp:413-434): the pairs whose next point has no map match are
 *     triangulated with (poses[t], poses[t+1]) and appended in pair order.
 * Poses are camera-in-world (4x4 column-major).  Outputs: poses_out[(steps+1)*16] ([0] = T0),
 * per step n_corr/n_in/rounds/n_new (n_new_out has steps+1 entries, [0] = bootstrap), the map
 * (xyz[3*cap], desc[dim*cap]).  Returns the final map size, or -1 if map_cap is exceeded. */
int64_t or_vo_segment(const float K[9], int rows, int cols, const int64_t* frame_off,
                      const float* uv, const float* desc, int dim, int64_t f0, int steps,
                      const float T0[16], const float T1[16], float threshold, int mode,
                      int max_rounds, float conv_eps, float* poses_out, int32_t* n_corr_out,
                      int32_t* n_in_out, int32_t* rounds_out, int32_t* n_new_out,
                      int64_t map_cap, float* map_xyz, float* map_desc);

/* Eigen::Isometry3f::inverse() (rigid inverse) */
void or_iso_inverse(const float T[16], float Tinv[16]);


/* ---- essential-matrix bootstrap (picp_essential.c; src/cam.cpp:37-91) ----
 * Nister's five-point solver: q1, q2 = five normalised points (x, y pairs), Es = up to 10
 * row-major 3x3 essential matrices (unit Frobenius norm) with q2^T E q1 = 0; returns the count. */
int or_five_point(const double* q1, const double* q2, double* Es);
/* the RANSAC subsets of OpenCV's RANSACPointSetRegistrator (its cv::RNG((uint64)-1) stream):
 * 5 * max_iters indices into n points */
int or_essential_samples(int n, int max_iters, int* idx);
/* RANSACUpdateNumIters */
int or_ransac_update_iters(double p, double ep, int model_points, int max_iters);
/* cv::findEssentialMat(p1, p2, K, RANSAC, prob, threshold, maxIters): p1/p2 = n float pixel
 * (x, y) pairs, K = {fx, fy, cx, cy}, q_scratch = 4n doubles, idx_scratch = 5 * max_iters ints.
 * Returns the inlier count of the best E (written row-major); 0 = no model. */
int or_find_essential(const float* p1, const float* p2, int n, const double K[4], double prob,
                      double threshold, int max_iters, double* q_scratch, int* idx_scratch,
                      double E_out[9]);
/* cv::decomposeEssentialMat */
void or_decompose_essential(const double* E, double R1[9], double R2[9], double t[3]);
/* cv::recoverPose(E, p1, p2, K, R, t, distanceThresh, mask): R row-major, t unit; mask (n bytes,
 * may be NULL) marks the points in front of both cameras; returns their count */
int or_recover_pose(const double E[9], const float* p1, const float* p2, int n, const double K[4],
                    double dist, double* q_scratch, double R_out[9], double t_out[3], uint8_t* mask);
/* one point of cv::triangulatePoints in double: homogeneous X4 (unnormalised) */
void or_triangulate_h(const double P1[12], const double P2[12], const double* a, const double* b,
                      double X4[4]);

#ifdef __cplusplus
}
#endif
#endif
