/*
 * picp_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker; see picp_oracle.h).
 *
 * Plain-C restatement of the reference's PICP hot path.  Every function cites the
 * reference file:line it follows (paths relative to the reference repo root).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off: no FMA contraction, so every float
 * operation rounds exactly as the reference's unfused scalar Eigen code would).
 *
 * Association order of the small Eigen products (e.g. whether R*p is summed as
 * (a0+a1)+a2 or a0+(a1+a2)) cannot be pinned: the reference does not build here.  This
 * restatement sums left to right; the MI355X kernels use the same order for every value
 * that feeds a branch (projection, error, chi), so the gating decisions agree bit for bit
 * with this oracle at the same pose.
 */
#include "picp_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define TM(T, i, j) ((T)[(j) * 4 + (i)]) /* column-major 4x4 */
#define KM(K, i, j) ((K)[(j) * 3 + (i)]) /* column-major 3x3 */

/* Isometry3f * Vector3f  = linear()*p + translation()  (Eigen Transform, src/camera.h:25) */
static void iso_apply(const float T[16], const float p[3], float out[3]) {
  for (int i = 0; i < 3; ++i) {
    float s = TM(T, i, 0) * p[0];
    s = s + TM(T, i, 1) * p[1];
    s = s + TM(T, i, 2) * p[2];
    out[i] = s + TM(T, i, 3);
  }
}

static void mat3_vec(const float K[9], const float p[3], float out[3]) {
  for (int i = 0; i < 3; ++i) {
    float s = KM(K, i, 0) * p[0];
    s = s + KM(K, i, 1) * p[1];
    s = s + KM(K, i, 2) * p[2];
    out[i] = s;
  }
}

/* pr::Camera::projectPoint, src/camera.h:24-36 */
int or_project_point(const float T[16], const float K[9], int rows, int cols,
                     const float p[3], float img[2]) {
  float pc[3], ph[3];
  iso_apply(T, p, pc);               /* camera.h:26 */
  if (pc[2] <= 0.0f) return 0;       /* camera.h:27-28 (NaN passes, as in the reference) */
  mat3_vec(K, pc, ph);               /* camera.h:29 */
  /* camera.h:30: head<2>()*(1./z) -- double reciprocal narrowed to float.  For IEEE
   * binary32 operands, (float)(1.0/(double)z) equals the correctly rounded 1.0f/z
   * (double rounding is innocuous for division when 53 >= 2*24+2). */
  float iz = (float)(1.0 / (double)ph[2]);
  img[0] = ph[0] * iz;
  img[1] = ph[1] * iz;
  if (img[0] < 0.0f || img[0] > (float)(cols - 1)) return 0; /* camera.h:31-32 */
  if (img[1] < 0.0f || img[1] > (float)(rows - 1)) return 0; /* camera.h:33-34 */
  return 1;
}

/* PICPSolver::errorAndJacobian, src/picp_solver.cpp:26-54 */
int or_error_and_jacobian(const float T[16], const float K[9], int rows, int cols,
                          const float p[3], const float z[2], float e[2], float J[12]) {
  float img[2];
  if (!or_project_point(T, K, rows, cols, p, img)) return 0; /* :30-33 */
  e[0] = img[0] - z[0];                                       /* :34 */
  e[1] = img[1] - z[1];

  float pc[3], ph[3];
  iso_apply(T, p, pc); /* :38 (recomputed, as the reference does) */
  /* Jr = [I | skew(-pc)], :39-41 ; skew from src/defs.h:139-145 */
  float Jr[3][6];
  memset(Jr, 0, sizeof(Jr));
  Jr[0][0] = Jr[1][1] = Jr[2][2] = 1.0f;
  const float m0 = -pc[0], m1 = -pc[1], m2 = -pc[2];
  /* skew(v) = [[0,-v2,v1],[v2,0,-v0],[-v1,v0,0]] with v = -pc */
  Jr[0][3] = 0.0f;  Jr[0][4] = -m2;  Jr[0][5] = m1;
  Jr[1][3] = m2;    Jr[1][4] = 0.0f; Jr[1][5] = -m0;
  Jr[2][3] = -m1;   Jr[2][4] = m0;   Jr[2][5] = 0.0f;

  mat3_vec(K, pc, ph);                      /* :43 */
  float iz = (float)(1.0 / (double)ph[2]);  /* :44 */
  float iz2 = iz * iz;                      /* :45 */
  float Jp[2][3] = {{iz, 0.0f, -ph[0] * iz2}, {0.0f, iz, -ph[1] * iz2}}; /* :47-50 */

  /* J = Jp*K*Jr, :52 -- (Jp*K) first, then times Jr */
  float JpK[2][3];
  for (int r = 0; r < 2; ++r)
    for (int c = 0; c < 3; ++c) {
      float s = Jp[r][0] * KM(K, 0, c);
      s = s + Jp[r][1] * KM(K, 1, c);
      s = s + Jp[r][2] * KM(K, 2, c);
      JpK[r][c] = s;
    }
  for (int r = 0; r < 2; ++r)
    for (int c = 0; c < 6; ++c) {
      float s = JpK[r][0] * Jr[0][c];
      s = s + JpK[r][1] * Jr[1][c];
      s = s + JpK[r][2] * Jr[2][c];
      J[c * 2 + r] = s;
    }
  return 1;
}

/* One correspondence's contribution (src/picp_solver.cpp:63-89), shared by both
 * linearize entry points.  Accumulators are double in both modes; FAITHFUL mode rounds
 * each partial sum back to float so the running sums are exactly the reference's
 * sequential float32 sums. */
typedef struct {
  float Hf[36], bf[6], chi_in_f, chi_out_f;
  double Hd[36], bd[6], chi_in_d, chi_out_d;
  int32_t n_in, n_proj;
} acc_t;

static void acc_one(acc_t* a, const float T[16], const float K[9], int rows, int cols,
                    const float p[3], const float zz[2], float threshold, int keep_outliers,
                    int mode) {
  float e[2], J[12];
  if (!or_error_and_jacobian(T, K, rows, cols, p, zz, e, J)) return; /* :67-72 */
  a->n_proj++;
  float chi = e[0] * e[0] + e[1] * e[1]; /* :74 */
  float lambda = 1.0f;                   /* :75 */
  int is_inlier = 1;
  if (chi > threshold) { /* :77 strict */
    lambda = sqrtf(threshold / chi);
    is_inlier = 0;
    if (mode == OR_MODE_FAITHFUL) a->chi_out_f += chi; else a->chi_out_d += (double)chi;
  } else {
    if (mode == OR_MODE_FAITHFUL) a->chi_in_f += chi; else a->chi_in_d += (double)chi;
    a->n_in++;
  }
  if (is_inlier || keep_outliers) { /* :86-89 */
    for (int c = 0; c < 6; ++c) {
      for (int r = 0; r < 6; ++r) {
        float h = J[r * 2 + 0] * J[c * 2 + 0];
        h = h + J[r * 2 + 1] * J[c * 2 + 1];
        h = h * lambda;
        if (mode == OR_MODE_FAITHFUL) a->Hf[c * 6 + r] += h; else a->Hd[c * 6 + r] += (double)h;
      }
      float g = J[c * 2 + 0] * e[0];
      g = g + J[c * 2 + 1] * e[1];
      g = g * lambda;
      if (mode == OR_MODE_FAITHFUL) a->bf[c] += g; else a->bd[c] += (double)g;
    }
  }
}

static void acc_out(const acc_t* a, int mode, or_lin_t* out) {
  for (int i = 0; i < 36; ++i) out->H[i] = (mode == OR_MODE_FAITHFUL) ? (double)a->Hf[i] : a->Hd[i];
  for (int i = 0; i < 6; ++i) out->b[i] = (mode == OR_MODE_FAITHFUL) ? (double)a->bf[i] : a->bd[i];
  out->chi_in = (mode == OR_MODE_FAITHFUL) ? (double)a->chi_in_f : a->chi_in_d;
  out->chi_out = (mode == OR_MODE_FAITHFUL) ? (double)a->chi_out_f : a->chi_out_d;
  out->n_in = a->n_in;
  out->n_projected = a->n_proj;
}

/* PICPSolver::linearize, src/picp_solver.cpp:56-91 */
void or_linearize(const float T[16], const float K[9], int rows, int cols,
                  const float* world, const float* image, const int32_t* pairs, int64_t m,
                  float threshold, int keep_outliers, int mode, or_lin_t* out) {
  acc_t a;
  memset(&a, 0, sizeof(a)); /* :57-61 */
  for (int64_t k = 0; k < m; ++k) {
    const int32_t ref_idx = pairs[2 * k + 0];  /* :65 (image) */
    const int32_t curr_idx = pairs[2 * k + 1]; /* :66 (world) */
    acc_one(&a, T, K, rows, cols, world + 3 * (int64_t)curr_idx, image + 2 * (int64_t)ref_idx,
            threshold, keep_outliers, mode);
  }
  acc_out(&a, mode, out);
}

void or_linearize_soa(const float T[16], const float K[9], int rows, int cols,
                      const float* x, const float* y, const float* z, const float* u,
                      const float* v, int64_t m, float threshold, int keep_outliers, int mode,
                      or_lin_t* out) {
  acc_t a;
  memset(&a, 0, sizeof(a));
  for (int64_t k = 0; k < m; ++k) {
    const float p[3] = {x[k], y[k], z[k]};
    const float zz[2] = {u[k], v[k]};
    acc_one(&a, T, K, rows, cols, p, zz, threshold, keep_outliers, mode);
  }
  acc_out(&a, mode, out);
}

/* Chunked-reduction linearize for the all-cores CPU baseline (SURVEY.md §8d "a chunked
 * reduction (C2/C3) on all host cores"): contiguous chunks, one per OpenMP thread, each
 * accumulated exactly like or_linearize_soa, then combined in chunk order.  The summation order
 * is not the reference's sequential one, so this is TIMING ONLY (bench.py cpu_baseline_mt),
 * never a parity oracle. */
#define OR_MT_MAX 256
void or_linearize_soa_mt(const float T[16], const float K[9], int rows, int cols,
                         const float* x, const float* y, const float* z, const float* u,
                         const float* v, int64_t m, float threshold, int keep_outliers, int mode,
                         int threads, or_lin_t* out) {
  static acc_t parts[OR_MT_MAX];
  const int nt = threads < 1 ? 1 : (threads > OR_MT_MAX ? OR_MT_MAX : threads);
#pragma omp parallel for num_threads(nt) schedule(static, 1)
  for (int t = 0; t < nt; ++t) {
    acc_t a;
    memset(&a, 0, sizeof(a));
    const int64_t lo = m * t / nt, hi = m * (t + 1) / nt;
    for (int64_t k = lo; k < hi; ++k) {
      const float p[3] = {x[k], y[k], z[k]};
      const float zz[2] = {u[k], v[k]};
      acc_one(&a, T, K, rows, cols, p, zz, threshold, keep_outliers, mode);
    }
    parts[t] = a;
  }
  acc_t a = parts[0];
  for (int t = 1; t < nt; ++t) {
    const acc_t* b = &parts[t];
    for (int i = 0; i < 36; ++i) { a.Hf[i] += b->Hf[i]; a.Hd[i] += b->Hd[i]; }
    for (int i = 0; i < 6; ++i) { a.bf[i] += b->bf[i]; a.bd[i] += b->bd[i]; }
    a.chi_in_f += b->chi_in_f; a.chi_out_f += b->chi_out_f;
    a.chi_in_d += b->chi_in_d; a.chi_out_d += b->chi_out_d;
    a.n_in += b->n_in; a.n_proj += b->n_proj;
  }
  acc_out(&a, mode, out);
}

/* Rx, Ry, Rz, v2tEuler: src/defs.h:100-136 (row-major 3x3 temporaries) */
static void rot_x(float a, float R[3][3]) {
  float c = cosf(a), s = sinf(a);
  float M[3][3] = {{1, 0, 0}, {0, c, -s}, {0, s, c}};
  memcpy(R, M, sizeof(M));
}
static void rot_y(float a, float R[3][3]) {
  float c = cosf(a), s = sinf(a);
  float M[3][3] = {{c, 0, s}, {0, 1, 0}, {-s, 0, c}};
  memcpy(R, M, sizeof(M));
}
static void rot_z(float a, float R[3][3]) {
  float c = cosf(a), s = sinf(a);
  float M[3][3] = {{c, -s, 0}, {s, c, 0}, {0, 0, 1}};
  memcpy(R, M, sizeof(M));
}
static void mul33(float A[3][3], float B[3][3], float C[3][3]) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      float s = A[i][0] * B[0][j];
      s = s + A[i][1] * B[1][j];
      s = s + A[i][2] * B[2][j];
      C[i][j] = s;
    }
}

void or_v2t_euler(const float v[6], float T[16]) {
  float Rx[3][3], Ry[3][3], Rz[3][3], Rxy[3][3], R[3][3];
  rot_x(v[3], Rx);
  rot_y(v[4], Ry);
  rot_z(v[5], Rz);
  mul33(Rx, Ry, Rxy); /* defs.h:133, left to right */
  mul33(Rxy, Rz, R);
  memset(T, 0, 16 * sizeof(float));
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) TM(T, i, j) = R[i][j];
  TM(T, 0, 3) = v[0]; /* defs.h:134 */
  TM(T, 1, 3) = v[1];
  TM(T, 2, 3) = v[2];
  TM(T, 3, 3) = 1.0f;
}

/* Isometry3f * Isometry3f : linear = A.linear*B.linear, t = A.linear*B.t + A.t */
static void iso_mul(const float A[16], const float B[16], float C[16]) {
  float out[16];
  memset(out, 0, sizeof(out));
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) {
      float s = TM(A, i, 0) * TM(B, 0, j);
      s = s + TM(A, i, 1) * TM(B, 1, j);
      s = s + TM(A, i, 2) * TM(B, 2, j);
      TM(out, i, j) = s;
    }
    float s = TM(A, i, 0) * TM(B, 0, 3);
    s = s + TM(A, i, 1) * TM(B, 1, 3);
    s = s + TM(A, i, 2) * TM(B, 2, 3);
    TM(out, i, 3) = s + TM(A, i, 3);
  }
  TM(out, 3, 3) = 1.0f;
  memcpy(C, out, sizeof(out));
}

void or_iso_inverse(const float T[16], float Tinv[16]) {
  float out[16];
  memset(out, 0, sizeof(out));
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) TM(out, i, j) = TM(T, j, i);
  for (int i = 0; i < 3; ++i) {
    float s = TM(out, i, 0) * TM(T, 0, 3);
    s = s + TM(out, i, 1) * TM(T, 1, 3);
    s = s + TM(out, i, 2) * TM(T, 2, 3);
    TM(out, i, 3) = -s;
  }
  TM(out, 3, 3) = 1.0f;
  memcpy(Tinv, out, sizeof(out));
}

/* Eigen's LDLT<Matrix6f> (lower, diagonal pivoting) factor + solve, the published
 * algorithm of Eigen/src/Cholesky/LDLT.h (ldlt_inplace<Lower>::unblocked, _solve_impl),
 * restated for a dense 6x6.  Used for `H.ldlt().solve(-b)` (src/picp_solver.cpp:102). */
#define LDLT_BODY(TYPE, TINY)                                                                \
  TYPE L[6][6];                                                                              \
  int perm[6];                                                                               \
  for (int c = 0; c < 6; ++c)                                                                \
    for (int r = 0; r < 6; ++r) L[r][c] = A[c * 6 + r];                                      \
  int tr[6];                                                                                 \
  TYPE temp[6];                                                                              \
  for (int k = 0; k < 6; ++k) {                                                              \
    int big = k;                                                                             \
    TYPE bigv = (TYPE)fabs((double)L[k][k]);                                                 \
    for (int i = k + 1; i < 6; ++i)                                                          \
      if ((TYPE)fabs((double)L[i][i]) > bigv) { bigv = (TYPE)fabs((double)L[i][i]); big = i; } \
    tr[k] = big;                                                                             \
    if (k != big) {                                                                          \
      for (int j = 0; j < k; ++j) { TYPE t_ = L[k][j]; L[k][j] = L[big][j]; L[big][j] = t_; } \
      for (int i = big + 1; i < 6; ++i) { TYPE t_ = L[i][k]; L[i][k] = L[i][big]; L[i][big] = t_; } \
      { TYPE t_ = L[k][k]; L[k][k] = L[big][big]; L[big][big] = t_; }                        \
      for (int i = k + 1; i < big; ++i) { TYPE t_ = L[i][k]; L[i][k] = L[big][i]; L[big][i] = t_; } \
    }                                                                                        \
    if (k > 0) {                                                                             \
      for (int j = 0; j < k; ++j) temp[j] = L[j][j] * L[k][j];                               \
      TYPE s_ = 0;                                                                           \
      for (int j = 0; j < k; ++j) s_ = s_ + L[k][j] * temp[j];                               \
      L[k][k] -= s_;                                                                         \
      for (int i = k + 1; i < 6; ++i) {                                                      \
        TYPE s2 = 0;                                                                         \
        for (int j = 0; j < k; ++j) s2 = s2 + L[i][j] * temp[j];                             \
        L[i][k] -= s2;                                                                       \
      }                                                                                      \
    }                                                                                        \
    TYPE akk = L[k][k];                                                                      \
    if (fabs((double)akk) > 0.0)                                                             \
      for (int i = k + 1; i < 6; ++i) L[i][k] /= akk;                                        \
  }                                                                                          \
  for (int i = 0; i < 6; ++i) perm[i] = i;                                                   \
  TYPE y[6];                                                                                 \
  for (int i = 0; i < 6; ++i) y[i] = rhs[i];                                                 \
  for (int k = 0; k < 6; ++k)                                                                \
    if (tr[k] != k) { TYPE t_ = y[k]; y[k] = y[tr[k]]; y[tr[k]] = t_; }                      \
  for (int i = 0; i < 6; ++i)                                                                \
    for (int j = 0; j < i; ++j) y[i] -= L[i][j] * y[j];                                      \
  for (int i = 0; i < 6; ++i) {                                                              \
    TYPE d_ = L[i][i];                                                                       \
    y[i] = (fabs((double)d_) > (double)(TINY)) ? y[i] / d_ : (TYPE)0;                        \
  }                                                                                          \
  for (int i = 5; i >= 0; --i)                                                               \
    for (int j = i + 1; j < 6; ++j) y[i] -= L[j][i] * y[j];                                  \
  for (int k = 5; k >= 0; --k)                                                               \
    if (tr[k] != k) { TYPE t_ = y[k]; y[k] = y[tr[k]]; y[tr[k]] = t_; }                      \
  (void)perm;                                                                                \
  for (int i = 0; i < 6; ++i) x[i] = y[i];

void or_ldlt_solve6_f(const float A[36], const float rhs[6], float x[6]) { LDLT_BODY(float, FLT_MIN) }
void or_ldlt_solve6_d(const double A[36], const double rhs[6], double x[6]) { LDLT_BODY(double, DBL_MIN) }

/* oneRound tail shared by the AoS and SoA forms: src/picp_solver.cpp:95-104 */
static int round_tail(float T[16], const or_lin_t* lin, float damping, int min_inliers,
                      int mode, or_stats_t* stats) {
  if (stats) {
    stats->chi_in = (float)lin->chi_in;
    stats->chi_out = (float)lin->chi_out;
    stats->n_in = lin->n_in;
  }
  float dx[6];
  if (mode == OR_MODE_FAITHFUL) {
    float H[36], nb[6];
    for (int i = 0; i < 36; ++i) H[i] = (float)lin->H[i];
    for (int i = 0; i < 6; ++i) H[i * 6 + i] += 1.0f * damping; /* :96 */
    if (lin->n_in < min_inliers) { if (stats) stats->ok = 0; return 0; } /* :97-100 */
    for (int i = 0; i < 6; ++i) nb[i] = -(float)lin->b[i];
    or_ldlt_solve6_f(H, nb, dx); /* :102 */
  } else {
    double H[36], nb[6], dxd[6];
    for (int i = 0; i < 36; ++i) H[i] = lin->H[i];
    for (int i = 0; i < 6; ++i) H[i * 6 + i] += (double)damping;
    if (lin->n_in < min_inliers) { if (stats) stats->ok = 0; return 0; }
    for (int i = 0; i < 6; ++i) nb[i] = -lin->b[i];
    or_ldlt_solve6_d(H, nb, dxd);
    for (int i = 0; i < 6; ++i) dx[i] = (float)dxd[i];
  }
  float D[16];
  or_v2t_euler(dx, D); /* :103 */
  iso_mul(D, T, T);
  if (stats) stats->ok = 1;
  return 1;
}

int or_one_round(float T[16], const float K[9], int rows, int cols, const float* world,
                 const float* image, const int32_t* pairs, int64_t m, float threshold,
                 float damping, int min_inliers, int keep_outliers, int mode,
                 or_stats_t* stats) {
  or_lin_t lin;
  or_linearize(T, K, rows, cols, world, image, pairs, m, threshold, keep_outliers, mode, &lin);
  return round_tail(T, &lin, damping, min_inliers, mode, stats);
}

/* exec/icp_test.cpp:88-107 -- shared driver; lin_fn does one linearization */
static int conv_check(float* prev, float cur, float eps) {
  /* icp_test.cpp:99-106 */
  float rel = (*prev > 1e-10f) ? fabsf(*prev - cur) / *prev : 0.0f;
  if (rel < eps) return 1;
  *prev = cur;
  return 0;
}

int or_solve(float T[16], const float K[9], int rows, int cols, const float* world,
             const float* image, const int32_t* pairs, int64_t m, float threshold,
             float damping, int min_inliers, int keep_outliers, int mode, int max_rounds,
             float conv_eps, or_stats_t* last_stats, int* converged) {
  float prev = FLT_MAX;
  int rounds = 0;
  or_stats_t st;
  memset(&st, 0, sizeof(st));
  if (converged) *converged = 0;
  for (int j = 0; j < max_rounds; ++j) {
    int ok = or_one_round(T, K, rows, cols, world, image, pairs, m, threshold, damping,
                          min_inliers, keep_outliers, mode, &st);
    rounds++;
    if (!ok) break; /* icp_test.cpp:95-98 */
    if (conv_check(&prev, st.chi_in, conv_eps)) {
      if (converged) *converged = 1;
      break;
    }
  }
  if (last_stats) *last_stats = st;
  return rounds;
}

int or_solve_soa(float T[16], const float K[9], int rows, int cols, const float* x,
                 const float* y, const float* z, const float* u, const float* v, int64_t m,
                 float threshold, float damping, int min_inliers, int keep_outliers, int mode,
                 int max_rounds, float conv_eps, or_stats_t* last_stats, int* converged) {
  float prev = FLT_MAX;
  int rounds = 0;
  or_stats_t st;
  memset(&st, 0, sizeof(st));
  if (converged) *converged = 0;
  for (int j = 0; j < max_rounds; ++j) {
    or_lin_t lin;
    or_linearize_soa(T, K, rows, cols, x, y, z, u, v, m, threshold, keep_outliers, mode, &lin);
    int ok = round_tail(T, &lin, damping, min_inliers, mode, &st);
    rounds++;
    if (!ok) break;
    if (conv_check(&prev, st.chi_in, conv_eps)) {
      if (converged) *converged = 1;
      break;
    }
  }
  if (last_stats) *last_stats = st;
  return rounds;
}

/* or_solve_soa over the chunked-reduction linearize (timing only, see or_linearize_soa_mt). */
int or_solve_soa_mt(float T[16], const float K[9], int rows, int cols, const float* x,
                    const float* y, const float* z, const float* u, const float* v, int64_t m,
                    float threshold, float damping, int min_inliers, int keep_outliers, int mode,
                    int max_rounds, float conv_eps, int threads, or_stats_t* last_stats,
                    int* converged) {
  float prev = FLT_MAX;
  int rounds = 0;
  or_stats_t st;
  memset(&st, 0, sizeof(st));
  if (converged) *converged = 0;
  for (int j = 0; j < max_rounds; ++j) {
    or_lin_t lin;
    or_linearize_soa_mt(T, K, rows, cols, x, y, z, u, v, m, threshold, keep_outliers, mode,
                        threads, &lin);
    int ok = round_tail(T, &lin, damping, min_inliers, mode, &st);
    rounds++;
    if (!ok) break;
    if (conv_check(&prev, st.chi_in, conv_eps)) {
      if (converged) *converged = 1;
      break;
    }
  }
  if (last_stats) *last_stats = st;
  return rounds;
}

/* P = K * (T_cw^-1)(0:3, 0:4), src/cam.cpp:109-112 ; row-major 3x4 out */
void or_projection_matrix(const float K[9], const float T_cw[16], float P[12]) {
  float Ti[16];
  or_iso_inverse(T_cw, Ti);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) {
      float s = KM(K, i, 0) * TM(Ti, 0, j);
      s = s + KM(K, i, 1) * TM(Ti, 1, j);
      s = s + KM(K, i, 2) * TM(Ti, 2, j);
      P[i * 4 + j] = s;
    }
}

/* Symmetric 4x4 cyclic Jacobi eigen-decomposition (long double). Returns the eigenvector
 * of the smallest eigenvalue in v[4]. */
static void sym4_min_eigvec(long double S[4][4], long double v[4]) {
  long double V[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) V[i][j] = (i == j) ? 1.0L : 0.0L;
  for (int sweep = 0; sweep < 60; ++sweep) {
    long double off = 0.0L;
    for (int p = 0; p < 4; ++p)
      for (int q = p + 1; q < 4; ++q) off += S[p][q] * S[p][q];
    if (off == 0.0L) break;
    for (int p = 0; p < 4; ++p)
      for (int q = p + 1; q < 4; ++q) {
        if (S[p][q] == 0.0L) continue;
        long double theta = (S[q][q] - S[p][p]) / (2.0L * S[p][q]);
        long double t = (theta >= 0 ? 1.0L : -1.0L) / (fabsl(theta) + sqrtl(theta * theta + 1.0L));
        long double c = 1.0L / sqrtl(t * t + 1.0L), s = t * c;
        for (int k = 0; k < 4; ++k) { /* S <- S J */
          long double skp = S[k][p], skq = S[k][q];
          S[k][p] = c * skp - s * skq;
          S[k][q] = s * skp + c * skq;
        }
        for (int k = 0; k < 4; ++k) { /* S <- J^T S */
          long double spk = S[p][k], sqk = S[q][k];
          S[p][k] = c * spk - s * sqk;
          S[q][k] = s * spk + c * sqk;
        }
        for (int k = 0; k < 4; ++k) {
          long double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = c * vkp - s * vkq;
          V[k][q] = s * vkp + c * vkq;
        }
      }
  }
  int best = 0;
  for (int i = 1; i < 4; ++i)
    if (S[i][i] < S[best][best]) best = i;
  for (int k = 0; k < 4; ++k) v[k] = V[k][best];
}

/* cv::triangulatePoints (DLT, per point: A rows x*P3-P1, y*P3-P2 for both views, X = right
 * singular vector of the smallest singular value, computed in double) followed by
 * cv::convertPointsFromHomogeneous (float; scale 1 when |w| <= FLT_EPSILON), as called from
 * src/cam.cpp:115-118. */
void or_triangulate(const float P1[12], const float P2[12], const float* uv1, const float* uv2,
                    int64_t q, float* xyz_out) {
  for (int64_t i = 0; i < q; ++i) {
    long double A[4][4];
    const float* Ps[2] = {P1, P2};
    const float* pts[2] = {uv1 + 2 * i, uv2 + 2 * i};
    for (int j = 0; j < 2; ++j) {
      const double x = pts[j][0], y = pts[j][1];
      for (int k = 0; k < 4; ++k) {
        A[2 * j + 0][k] = (long double)(x * (double)Ps[j][8 + k] - (double)Ps[j][0 + k]);
        A[2 * j + 1][k] = (long double)(y * (double)Ps[j][8 + k] - (double)Ps[j][4 + k]);
      }
    }
    long double S[4][4];
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 4; ++c) {
        long double s = 0.0L;
        for (int k = 0; k < 4; ++k) s += A[k][r] * A[k][c];
        S[r][c] = s;
      }
    long double v[4];
    sym4_min_eigvec(S, v);
    float X4[4] = {(float)v[0], (float)v[1], (float)v[2], (float)v[3]}; /* points4D is float */
    float w = X4[3];
    float scale = (fabsf(w) > FLT_EPSILON) ? 1.0f / w : 1.0f;
    xyz_out[3 * i + 0] = X4[0] * scale;
    xyz_out[3 * i + 1] = X4[1] * scale;
    xyz_out[3 * i + 2] = X4[2] * scale;
  }
}

/* One point of cv::triangulatePoints in double (recoverPose's use, normalised coordinates):
 * the homogeneous DLT solution X4 (unnormalised, sign arbitrary). */
void or_triangulate_h(const double P1[12], const double P2[12], const double* a, const double* b,
                      double X4[4]) {
  long double A[4][4];
  const double* Ps[2] = {P1, P2};
  const double* pts[2] = {a, b};
  for (int j = 0; j < 2; ++j) {
    const double x = pts[j][0], y = pts[j][1];
    for (int k = 0; k < 4; ++k) {
      A[2 * j + 0][k] = (long double)(x * Ps[j][8 + k] - Ps[j][0 + k]);
      A[2 * j + 1][k] = (long double)(y * Ps[j][8 + k] - Ps[j][4 + k]);
    }
  }
  long double S[4][4];
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) {
      long double s = 0.0L;
      for (int k = 0; k < 4; ++k) s += A[k][r] * A[k][c];
      S[r][c] = s;
    }
  long double v[4];
  sym4_min_eigvec(S, v);
  for (int k = 0; k < 4; ++k) X4[k] = (double)v[k];
}

/* match_points, src/my_utilities.h:70-120 (see picp_oracle.h) */
int64_t or_match_points(const float* d1, int64_t n1, const float* d2, int64_t n2, int dim,
                        float dist_thr, float ratio_thr, int32_t* best_idx, float* best_dist,
                        float* second_dist, int32_t* accepted) {
  int64_t na = 0;
  for (int64_t i = 0; i < n1; ++i) {
    float best = FLT_MAX, second = FLT_MAX; /* :78-79 */
    int32_t bi = -1;
    for (int64_t j = 0; j < n2; ++j) {      /* :83-97 */
      float d = 0.0f;
      for (int k = 0; k < dim; ++k) {
        const float t = d1[i * dim + k] - d2[j * dim + k];
        d = d + t * t;
      }
      if (d < best) {
        second = best;
        best = d;
        bi = (int32_t)j;
      } else if (d < second) {
        second = d;
      }
    }
    const int acc = (bi != -1 && best < dist_thr && best / second < ratio_thr); /* :100-103 */
    best_idx[i] = bi;
    best_dist[i] = best;
    second_dist[i] = second;
    accepted[i] = acc;
    na += acc;
  }
  return na;
}

/* ---------------------------------------------------------------------------------------
 * VO segment loop, exec/icp_test.cpp:36-136 (see picp_oracle.h)
 * ------------------------------------------------------------------------------------- */
static int64_t vo_append(const float K[9], const float Tprev[16], const float Test[16],
                         const float* uv_a, const float* uv_b, const float* desc_a, int dim,
                         const int32_t* ia, const int32_t* ib, int64_t q, int64_t map_n,
                         int64_t map_cap, float* map_xyz, float* map_desc) {
  if (q == 0) return map_n;
  if (map_n + q > map_cap) return -1;
  float P1[12], P2[12];
  or_projection_matrix(K, Tprev, P1); /* src/cam.cpp:109-112 */
  or_projection_matrix(K, Test, P2);
  float* a = (float*)malloc((size_t)q * 2 * sizeof(float));
  float* b = (float*)malloc((size_t)q * 2 * sizeof(float));
  for (int64_t k = 0; k < q; ++k) {
    a[2 * k] = uv_a[2 * ia[k]];
    a[2 * k + 1] = uv_a[2 * ia[k] + 1];
    b[2 * k] = uv_b[2 * ib[k]];
    b[2 * k + 1] = uv_b[2 * ib[k] + 1];
    memcpy(map_desc + (map_n + k) * dim, desc_a + (int64_t)ia[k] * dim, (size_t)dim * sizeof(float));
  }
  or_triangulate(P1, P2, a, b, q, map_xyz + 3 * map_n); /* src/cam.cpp:115-139 */
  free(a);
  free(b);
  return map_n + q;
}

int64_t or_vo_segment(const float K[9], int rows, int cols, const int64_t* frame_off,
                      const float* uv, const float* desc, int dim, int64_t f0, int steps,
                      const float T0[16], const float T1[16], float threshold, int mode,
                      int max_rounds, float conv_eps, float* poses_out, int32_t* n_corr_out,
                      int32_t* n_in_out, int32_t* rounds_out, int32_t* n_new_out,
                      int64_t map_cap, float* map_xyz, float* map_desc) {
  int64_t nmax = 0;
  for (int64_t f = f0; f <= f0 + steps; ++f) nmax = frame_off[f + 1] - frame_off[f] > nmax ? frame_off[f + 1] - frame_off[f] : nmax;
  const size_t nb = (size_t)(nmax > 0 ? nmax : 1);
  int32_t* bi = (int32_t*)malloc(nb * 4);
  int32_t* acc = (int32_t*)malloc(nb * 4);
  int32_t* wacc = (int32_t*)malloc(nb * 4);
  int32_t* ia = (int32_t*)malloc(nb * 4);
  int32_t* ib = (int32_t*)malloc(nb * 4);
  int32_t* pairs = (int32_t*)malloc(nb * 8);
  float* bd = (float*)malloc(nb * 4);
  float* sd = (float*)malloc(nb * 4);
  int64_t map_n = 0;
#define FR_N(f) (frame_off[(f) + 1] - frame_off[(f)])
#define FR_UV(f) (uv + 2 * frame_off[(f)])
#define FR_DESC(f) (desc + (int64_t)dim * frame_off[(f)])
  /* bootstrap: match(first, second) -> triangulate(T0, T1) (exec/icp_test.cpp:44-58) */
  {
    const int64_t na = FR_N(f0), nbb = FR_N(f0 + 1);
    or_match_points(FR_DESC(f0), na, FR_DESC(f0 + 1), nbb, dim, 0.2f, 0.8f, bi, bd, sd, acc);
    int64_t q = 0;
    for (int64_t i = 0; i < na; ++i)
      if (acc[i]) { ia[q] = (int32_t)i; ib[q] = bi[i]; ++q; }
    map_n = vo_append(K, T0, T1, FR_UV(f0), FR_UV(f0 + 1), FR_DESC(f0), dim, ia, ib, q, 0, map_cap,
                      map_xyz, map_desc);
    if (n_new_out) n_new_out[0] = (int32_t)q;
  }
  memcpy(poses_out, T0, 16 * sizeof(float)); /* poses = {T0} (:36 with the bootstrap frame) */
  for (int t = 0; t < steps && map_n >= 0; ++t) {
    const int64_t cf = f0 + t, nf = cf + 1;
    const int64_t nc = FR_N(cf), nn = FR_N(nf);
    /* corr = match(next, world) (:72-73); pairs (image idx, world idx) */
    or_match_points(FR_DESC(nf), nn, map_desc, map_n, dim, 0.2f, 0.8f, bi, bd, sd, wacc);
    int64_t m = 0;
    for (int64_t i = 0; i < nn; ++i)
      if (wacc[i]) { pairs[2 * m] = (int32_t)i; pairs[2 * m + 1] = bi[i]; ++m; }
    /* PICP from the previous pose (:76-107) */
    float T[16];
    or_iso_inverse(poses_out + 16 * t, T);
    or_stats_t st;
    int conv = 0;
    const int rounds = or_solve(T, K, rows, cols, map_xyz, FR_UV(nf), pairs, m, threshold, 1.0f, 0,
                                0, mode, max_rounds, conv_eps, &st, &conv);
    or_iso_inverse(T, poses_out + 16 * (t + 1)); /* :113 */
    if (n_corr_out) n_corr_out[t] = (int32_t)m;
    if (n_in_out) n_in_out[t] = st.n_in;
    if (rounds_out) rounds_out[t] = rounds;
    /* img matches curr -> next, add_new_world_points, triangulate (:117-130) */
    or_match_points(FR_DESC(cf), nc, FR_DESC(nf), nn, dim, 0.2f, 0.8f, bi, bd, sd, acc);
    int64_t q = 0;
    for (int64_t i = 0; i < nc; ++i)
      if (acc[i] && !wacc[bi[i]]) { ia[q] = (int32_t)i; ib[q] = bi[i]; ++q; }
    map_n = vo_append(K, poses_out + 16 * t, poses_out + 16 * (t + 1), FR_UV(cf), FR_UV(nf), FR_DESC(cf),
                      dim, ia, ib, q, map_n, map_cap, map_xyz, map_desc);
    if (n_new_out) n_new_out[t + 1] = (int32_t)q;
  }
#undef FR_N
#undef FR_UV
#undef FR_DESC
  free(bi); free(acc); free(wacc); free(ia); free(ib); free(pairs); free(bd); free(sd);
  return map_n;
}
