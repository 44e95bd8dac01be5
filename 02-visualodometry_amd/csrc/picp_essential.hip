// picp_essential.hip -- the essential-matrix bootstrap of the reference:
//
//   src/cam.cpp:37-91  Cam::computeEssentialAndRecoverPose
//     E = cv::findEssentialMat(p1, p2, K, cv::RANSAC)   (prob 0.999, 1 px, maxIters 1000)
//     cv::recoverPose(E, p1, p2, K, R, t, mask)          (distanceThresh 50)
//     pose of the second camera = [R | t]^-1             (:76-81, Cam::getPose)
//
// for many independent two-view problems at once (one per VO segment, C5).  The algorithm is the
// oracle's restatement (oracle/picp_essential.c): Nister's five-point solver, OpenCV's RANSAC
// subsets (its cv::RNG((uint64)-1) stream) and selection rule, recoverPose's four-way
// cheirality test.  Every double operation is evaluated as in the oracle (FP contraction off),
// so the models, their inlier counts and the chosen pose match it.
//
// The sequential RANSAC loop becomes four launches:
//   1. picp_ess_samples_kernel  one lane per problem: the subset stream (sequential MWC draws);
//   2. picp_ess_hyp_kernel      one lane per (problem, hypothesis): the five-point solver;
//   3. picp_ess_score_kernel    one wave per (problem, hypothesis): Sampson inlier counts of its
//                               solutions, lanes over points;
//   4. picp_ess_pose_kernel     one block per problem: OpenCV's selection replayed over the
//                               counts in hypothesis order (strict improvement, adaptive
//                               iteration bound), then recoverPose with lanes over points.
// Every hypothesis up to maxIters is scored; the replay stops where OpenCV's loop would, so
// the model chosen is the one its sequential loop returns.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "picp_internal.h"

#pragma clang fp contract(off)

namespace {

constexpr int NM = 20;
// monomials x^a y^b z^c of degree <= 3 in Nister's order (the first ten are eliminated)
__constant__ int8_t c_mon[NM][3] = {
    {3, 0, 0}, {0, 3, 0}, {2, 1, 0}, {1, 2, 0}, {2, 0, 1}, {2, 0, 0}, {0, 2, 1}, {0, 2, 0}, {1, 1, 1}, {1, 1, 0},
    {1, 0, 2}, {1, 0, 1}, {1, 0, 0}, {0, 1, 2}, {0, 1, 1}, {0, 1, 0}, {0, 0, 3}, {0, 0, 2}, {0, 0, 1}, {0, 0, 0}};
// index of x^a y^b z^c in that order (a, b, c < 4; -1 if degree > 3)
__constant__ int8_t c_idx[4][4][4] = {{{19, 18, 17, 16}, {15, 14, 13, -1}, {7, 6, -1, -1}, {1, -1, -1, -1}}, {{12, 11, 10, -1}, {9, 8, -1, -1}, {3, -1, -1, -1}, {-1, -1, -1, -1}}, {{5, 4, -1, -1}, {2, -1, -1, -1}, {-1, -1, -1, -1}, {-1, -1, -1, -1}}, {{0, -1, -1, -1}, {-1, -1, -1, -1}, {-1, -1, -1, -1}, {-1, -1, -1, -1}}};
constexpr int M_X = 12, M_Y = 15, M_Z = 18, M_1 = 19;

struct P3 {
  double c[NM];
};

__device__ void p3_zero(P3& r) {
  for (int i = 0; i < NM; ++i) r.c[i] = 0.0;
}

__device__ void p3_mul(const P3& p, const P3& q, P3& r) {
  p3_zero(r);
  for (int i = 0; i < NM; ++i) {
    if (p.c[i] == 0.0) continue;
    for (int j = 0; j < NM; ++j) {
      if (q.c[j] == 0.0) continue;
      const int a = c_mon[i][0] + c_mon[j][0], b = c_mon[i][1] + c_mon[j][1], c = c_mon[i][2] + c_mon[j][2];
      if (a + b + c > 3) continue;
      r.c[c_idx[a][b][c]] += p.c[i] * q.c[j];
    }
  }
}

__device__ void p3_axpy(P3& r, const P3& p, double s) {
  for (int i = 0; i < NM; ++i) r.c[i] += s * p.c[i];
}

// null space of the 5x9 epipolar system (columns of A^T = rows of the system), Householder QR
__device__ void nullspace4(double A[9][5], double N[4][9]) {
  double Qm[9][9];
  for (int i = 0; i < 9; ++i)
    for (int j = 0; j < 9; ++j) Qm[i][j] = (i == j) ? 1.0 : 0.0;
  for (int k = 0; k < 5; ++k) {
    double nrm = 0.0;
    for (int i = k; i < 9; ++i) nrm += A[i][k] * A[i][k];
    nrm = sqrt(nrm);
    if (nrm == 0.0) continue;
    double v[9];
    for (int i = 0; i < 9; ++i) v[i] = 0.0;
    const double alpha = (A[k][k] > 0.0) ? -nrm : nrm;
    for (int i = k; i < 9; ++i) v[i] = A[i][k];
    v[k] -= alpha;
    double vv = 0.0;
    for (int i = k; i < 9; ++i) vv += v[i] * v[i];
    if (vv == 0.0) continue;
    for (int j = 0; j < 5; ++j) {
      double s = 0.0;
      for (int i = k; i < 9; ++i) s += v[i] * A[i][j];
      s = 2.0 * s / vv;
      for (int i = k; i < 9; ++i) A[i][j] -= s * v[i];
    }
    for (int j = 0; j < 9; ++j) {
      double s = 0.0;
      for (int i = k; i < 9; ++i) s += Qm[j][i] * v[i];
      s = 2.0 * s / vv;
      for (int i = k; i < 9; ++i) Qm[j][i] -= s * v[i];
    }
  }
  for (int n = 0; n < 4; ++n)
    for (int i = 0; i < 9; ++i) N[n][i] = Qm[i][5 + n];
}

__device__ void umul(const double* a, int da, const double* b, int db, double* r) {
  for (int k = 0; k <= da + db; ++k) r[k] = 0.0;
  for (int i = 0; i <= da; ++i)
    for (int j = 0; j <= db; ++j) r[i + j] += a[i] * b[j];
}

__device__ double ueval(const double* a, int d, double z) {
  double s = a[d];
  for (int k = d - 1; k >= 0; --k) s = s * z + a[k];
  return s;
}

// real roots (ascending) of a degree-d polynomial, d <= 10: bottom-up through the derivatives,
// one bisection per monotone interval between consecutive critical points (oracle: real_roots)
__device__ int real_roots(const double* p_in, int d, double* roots) {
  double p[11];
  for (int k = 0; k <= d; ++k) p[k] = p_in[k];
  double amax = 0.0;
  for (int k = 0; k <= d; ++k) amax = fmax(amax, fabs(p[k]));
  if (amax == 0.0) return 0;
  while (d > 0 && fabs(p[d]) <= 1e-14 * amax) --d;
  if (d == 0) return 0;
  double bound = 0.0;
  for (int k = 0; k < d; ++k) bound = fmax(bound, fabs(p[k] / p[d]));
  bound += 1.0;
  double der[11][11];
  for (int k = 0; k <= d; ++k) der[d][k] = p[k];
  for (int deg = d - 1; deg >= 1; --deg)
    for (int k = 0; k <= deg; ++k) der[deg][k] = der[deg + 1][k + 1] * (double)(k + 1);
  double crit[11], cur[11];
  int nc = 0, nr = 0;
  for (int deg = 1; deg <= d; ++deg) {
    double ends[12];
    int ne = 0;
    ends[ne++] = -bound;
    for (int i = 0; i < nc; ++i) ends[ne++] = crit[i];
    ends[ne++] = bound;
    nr = 0;
    for (int i = 0; i + 1 < ne; ++i) {
      double lo = ends[i], hi = ends[i + 1];
      double flo = ueval(der[deg], deg, lo), fhi = ueval(der[deg], deg, hi);
      if (flo == 0.0) {
        if (nr == 0 || cur[nr - 1] != lo) cur[nr++] = lo;
        continue;
      }
      if ((flo < 0.0) == (fhi < 0.0)) continue;
      for (int it = 0; it < 200 && hi - lo > 0.0; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (mid <= lo || mid >= hi) break;
        const double fm = ueval(der[deg], deg, mid);
        if (fm == 0.0) {
          lo = hi = mid;
          break;
        }
        if ((fm < 0.0) == (flo < 0.0)) {
          lo = mid;
          flo = fm;
        } else {
          hi = mid;
        }
      }
      cur[nr++] = 0.5 * (lo + hi);
    }
    for (int i = 0; i < nr; ++i) crit[i] = cur[i];
    nc = nr;
  }
  for (int i = 0; i < nr; ++i) roots[i] = cur[i];
  return nr;
}

// Nister's five-point solver (oracle: or_five_point): up to 10 unit-norm row-major E
__device__ int five_point(const double* q1, const double* q2, double* Es) {
  double A[9][5];
  for (int i = 0; i < 5; ++i) {
    const double x1 = q1[2 * i], y1 = q1[2 * i + 1], x2 = q2[2 * i], y2 = q2[2 * i + 1];
    const double row[9] = {x2 * x1, x2 * y1, x2, y2 * x1, y2 * y1, y2, x1, y1, 1.0};
    for (int k = 0; k < 9; ++k) A[k][i] = row[k];
  }
  double N[4][9];
  nullspace4(A, N);
  P3 E[3][3];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      p3_zero(E[r][c]);
      E[r][c].c[M_X] = N[0][3 * r + c];
      E[r][c].c[M_Y] = N[1][3 * r + c];
      E[r][c].c[M_Z] = N[2][3 * r + c];
      E[r][c].c[M_1] = N[3][3 * r + c];
    }
  double Mx[10][NM];
  {
    P3 t1, t2, m, acc;
    p3_zero(acc);
    p3_mul(E[1][1], E[2][2], t1);
    p3_mul(E[1][2], E[2][1], t2);
    p3_axpy(t1, t2, -1.0);
    p3_mul(E[0][0], t1, m);
    p3_axpy(acc, m, 1.0);
    p3_mul(E[1][0], E[2][2], t1);
    p3_mul(E[1][2], E[2][0], t2);
    p3_axpy(t1, t2, -1.0);
    p3_mul(E[0][1], t1, m);
    p3_axpy(acc, m, -1.0);
    p3_mul(E[1][0], E[2][1], t1);
    p3_mul(E[1][1], E[2][0], t2);
    p3_axpy(t1, t2, -1.0);
    p3_mul(E[0][2], t1, m);
    p3_axpy(acc, m, 1.0);
    for (int k = 0; k < NM; ++k) Mx[0][k] = acc.c[k];
  }
  {
    P3 EEt[3][3], tr, t;
    p3_zero(tr);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        p3_zero(EEt[i][j]);
        for (int k = 0; k < 3; ++k) {
          p3_mul(E[i][k], E[j][k], t);
          p3_axpy(EEt[i][j], t, 1.0);
        }
      }
    for (int i = 0; i < 3; ++i) p3_axpy(tr, EEt[i][i], 1.0);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        P3 acc;
        p3_zero(acc);
        for (int k = 0; k < 3; ++k) {
          p3_mul(EEt[i][k], E[k][j], t);
          p3_axpy(acc, t, 2.0);
        }
        p3_mul(tr, E[i][j], t);
        p3_axpy(acc, t, -1.0);
        for (int k = 0; k < NM; ++k) Mx[1 + 3 * i + j][k] = acc.c[k];
      }
  }
  for (int col = 0; col < 10; ++col) {
    int piv = col;
    for (int r = col + 1; r < 10; ++r)
      if (fabs(Mx[r][col]) > fabs(Mx[piv][col])) piv = r;
    if (fabs(Mx[piv][col]) < 1e-300) return 0;
    if (piv != col)
      for (int k = 0; k < NM; ++k) {
        const double tmp = Mx[col][k];
        Mx[col][k] = Mx[piv][k];
        Mx[piv][k] = tmp;
      }
    const double inv = 1.0 / Mx[col][col];
    for (int k = 0; k < NM; ++k) Mx[col][k] *= inv;
    for (int r = 0; r < 10; ++r) {
      if (r == col || Mx[r][col] == 0.0) continue;
      const double f = Mx[r][col];
      for (int k = 0; k < NM; ++k) Mx[r][k] -= f * Mx[col][k];
    }
  }
  double B[3][3][5];
  for (int rr = 0; rr < 3; ++rr) {
    const double* e = Mx[4 + 2 * rr];
    const double* f = Mx[5 + 2 * rr];
    double* bx = B[rr][0];
    double* by = B[rr][1];
    double* b1 = B[rr][2];
    bx[0] = e[12]; bx[1] = e[11] - f[12]; bx[2] = e[10] - f[11]; bx[3] = -f[10]; bx[4] = 0.0;
    by[0] = e[15]; by[1] = e[14] - f[15]; by[2] = e[13] - f[14]; by[3] = -f[13]; by[4] = 0.0;
    b1[0] = e[19]; b1[1] = e[18] - f[19]; b1[2] = e[17] - f[18]; b1[3] = e[16] - f[17]; b1[4] = -f[16];
  }
  double n10[11], t7a[8], t7b[8], t10[12];
  for (int k = 0; k <= 10; ++k) n10[k] = 0.0;
  {
    double c0[8], c1[8], c2[8];
    umul(B[1][1], 3, B[2][2], 4, t7a);
    umul(B[1][2], 4, B[2][1], 3, t7b);
    for (int k = 0; k <= 7; ++k) c0[k] = t7a[k] - t7b[k];
    umul(B[1][0], 3, B[2][2], 4, t7a);
    umul(B[1][2], 4, B[2][0], 3, t7b);
    for (int k = 0; k <= 7; ++k) c1[k] = t7a[k] - t7b[k];
    double s6a[7], s6b[7];
    umul(B[1][0], 3, B[2][1], 3, s6a);
    umul(B[1][1], 3, B[2][0], 3, s6b);
    for (int k = 0; k <= 6; ++k) c2[k] = s6a[k] - s6b[k];
    c2[7] = 0.0;
    umul(B[0][0], 3, c0, 7, t10);
    for (int k = 0; k <= 10; ++k) n10[k] += t10[k];
    umul(B[0][1], 3, c1, 7, t10);
    for (int k = 0; k <= 10; ++k) n10[k] -= t10[k];
    umul(B[0][2], 4, c2, 7, t10);
    for (int k = 0; k <= 10; ++k) n10[k] += t10[k];
  }
  double zs[10];
  const int nz = real_roots(n10, 10, zs);
  int ns = 0;
  for (int s = 0; s < nz; ++s) {
    const double z = zs[s];
    double R[3][3];
    for (int rr = 0; rr < 3; ++rr) {
      R[rr][0] = ueval(B[rr][0], 3, z);
      R[rr][1] = ueval(B[rr][1], 3, z);
      R[rr][2] = ueval(B[rr][2], 4, z);
    }
    double best[3] = {0.0, 0.0, 0.0}, bn = -1.0;
    for (int a = 0; a < 3; ++a) {
      const int b = (a + 1) % 3;
      const double v[3] = {R[a][1] * R[b][2] - R[a][2] * R[b][1], R[a][2] * R[b][0] - R[a][0] * R[b][2],
                           R[a][0] * R[b][1] - R[a][1] * R[b][0]};
      const double nv = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
      if (nv > bn) {
        bn = nv;
        best[0] = v[0];
        best[1] = v[1];
        best[2] = v[2];
      }
    }
    if (!(fabs(best[2]) > 0.0)) continue;
    const double x = best[0] / best[2], y = best[1] / best[2];
    double* Eo = Es + 9 * ns;
    double nrm = 0.0;
    for (int k = 0; k < 9; ++k) {
      Eo[k] = x * N[0][k] + y * N[1][k] + z * N[2][k] + N[3][k];
      nrm += Eo[k] * Eo[k];
    }
    nrm = sqrt(nrm);
    if (!(nrm > 0.0)) continue;
    for (int k = 0; k < 9; ++k) Eo[k] /= nrm;
    ++ns;
  }
  return ns;
}

__device__ __forceinline__ double sampson2(const double* E, double x1, double y1, double x2, double y2) {
  const double ex0 = E[0] * x1 + E[1] * y1 + E[2];
  const double ex1 = E[3] * x1 + E[4] * y1 + E[5];
  const double ex2 = E[6] * x1 + E[7] * y1 + E[8];
  const double etx0 = E[0] * x2 + E[3] * y2 + E[6];
  const double etx1 = E[1] * x2 + E[4] * y2 + E[7];
  const double x2tex1 = x2 * ex0 + y2 * ex1 + ex2;
  const double a = ex0 * ex0 + ex1 * ex1, b = etx0 * etx0 + etx1 * etx1;
  return x2tex1 * x2tex1 / (a + b);
}

__device__ __forceinline__ void norm_pt(const float* p, int i, const EssArgs& A, double& x, double& y) {
  x = ((double)p[2 * i] - A.cx) / A.fx;
  y = ((double)p[2 * i + 1] - A.cy) / A.fy;
}

__device__ void jacobi3(double S[3][3], double V[3][3]) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) V[i][j] = (i == j) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 50; ++sweep) {
    const double off = S[0][1] * S[0][1] + S[0][2] * S[0][2] + S[1][2] * S[1][2];
    if (off < 1e-300) break;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        if (fabs(S[p][q]) < 1e-300) continue;
        const double theta = (S[q][q] - S[p][p]) / (2.0 * S[p][q]);
        const double t = ((theta >= 0.0) ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 3; ++k) {
          const double skp = S[k][p], skq = S[k][q];
          S[k][p] = c * skp - s * skq;
          S[k][q] = s * skp + c * skq;
        }
        for (int k = 0; k < 3; ++k) {
          const double spk = S[p][k], sqk = S[q][k];
          S[p][k] = c * spk - s * sqk;
          S[q][k] = s * spk + c * sqk;
        }
        for (int k = 0; k < 3; ++k) {
          const double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = c * vkp - s * vkq;
          V[k][q] = s * vkp + c * vkq;
        }
      }
  }
}

__device__ double det3(double M[3][3]) {
  return M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) - M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]) +
         M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]);
}

// cv::decomposeEssentialMat (oracle: or_decompose_essential)
__device__ void decompose_essential(const double* Ein, double* R1, double* R2, double* t) {
  double E[3][3], S[3][3], V[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) E[i][j] = Ein[3 * i + j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      S[i][j] = 0.0;
      for (int k = 0; k < 3; ++k) S[i][j] += E[k][i] * E[k][j];
    }
  jacobi3(S, V);
  int ord[3] = {0, 1, 2};
  for (int a = 0; a < 3; ++a)
    for (int b = a + 1; b < 3; ++b)
      if (S[ord[b]][ord[b]] > S[ord[a]][ord[a]]) {
        const int tmp = ord[a];
        ord[a] = ord[b];
        ord[b] = tmp;
      }
  double Vs[3][3], U[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Vs[i][j] = V[i][ord[j]];
  for (int j = 0; j < 2; ++j) {
    double u[3], nu = 0.0;
    for (int i = 0; i < 3; ++i) {
      u[i] = E[i][0] * Vs[0][j] + E[i][1] * Vs[1][j] + E[i][2] * Vs[2][j];
      nu += u[i] * u[i];
    }
    nu = sqrt(nu);
    for (int i = 0; i < 3; ++i) U[i][j] = (nu > 0.0) ? u[i] / nu : 0.0;
  }
  U[0][2] = U[1][0] * U[2][1] - U[2][0] * U[1][1];
  U[1][2] = U[2][0] * U[0][1] - U[0][0] * U[2][1];
  U[2][2] = U[0][0] * U[1][1] - U[1][0] * U[0][1];
  if (det3(Vs) < 0.0)
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Vs[i][j] = -Vs[i][j];
  const double W[3][3] = {{0, 1, 0}, {-1, 0, 0}, {0, 0, 1}};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double a = 0.0, b = 0.0;
      for (int k = 0; k < 3; ++k)
        for (int l = 0; l < 3; ++l) {
          a += U[i][k] * W[k][l] * Vs[j][l];
          b += U[i][k] * W[l][k] * Vs[j][l];
        }
      R1[3 * i + j] = a;
      R2[3 * i + j] = b;
    }
  for (int i = 0; i < 3; ++i) t[i] = U[i][2];
}

// one point of cv::triangulatePoints in double (recoverPose's): the homogeneous DLT solution,
// the smallest-eigenvalue eigenvector of A^T A by cyclic Jacobi (oracle: or_triangulate_h)
__device__ void triangulate_h(const double* P1, const double* P2, double ax, double ay, double bx, double by,
                              double X4[4]) {
  double A[4][4];
  for (int k = 0; k < 4; ++k) {
    A[0][k] = ax * P1[8 + k] - P1[0 + k];
    A[1][k] = ay * P1[8 + k] - P1[4 + k];
    A[2][k] = bx * P2[8 + k] - P2[0 + k];
    A[3][k] = by * P2[8 + k] - P2[4 + k];
  }
  double S[4][4], V[4][4];
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) {
      double s = 0.0;
      for (int k = 0; k < 4; ++k) s += A[k][r] * A[k][c];
      S[r][c] = s;
      V[r][c] = (r == c) ? 1.0 : 0.0;
    }
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0;
    for (int p = 0; p < 4; ++p)
      for (int q = p + 1; q < 4; ++q) off += S[p][q] * S[p][q];
    if (off == 0.0) break;
    for (int p = 0; p < 4; ++p)
      for (int q = p + 1; q < 4; ++q) {
        if (S[p][q] == 0.0) continue;
        const double theta = (S[q][q] - S[p][p]) / (2.0 * S[p][q]);
        const double t = ((theta >= 0.0) ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 4; ++k) {
          const double skp = S[k][p], skq = S[k][q];
          S[k][p] = c * skp - s * skq;
          S[k][q] = s * skp + c * skq;
        }
        for (int k = 0; k < 4; ++k) {
          const double spk = S[p][k], sqk = S[q][k];
          S[p][k] = c * spk - s * sqk;
          S[q][k] = s * spk + c * sqk;
        }
        for (int k = 0; k < 4; ++k) {
          const double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = c * vkp - s * vkq;
          V[k][q] = s * vkp + c * vkq;
        }
      }
  }
  int m = 0;
  for (int i = 1; i < 4; ++i)
    if (S[i][i] < S[m][m]) m = i;
  for (int k = 0; k < 4; ++k) X4[k] = V[k][m];
}

// recoverPose's test of one point for P1 = [R | s t]
__device__ int cheiral(const double* P1, double ax, double ay, double bx, double by, double dist) {
  const double P0[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
  double X4[4];
  triangulate_h(P0, P1, ax, ay, bx, by, X4);
  if (!(X4[2] * X4[3] > 0.0)) return 0;
  const double X0 = X4[0] / X4[3], X1 = X4[1] / X4[3], X2 = X4[2] / X4[3];
  if (!(X2 < dist)) return 0;
  const double z1 = P1[8] * X0 + P1[9] * X1 + P1[10] * X2 + P1[11];
  return (z1 > 0.0 && z1 < dist) ? 1 : 0;
}

__device__ int update_iters(double p, double ep, int model_points, int max_iters) {
  p = fmin(fmax(p, 0.0), 1.0);
  ep = fmin(fmax(ep, 0.0), 1.0);
  double num = fmax(1.0 - p, 2.2250738585072014e-308);
  double denom = 1.0 - pow(1.0 - ep, (double)model_points);
  if (denom < 2.2250738585072014e-308) return 0;
  num = log(num);
  denom = log(denom);
  if (denom >= 0.0 || -num >= (double)max_iters * (-denom)) return max_iters;
  return (int)rint(num / denom);
}

}  // namespace

// 1. OpenCV RANSAC's subsets (its cv::RNG((uint64)-1) multiply-with-carry stream)
extern "C" __global__ void picp_ess_samples_kernel(EssArgs A, const int64_t* __restrict__ offs,
                                                   int32_t* __restrict__ idx) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= A.n_problems) return;
  const int n = (int)(offs[p + 1] - offs[p]);
  int32_t* out = idx + (size_t)p * A.max_iters * 5;
  if (n < 5) return;
  if (n == 5) {
    for (int i = 0; i < 5; ++i) out[i] = i;
    return;
  }
  uint64_t st = ~0ull;
  for (int h = 0; h < A.max_iters; ++h) {
    int32_t* id = out + 5 * h;
    for (int i = 0; i < 5; ++i) {
      for (;;) {
        st = (uint64_t)(uint32_t)st * 4164903690u + (uint32_t)(st >> 32);
        const int c = (int)((uint32_t)st % (uint32_t)n);
        int j = 0;
        while (j < i && id[j] != c) ++j;
        if (j == i) {
          id[i] = c;
          break;
        }
      }
    }
  }
}

// 2. the five-point solutions of hypothesis h of problem p
extern "C" __global__ void picp_ess_hyp_kernel(EssArgs A, const int64_t* __restrict__ offs,
                                               const float* __restrict__ p1, const float* __restrict__ p2,
                                               const int32_t* __restrict__ idx, double* __restrict__ Es,
                                               int32_t* __restrict__ ns) {
  const int p = blockIdx.y;
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= A.max_iters) return;
  const int64_t o = offs[p];
  const int n = (int)(offs[p + 1] - o);
  int32_t* nso = ns + (size_t)p * A.max_iters + h;
  if (n < 5 || (n == 5 && h > 0)) {
    *nso = 0;
    return;
  }
  const int32_t* id = idx + ((size_t)p * A.max_iters + h) * 5;
  double s1[10], s2[10];
  for (int j = 0; j < 5; ++j) {
    norm_pt(p1 + 2 * o, id[j], A, s1[2 * j], s1[2 * j + 1]);
    norm_pt(p2 + 2 * o, id[j], A, s2[2 * j], s2[2 * j + 1]);
  }
  *nso = five_point(s1, s2, Es + ((size_t)p * A.max_iters + h) * 90);
}

// 3. inlier counts of the solutions of (p, h): one wave, lanes over the points
extern "C" __global__ void picp_ess_score_kernel(EssArgs A, const int64_t* __restrict__ offs,
                                                 const float* __restrict__ p1, const float* __restrict__ p2,
                                                 const double* __restrict__ Es, const int32_t* __restrict__ ns,
                                                 int32_t* __restrict__ cnt) {
  const int p = blockIdx.y, h = blockIdx.x, lane = threadIdx.x;
  const int64_t o = offs[p];
  const int n = (int)(offs[p + 1] - o);
  const size_t ph = (size_t)p * A.max_iters + h;
  const int k = ns[ph];
  const double* E0 = Es + ph * 90;
  const double thr = A.threshold / ((A.fx + A.fy) * 0.5);
  const double thr2 = thr * thr;
  for (int s = 0; s < k; ++s) {
    const double* E = E0 + 9 * s;
    int c = 0;
    for (int i = lane; i < n; i += 64) {
      double x1, y1, x2, y2;
      norm_pt(p1 + 2 * o, i, A, x1, y1);
      norm_pt(p2 + 2 * o, i, A, x2, y2);
      c += (sampson2(E, x1, y1, x2, y2) <= thr2) ? 1 : 0;
    }
    for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m);
    if (lane == 0) cnt[ph * 10 + s] = c;
  }
}

// 4. OpenCV's selection replayed in hypothesis order, then recoverPose
#define ESS_BLOCK 256
extern "C" __global__ __launch_bounds__(ESS_BLOCK) void picp_ess_pose_kernel(
    EssArgs A, const int64_t* __restrict__ offs, const float* __restrict__ p1, const float* __restrict__ p2,
    const double* __restrict__ Es, const int32_t* __restrict__ ns, const int32_t* __restrict__ cnt,
    float* __restrict__ T_out, int32_t* __restrict__ inliers, int32_t* __restrict__ good,
    uint8_t* __restrict__ mask) {
  __shared__ double s_E[9], s_R[2][9], s_t[3];
  __shared__ int s_best, s_red[4][ESS_BLOCK / 64], s_ch;
  const int p = blockIdx.x, tid = threadIdx.x;
  const int64_t o = offs[p];
  const int n = (int)(offs[p + 1] - o);
  if (tid == 0) {
    int best = 0, niters = A.max_iters;
    for (int h = 0; h < niters && h < A.max_iters; ++h) {
      const size_t ph = (size_t)p * A.max_iters + h;
      const int k = ns[ph];
      for (int s = 0; s < k; ++s) {
        const int c = cnt[ph * 10 + s];
        if (c > (best > 4 ? best : 4)) {
          best = c;
          for (int i = 0; i < 9; ++i) s_E[i] = Es[ph * 90 + 9 * s + i];
          niters = update_iters(A.prob, (double)(n - c) / n, 5, niters);
        }
      }
      if (n == 5) break;
    }
    s_best = best;
    inliers[p] = best;
    if (best > 0) decompose_essential(s_E, s_R[0], s_R[1], s_t);
  }
  __syncthreads();
  if (s_best == 0) {  // no model: identity pose, nothing in front
    if (tid < 16) T_out[16 * p + tid] = (tid % 5 == 0) ? 1.0f : 0.0f;
    if (tid == 0) good[p] = 0;
    if (mask)
      for (int i = tid; i < n; i += ESS_BLOCK) mask[o + i] = 0;
    return;
  }
  // the four candidates (R1,t) (R2,t) (R1,-t) (R2,-t)
  int g[4] = {0, 0, 0, 0};
  for (int i = tid; i < n; i += ESS_BLOCK) {
    double x1, y1, x2, y2;
    norm_pt(p1 + 2 * o, i, A, x1, y1);
    norm_pt(p2 + 2 * o, i, A, x2, y2);
    for (int c = 0; c < 4; ++c) {
      const double* R = s_R[c & 1];
      const double sg = (c < 2) ? 1.0 : -1.0;
      double P1[12];
      for (int r = 0; r < 3; ++r) {
        for (int q = 0; q < 3; ++q) P1[4 * r + q] = R[3 * r + q];
        P1[4 * r + 3] = sg * s_t[r];
      }
      g[c] += cheiral(P1, x1, y1, x2, y2, A.dist);
    }
  }
  const int lane = tid & 63, w = tid >> 6;
  for (int c = 0; c < 4; ++c) {
    int v = g[c];
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
    if (lane == 0) s_red[c][w] = v;
  }
  __syncthreads();
  if (tid == 0) {
    int G[4];
    for (int c = 0; c < 4; ++c) {
      G[c] = 0;
      for (int k = 0; k < ESS_BLOCK / 64; ++k) G[c] += s_red[c][k];
    }
    int ch;
    if (G[0] >= G[1] && G[0] >= G[2] && G[0] >= G[3]) ch = 0;
    else if (G[1] >= G[0] && G[1] >= G[2] && G[1] >= G[3]) ch = 1;
    else if (G[2] >= G[0] && G[2] >= G[1] && G[2] >= G[3]) ch = 2;
    else ch = 3;
    s_ch = ch;
    good[p] = G[ch];
    // camera-in-world of the second view: [R | t]^-1 = [R^T | -R^T t], column-major 4x4
    const double* R = s_R[ch & 1];
    const double sg = (ch < 2) ? 1.0 : -1.0;
    float* T = T_out + 16 * p;
    for (int c = 0; c < 3; ++c)
      for (int r = 0; r < 3; ++r) T[4 * c + r] = (float)R[3 * c + r];  // (R^T)(r, c) = R(c, r)
    for (int r = 0; r < 3; ++r) {
      double s = 0.0;
      for (int k = 0; k < 3; ++k) s += R[3 * k + r] * (sg * s_t[k]);
      T[12 + r] = (float)(-s);
    }
    T[3] = T[7] = T[11] = 0.0f;
    T[15] = 1.0f;
  }
  __syncthreads();
  if (mask) {
    const int ch = s_ch;
    const double* R = s_R[ch & 1];
    const double sg = (ch < 2) ? 1.0 : -1.0;
    double P1[12];
    for (int r = 0; r < 3; ++r) {
      for (int q = 0; q < 3; ++q) P1[4 * r + q] = R[3 * r + q];
      P1[4 * r + 3] = sg * s_t[r];
    }
    for (int i = tid; i < n; i += ESS_BLOCK) {
      double x1, y1, x2, y2;
      norm_pt(p1 + 2 * o, i, A, x1, y1);
      norm_pt(p2 + 2 * o, i, A, x2, y2);
      mask[o + i] = (uint8_t)cheiral(P1, x1, y1, x2, y2, A.dist);
    }
  }
}

// ------------------------------- host launch wrapper -------------------------------
// Buffers (device): offs n_problems+1; p1/p2 float pixel pairs; idx 5*max_iters per problem;
// Es 90*max_iters doubles per problem; ns max_iters per problem; cnt 10*max_iters per problem.
extern "C" hipError_t picp_launch_essential(hipStream_t stream, const EssArgs* args, const int64_t* offs,
                                           const float* p1, const float* p2, int32_t* idx, double* Es,
                                           int32_t* ns, int32_t* cnt, float* T_out, int32_t* inliers,
                                           int32_t* good, uint8_t* mask) {
  if (!args || args->n_problems <= 0 || args->max_iters <= 0) return hipErrorInvalidValue;
  const EssArgs A = *args;
  hipError_t e;
  hipLaunchKernelGGL(picp_ess_samples_kernel, dim3((A.n_problems + 63) / 64), dim3(64), 0, stream, A, offs, idx);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(picp_ess_hyp_kernel, dim3((A.max_iters + 63) / 64, A.n_problems), dim3(64), 0, stream, A, offs,
                     p1, p2, idx, Es, ns);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(picp_ess_score_kernel, dim3(A.max_iters, A.n_problems), dim3(64), 0, stream, A, offs, p1, p2,
                     Es, ns, cnt);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(picp_ess_pose_kernel, dim3(A.n_problems), dim3(ESS_BLOCK), 0, stream, A, offs, p1, p2, Es, ns,
                     cnt, T_out, inliers, good, mask);
  return hipGetLastError();
}
