/* picp_essential.c -- CPU oracle (TEST INFRASTRUCTURE ONLY: tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline may use it; the product never does) for the essential-matrix
 * bootstrap of the reference, SURVEY.md §8f rank 4:
 *
 *   src/cam.cpp:37-91  Cam::computeEssentialAndRecoverPose
 *     cv::setRNGSeed(42); E = cv::findEssentialMat(p1, p2, K, cv::RANSAC)   (prob 0.999,
 *     threshold 1 px, maxIters 1000: OpenCV's defaults for this overload);
 *     cv::recoverPose(E, p1, p2, K, R, t, mask)                              (distanceThresh 50)
 *     camera pose of frame 1 = [R | t]^-1                                    (:76-81, getPose)
 *
 * OpenCV is not in this image; its published algorithms are restated:
 *  - minimal solver: Nister's five-point algorithm (null space of the 5x9 epipolar system,
 *    the ten cubic constraints det(E) = 0 and 2 E E^T E - tr(E E^T) E = 0, Gauss-Jordan in
 *    Nister's monomial order, the 3x3 hidden-variable matrix in z, its degree-10 determinant,
 *    real roots, back-substitution for x, y);
 *  - RANSAC scoring: OpenCV's EMEstimatorCallback error, the squared Sampson distance in
 *    normalised coordinates, inlier iff err <= (threshold / ((fx + fy) / 2))^2;
 *  - recoverPose: decomposeEssentialMat (R1 = U W V^T, R2 = U W^T V^T, t = U e3) and the
 *    four-way cheirality test on DLT-triangulated points (depth in (0, 50) in both cameras),
 *    with OpenCV's tie order (R1,t), (R2,t), (R1,-t), (R2,-t).
 * RANSAC follows RANSACPointSetRegistrator::run: the same subsets (its cv::RNG stream), the
 * same adaptive iteration bound and the same strict replacement rule, so the model chosen is
 * the reference's as long as the five-point roots of a subset come in the same order (only
 * ties between two solutions of one subset depend on it: OpenCV orders them as solvePoly
 * returns them, this restatement by ascending z).
 * Pinned by the reference's own run: data/ frames 0-1 give its published frame-1 pose
 * (output/estimated_trajectory.txt row 1; tests/test_oracle.py). */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "picp_oracle.h"

/* ---------------------------------------------------------------------------------------
 * polynomials in x, y, z of total degree <= 3, in Nister's monomial order */
enum { NM = 20 };
static const int MON[NM][3] = {
    {3, 0, 0}, {0, 3, 0}, {2, 1, 0}, {1, 2, 0}, {2, 0, 1}, {2, 0, 0}, {0, 2, 1}, {0, 2, 0},
    {1, 1, 1}, {1, 1, 0}, /* eliminated by Gauss-Jordan */
    {1, 0, 2}, {1, 0, 1}, {1, 0, 0}, {0, 1, 2}, {0, 1, 1}, {0, 1, 0}, {0, 0, 3}, {0, 0, 2},
    {0, 0, 1}, {0, 0, 0}};
enum { M_X = 12, M_Y = 15, M_Z = 18, M_1 = 19 };

static int mon_index(int a, int b, int c) {
  for (int i = 0; i < NM; ++i)
    if (MON[i][0] == a && MON[i][1] == b && MON[i][2] == c) return i;
  return -1;
}

typedef struct { double c[NM]; } poly3;

static void pmul(const poly3* p, const poly3* q, poly3* r) {
  memset(r, 0, sizeof(*r));
  for (int i = 0; i < NM; ++i) {
    if (p->c[i] == 0.0) continue;
    for (int j = 0; j < NM; ++j) {
      if (q->c[j] == 0.0) continue;
      const int a = MON[i][0] + MON[j][0], b = MON[i][1] + MON[j][1], c = MON[i][2] + MON[j][2];
      if (a + b + c > 3) continue; /* only products of degree <= 3 are ever formed */
      r->c[mon_index(a, b, c)] += p->c[i] * q->c[j];
    }
  }
}

static void padd(poly3* r, const poly3* p, double s) {
  for (int i = 0; i < NM; ++i) r->c[i] += s * p->c[i];
}

/* ---------------------------------------------------------------------------------------
 * the null space of the 5x9 epipolar system q2^T E q1 = 0 (E row-major), by Householder QR of
 * its 9x5 transpose: the last four columns of the 9x9 orthogonal factor */
static void nullspace4(double A[9][5], double N[4][9]) {
  double Qm[9][9];
  for (int i = 0; i < 9; ++i)
    for (int j = 0; j < 9; ++j) Qm[i][j] = (i == j) ? 1.0 : 0.0;
  for (int k = 0; k < 5; ++k) {
    double nrm = 0.0;
    for (int i = k; i < 9; ++i) nrm += A[i][k] * A[i][k];
    nrm = sqrt(nrm);
    if (nrm == 0.0) continue;
    double v[9] = {0};
    const double alpha = (A[k][k] > 0.0) ? -nrm : nrm;
    for (int i = k; i < 9; ++i) v[i] = A[i][k];
    v[k] -= alpha;
    double vv = 0.0;
    for (int i = k; i < 9; ++i) vv += v[i] * v[i];
    if (vv == 0.0) continue;
    for (int j = 0; j < 5; ++j) { /* A <- (I - 2 v v^T / v^T v) A */
      double s = 0.0;
      for (int i = k; i < 9; ++i) s += v[i] * A[i][j];
      s = 2.0 * s / vv;
      for (int i = k; i < 9; ++i) A[i][j] -= s * v[i];
    }
    for (int j = 0; j < 9; ++j) { /* Qm <- Qm H (Qm's columns span the reflected basis) */
      double s = 0.0;
      for (int i = k; i < 9; ++i) s += Qm[j][i] * v[i];
      s = 2.0 * s / vv;
      for (int i = k; i < 9; ++i) Qm[j][i] -= s * v[i];
    }
  }
  for (int n = 0; n < 4; ++n)
    for (int i = 0; i < 9; ++i) N[n][i] = Qm[i][5 + n];
}

/* ---------------------------------------------------------------------------------------
 * univariate polynomials: coefficient k of z^k */
static void umul(const double* a, int da, const double* b, int db, double* r) {
  for (int k = 0; k <= da + db; ++k) r[k] = 0.0;
  for (int i = 0; i <= da; ++i)
    for (int j = 0; j <= db; ++j) r[i + j] += a[i] * b[j];
}

static double ueval(const double* a, int d, double z) {
  double s = a[d];
  for (int k = d - 1; k >= 0; --k) s = s * z + a[k];
  return s;
}

/* Real roots of a degree-d polynomial (d <= 10), ascending.  The real roots of p^(k) separate
 * those of p^(k-1) (Rolle), so the roots are found bottom-up from the (d-1)-th derivative: on
 * each interval between consecutive critical points p is monotone and a sign change brackets
 * exactly one root, located by bisection to full precision.  All real roots lie within the
 * Cauchy bound of p (and by Gauss-Lucas so do those of every derivative). */
static int real_roots(const double* p_in, int d, double* roots) {
  double p[11];
  for (int k = 0; k <= d; ++k) p[k] = p_in[k];
  double amax = 0.0;
  for (int k = 0; k <= d; ++k) amax = fmax(amax, fabs(p[k]));
  if (amax == 0.0) return 0;
  while (d > 0 && fabs(p[d]) <= 1e-14 * amax) --d; /* numerically vanishing leading terms */
  if (d == 0) return 0;
  double bound = 0.0;
  for (int k = 0; k < d; ++k) bound = fmax(bound, fabs(p[k] / p[d]));
  bound += 1.0;
  double der[11][11]; /* der[k] = the (d-k)-th derivative of p, of degree k */
  for (int k = 0; k <= d; ++k) der[d][k] = p[k];
  for (int deg = d - 1; deg >= 1; --deg)
    for (int k = 0; k <= deg; ++k) der[deg][k] = der[deg + 1][k + 1] * (double)(k + 1);
  double crit[11], cur[11];
  int nc = 0, nr = 0;
  for (int deg = 1; deg <= d; ++deg) {
    /* roots of der[deg] from its critical points crit[0..nc) (the roots of der[deg-1]) */
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
        if (fm == 0.0) { lo = hi = mid; break; }
        if ((fm < 0.0) == (flo < 0.0)) { lo = mid; flo = fm; } else { hi = mid; }
      }
      cur[nr++] = 0.5 * (lo + hi);
    }
    for (int i = 0; i < nr; ++i) crit[i] = cur[i];
    nc = nr;
  }
  for (int i = 0; i < nr; ++i) roots[i] = cur[i];
  return nr;
}

/* ---------------------------------------------------------------------------------------
 * Nister's five-point solver: up to 10 essential matrices (row-major, unit Frobenius norm)
 * with q2^T E q1 = 0 for the five normalised correspondences */
int or_five_point(const double* q1, const double* q2, double* Es) {
  double A[9][5];
  for (int i = 0; i < 5; ++i) {
    const double x1 = q1[2 * i], y1 = q1[2 * i + 1], x2 = q2[2 * i], y2 = q2[2 * i + 1];
    const double row[9] = {x2 * x1, x2 * y1, x2, y2 * x1, y2 * y1, y2, x1, y1, 1.0};
    for (int k = 0; k < 9; ++k) A[k][i] = row[k];
  }
  double N[4][9];
  nullspace4(A, N);
  /* E = x N0 + y N1 + z N2 + N3, entries as polynomials of degree 1 */
  poly3 E[3][3];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      memset(&E[r][c], 0, sizeof(poly3));
      E[r][c].c[M_X] = N[0][3 * r + c];
      E[r][c].c[M_Y] = N[1][3 * r + c];
      E[r][c].c[M_Z] = N[2][3 * r + c];
      E[r][c].c[M_1] = N[3][3 * r + c];
    }
  double Mx[10][NM];
  /* det(E) = 0 */
  {
    poly3 t1, t2, m, acc;
    memset(&acc, 0, sizeof(acc));
    pmul(&E[1][1], &E[2][2], &t1);
    pmul(&E[1][2], &E[2][1], &t2);
    padd(&t1, &t2, -1.0);
    pmul(&E[0][0], &t1, &m);
    padd(&acc, &m, 1.0);
    pmul(&E[1][0], &E[2][2], &t1);
    pmul(&E[1][2], &E[2][0], &t2);
    padd(&t1, &t2, -1.0);
    pmul(&E[0][1], &t1, &m);
    padd(&acc, &m, -1.0);
    pmul(&E[1][0], &E[2][1], &t1);
    pmul(&E[1][1], &E[2][0], &t2);
    padd(&t1, &t2, -1.0);
    pmul(&E[0][2], &t1, &m);
    padd(&acc, &m, 1.0);
    for (int k = 0; k < NM; ++k) Mx[0][k] = acc.c[k];
  }
  /* 2 E E^T E - tr(E E^T) E = 0 */
  {
    poly3 EEt[3][3], tr, t;
    memset(&tr, 0, sizeof(tr));
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        memset(&EEt[i][j], 0, sizeof(poly3));
        for (int k = 0; k < 3; ++k) {
          pmul(&E[i][k], &E[j][k], &t);
          padd(&EEt[i][j], &t, 1.0);
        }
      }
    for (int i = 0; i < 3; ++i) padd(&tr, &EEt[i][i], 1.0);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        poly3 acc;
        memset(&acc, 0, sizeof(acc));
        for (int k = 0; k < 3; ++k) {
          pmul(&EEt[i][k], &E[k][j], &t);
          padd(&acc, &t, 2.0);
        }
        pmul(&tr, &E[i][j], &t);
        padd(&acc, &t, -1.0);
        for (int k = 0; k < NM; ++k) Mx[1 + 3 * i + j][k] = acc.c[k];
      }
  }
  /* Gauss-Jordan on the ten leading monomials, partial pivoting */
  for (int col = 0; col < 10; ++col) {
    int piv = col;
    for (int r = col + 1; r < 10; ++r)
      if (fabs(Mx[r][col]) > fabs(Mx[piv][col])) piv = r;
    if (fabs(Mx[piv][col]) < 1e-300) return 0; /* degenerate sample */
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
  /* rows 4..9 lead with x^2 z, x^2, y^2 z, y^2, xyz, xy:  <k> = <e> - z<f>, <l> = <g> - z<h>,
   * <m> = <i> - z<j>; each is x b_x(z) + y b_y(z) + b_1(z) (trailing columns 10..19 are
   * xz^2 xz x yz^2 yz y z^3 z^2 z 1) */
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
  /* det B(z): degree 3 + 3 + 4 = 10 */
  double n10[11] = {0}, t7a[8], t7b[8], t10[11];
  {
    /* cofactors of the first row */
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
    double t11[12];
    umul(B[0][2], 4, c2, 7, t11);
    for (int k = 0; k <= 10; ++k) n10[k] += t11[k];
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
    /* null vector (x, y, 1) of B(z): the largest of the three row cross products */
    double best[3] = {0, 0, 0}, bn = -1.0;
    for (int a = 0; a < 3; ++a) {
      const int b = (a + 1) % 3;
      const double v[3] = {R[a][1] * R[b][2] - R[a][2] * R[b][1], R[a][2] * R[b][0] - R[a][0] * R[b][2],
                           R[a][0] * R[b][1] - R[a][1] * R[b][0]};
      const double nv = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
      if (nv > bn) {
        bn = nv;
        best[0] = v[0]; best[1] = v[1]; best[2] = v[2];
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

/* ---------------------------------------------------------------------------------------
 * RANSAC over five-point samples, as OpenCV's RANSACPointSetRegistrator::run draws them: its own
 * cv::RNG seeded with (uint64)-1 (so the cv::setRNGSeed(42) of src/cam.cpp:40 does not reach it),
 * a multiply-with-carry generator, uniform(0, n) = next() % n, five distinct indices per subset
 * (a repeated index is redrawn) -- a sequential stream, generated once and shared with the GPU. */
static uint32_t cvrng_next(uint64_t* state) {
  *state = (uint64_t)(uint32_t)*state * 4164903690u + (uint32_t)(*state >> 32);
  return (uint32_t)*state;
}

/* the subsets of hypotheses 0..max_iters-1 (5 indices each) for n points; returns max_iters */
int or_essential_samples(int n, int max_iters, int* idx) {
  uint64_t st = ~0ull;
  for (int h = 0; h < max_iters; ++h) {
    int* id = idx + 5 * h;
    for (int i = 0; i < 5; ++i) {
      for (;;) {
        const int c = (int)(cvrng_next(&st) % (uint32_t)n);
        int j = 0;
        while (j < i && id[j] != c) ++j;
        if (j == i) { id[i] = c; break; }
      }
    }
  }
  return max_iters;
}

/* RANSACUpdateNumIters (OpenCV calib3d) */
int or_ransac_update_iters(double p, double ep, int model_points, int max_iters) {
  p = fmin(fmax(p, 0.0), 1.0);
  ep = fmin(fmax(ep, 0.0), 1.0);
  double num = fmax(1.0 - p, 2.2250738585072014e-308);
  double denom = 1.0 - pow(1.0 - ep, (double)model_points);
  if (denom < 2.2250738585072014e-308) return 0;
  num = log(num);
  denom = log(denom);
  if (denom >= 0.0 || -num >= (double)max_iters * (-denom)) return max_iters;
  return (int)lrint(num / denom);
}

/* OpenCV EMEstimatorCallback::computeError: squared Sampson distance */
static double sampson2(const double* E, double x1, double y1, double x2, double y2) {
  const double ex0 = E[0] * x1 + E[1] * y1 + E[2];
  const double ex1 = E[3] * x1 + E[4] * y1 + E[5];
  const double ex2 = E[6] * x1 + E[7] * y1 + E[8];
  const double etx0 = E[0] * x2 + E[3] * y2 + E[6];
  const double etx1 = E[1] * x2 + E[4] * y2 + E[7];
  const double x2tex1 = x2 * ex0 + y2 * ex1 + ex2;
  const double a = ex0 * ex0 + ex1 * ex1, b = etx0 * etx0 + etx1 * etx1;
  return x2tex1 * x2tex1 / (a + b);
}

static void normalize_pts(const float* p, int n, const double K[4], double* q) {
  for (int i = 0; i < n; ++i) {
    q[2 * i] = ((double)p[2 * i] - K[2]) / K[0];
    q[2 * i + 1] = ((double)p[2 * i + 1] - K[3]) / K[1];
  }
}

/* findEssentialMat(p1, p2, K, RANSAC, prob, threshold, maxIters): p1/p2 float pixel pairs,
 * K = {fx, fy, cx, cy}.  Hypotheses in OpenCV's order with its adaptive iteration bound; a model
 * replaces the best only with more inliers than max(best, 4).  Returns the inlier count of E
 * (0: no model; E untouched).  q_scratch: 4n doubles; idx_scratch: 5 * max_iters ints. */
int or_find_essential(const float* p1, const float* p2, int n, const double K[4], double prob,
                      double threshold, int max_iters, double* q_scratch, int* idx_scratch,
                      double E_out[9]) {
  if (n < 5) return 0;
  double* q1 = q_scratch;
  double* q2 = q_scratch + 2 * n;
  normalize_pts(p1, n, K, q1);
  normalize_pts(p2, n, K, q2);
  const double thr = threshold / ((K[0] + K[1]) * 0.5);
  const double thr2 = thr * thr;
  if (n > 5) or_essential_samples(n, max_iters, idx_scratch);
  int best = 0, niters = max_iters;
  for (int h = 0; h < niters; ++h) {
    int idx5[5] = {0, 1, 2, 3, 4};
    const int* idx = (n > 5) ? idx_scratch + 5 * h : idx5; /* n == 5: the single subset */
    double s1[10], s2[10], Es[90];
    for (int j = 0; j < 5; ++j) {
      s1[2 * j] = q1[2 * idx[j]]; s1[2 * j + 1] = q1[2 * idx[j] + 1];
      s2[2 * j] = q2[2 * idx[j]]; s2[2 * j + 1] = q2[2 * idx[j] + 1];
    }
    const int ns = or_five_point(s1, s2, Es);
    for (int s = 0; s < ns; ++s) {
      int cnt = 0;
      for (int i = 0; i < n; ++i)
        cnt += (sampson2(Es + 9 * s, q1[2 * i], q1[2 * i + 1], q2[2 * i], q2[2 * i + 1]) <= thr2);
      if (cnt > (best > 4 ? best : 4)) {
        best = cnt;
        memcpy(E_out, Es + 9 * s, 9 * sizeof(double));
        niters = or_ransac_update_iters(prob, (double)(n - cnt) / n, 5, niters);
      }
    }
    if (n == 5) break;
  }
  return best;
}

/* ---------------------------------------------------------------------------------------
 * recoverPose */
static void jacobi3(double S[3][3], double V[3][3]) { /* S symmetric -> eigenvalues on diag */
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
        for (int k = 0; k < 3; ++k) { /* S <- J^T S J */
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

static double det3(double M[3][3]) {
  return M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) - M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]) +
         M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]);
}

/* decomposeEssentialMat: R1 = U W V^T, R2 = U W^T V^T, t = U e3 (unit), from an SVD of E built
 * from the eigen-decomposition of E^T E (singular values s1 >= s2 >= s3 ~ 0) */
void or_decompose_essential(const double* Ein, double R1[9], double R2[9], double t[3]) {
  double E[3][3], S[3][3], V[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) E[i][j] = Ein[3 * i + j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      S[i][j] = 0.0;
      for (int k = 0; k < 3; ++k) S[i][j] += E[k][i] * E[k][j];
    }
  jacobi3(S, V);
  int ord[3] = {0, 1, 2}; /* eigenvalues descending */
  for (int a = 0; a < 3; ++a)
    for (int b = a + 1; b < 3; ++b)
      if (S[ord[b]][ord[b]] > S[ord[a]][ord[a]]) { const int tmp = ord[a]; ord[a] = ord[b]; ord[b] = tmp; }
  double Vs[3][3], U[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Vs[i][j] = V[i][ord[j]];
  for (int j = 0; j < 2; ++j) { /* u_j = E v_j / |E v_j| */
    double u[3], nu = 0.0;
    for (int i = 0; i < 3; ++i) {
      u[i] = E[i][0] * Vs[0][j] + E[i][1] * Vs[1][j] + E[i][2] * Vs[2][j];
      nu += u[i] * u[i];
    }
    nu = sqrt(nu);
    for (int i = 0; i < 3; ++i) U[i][j] = (nu > 0.0) ? u[i] / nu : 0.0;
  }
  U[0][2] = U[1][0] * U[2][1] - U[2][0] * U[1][1]; /* u3 = u1 x u2: det(U) = +1 */
  U[1][2] = U[2][0] * U[0][1] - U[0][0] * U[2][1];
  U[2][2] = U[0][0] * U[1][1] - U[1][0] * U[0][1];
  if (det3(Vs) < 0.0)
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Vs[i][j] = -Vs[i][j];
  static const double W[3][3] = {{0, 1, 0}, {-1, 0, 0}, {0, 0, 1}};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double a = 0.0, b = 0.0;
      for (int k = 0; k < 3; ++k)
        for (int l = 0; l < 3; ++l) {
          a += U[i][k] * W[k][l] * Vs[j][l]; /* U W V^T */
          b += U[i][k] * W[l][k] * Vs[j][l]; /* U W^T V^T */
        }
      R1[3 * i + j] = a;
      R2[3 * i + j] = b;
    }
  for (int i = 0; i < 3; ++i) t[i] = U[i][2];
}

/* OpenCV recoverPose's test of one point: Q = triangulate(P0, P); Q2*Q3 > 0; Q /= Q3; Q2 < dist;
 * Q' = P Q; 0 < Q'2 < dist */
static int cheiral(const double P0[12], const double P1[12], const double* a, const double* b, double dist) {
  double X4[4];
  or_triangulate_h(P0, P1, a, b, X4);
  if (!(X4[2] * X4[3] > 0.0)) return 0;
  const double X[3] = {X4[0] / X4[3], X4[1] / X4[3], X4[2] / X4[3]};
  if (!(X[2] < dist)) return 0;
  const double z1 = P1[8] * X[0] + P1[9] * X[1] + P1[10] * X[2] + P1[11];
  return (z1 > 0.0 && z1 < dist) ? 1 : 0;
}

/* recoverPose(E, p1, p2, K, R, t, distanceThresh, mask): the four (R, t) candidates, each
 * scored by the points triangulated (DLT, normalised coordinates, P0 = [I|0], P = [R|t]) with
 * depth in (0, dist) in both cameras; R (row-major), t and the chosen mask out.  Returns the
 * count of the chosen candidate. */
int or_recover_pose(const double E[9], const float* p1, const float* p2, int n, const double K[4],
                    double dist, double* q_scratch, double R_out[9], double t_out[3], uint8_t* mask) {
  double* q1 = q_scratch;
  double* q2 = q_scratch + 2 * n;
  normalize_pts(p1, n, K, q1);
  normalize_pts(p2, n, K, q2);
  double R1[9], R2[9], t[3];
  or_decompose_essential(E, R1, R2, t);
  const double* Rs[4] = {R1, R2, R1, R2};
  const double sg[4] = {1.0, 1.0, -1.0, -1.0};
  static const double P0[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
  int good[4];
  for (int c = 0; c < 4; ++c) {
    double P1[12];
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) P1[4 * i + j] = Rs[c][3 * i + j];
      P1[4 * i + 3] = sg[c] * t[i];
    }
    int cnt = 0;
    for (int k = 0; k < n; ++k) cnt += cheiral(P0, P1, q1 + 2 * k, q2 + 2 * k, dist);
    good[c] = cnt;
  }
  /* OpenCV's order: (R1,t) if good1 >= the others, else (R2,t), else (R1,-t), else (R2,-t) */
  int ch;
  if (good[0] >= good[1] && good[0] >= good[2] && good[0] >= good[3]) ch = 0;
  else if (good[1] >= good[0] && good[1] >= good[2] && good[1] >= good[3]) ch = 1;
  else if (good[2] >= good[0] && good[2] >= good[1] && good[2] >= good[3]) ch = 2;
  else ch = 3;
  for (int i = 0; i < 9; ++i) R_out[i] = Rs[ch][i];
  for (int i = 0; i < 3; ++i) t_out[i] = sg[ch] * t[i];
  if (mask) {
    double P1[12];
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) P1[4 * i + j] = R_out[3 * i + j];
      P1[4 * i + 3] = t_out[i];
    }
    for (int k = 0; k < n; ++k) mask[k] = (uint8_t)cheiral(P0, P1, q1 + 2 * k, q2 + 2 * k, dist);
  }
  return good[ch];
}
