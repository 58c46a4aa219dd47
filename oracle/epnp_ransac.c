/*
 * ORACLE -- test infrastructure only.  Never linked into libonepose_hip.so.
 *
 * Plain-C restatement of the pose solve on the OnePose hot path:
 *   ransac_PnP (src/utils/eval_utils.py:18-42) =
 *     cv2.solvePnPRansac(pts3d*scale, pts2d, K, zeros(8), reprojectionError=5,
 *                        iterationsCount=10000, flags=cv2.SOLVEPNP_EPNP)
 *     + cv2.Rodrigues + tvec/scale.
 * The reference pins opencv_python==4.4.0.46 (requirements.txt:5), which is NOT installed
 * in this environment, and no OpenCV source is vendored: this file restates OpenCV 4.4's
 * published algorithm (modules/calib3d/src/solvepnp.cpp solvePnPRansac,
 * ptsetreg.cpp RANSACPointSetRegistrator::run / getSubset / RANSACUpdateNumIters,
 * epnp.cpp epnp::compute_pose, calibration.cpp cvRodrigues2 / cvProjectPoints2,
 * core/include/opencv2/core/operations.hpp cv::RNG):
 *   - points are converted to float32 before RANSAC (solvepnp.cpp, CV_64F -> CV_32F);
 *   - RNG is cv::RNG((uint64)-1): multiply-with-carry, state = (u32)state*4164903690 +
 *     (state>>32); uniform(0,n) = next() % n;
 *   - subsets: 5 distinct indices, redrawing duplicates (getSubset);
 *   - model: EPnP on the 5 points (rvec, tvec); error: float32 squared reprojection
 *     distance, inlier iff err <= (float)(thr*thr);
 *   - a model replaces the best iff goodCount > max(best, 4); niters then shrinks to
 *     RANSACUpdateNumIters(0.99, (n-good)/n, 5, niters);
 *   - the final pose is EPnP on all inliers (float32 points widened back to double);
 *     inliers are the RANSAC mask.
 * PARITY UNPINNED against OpenCV itself (cv2 absent): pinned instead by known-answer
 * synthetic scenes in tests/test_pnp_oracle.py.  The GPU implementation
 * (onepose_amd/csrc/pnp.hip) is checked against this file.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ----------------------------------------------------------------------------------- */
/* cv::RNG                                                                              */
/* ----------------------------------------------------------------------------------- */
static uint64_t rng_state;
static unsigned rng_next(void) {
  rng_state = (uint64_t)(unsigned)rng_state * 4164903690ULL + (unsigned)(rng_state >> 32);
  return (unsigned)rng_state;
}
static int rng_uniform(int a, int b) { return a == b ? a : (int)(rng_next() % (unsigned)(b - a)) + a; }

/* exported for tests: first `count` raw draws of cv::RNG((uint64)-1) */
void oracle_rng_draws(unsigned* out, int count) {
  rng_state = 0xFFFFFFFFFFFFFFFFULL;
  for (int i = 0; i < count; ++i) out[i] = rng_next();
}

/* ----------------------------------------------------------------------------------- */
/* small dense linear algebra (double)                                                   */
/* ----------------------------------------------------------------------------------- */

/* Cyclic Jacobi eigen-decomposition of the symmetric n x n matrix a (destroyed).
 * On return w[i] are eigenvalues sorted in decreasing order and row i of vt the
 * corresponding unit eigenvector (the "U^T" rows cvSVD(..., CV_SVD_U_T) returns for a
 * symmetric PSD matrix). */
static void jacobi_eigen(double* a, int n, double* w, double* vt) {
  double v[144];
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) v[i * n + j] = (i == j) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0, diag = 0.0;
    for (int i = 0; i < n; ++i) {
      diag += a[i * n + i] * a[i * n + i];
      for (int j = i + 1; j < n; ++j) off += a[i * n + j] * a[i * n + j];
    }
    if (off <= 1e-30 * diag || off == 0.0) break;
    for (int p = 0; p < n - 1; ++p) {
      for (int q = p + 1; q < n; ++q) {
        const double apq = a[p * n + q];
        if (apq == 0.0) continue;
        const double app = a[p * n + p], aqq = a[q * n + q];
        const double theta = (aqq - app) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < n; ++k) {
          const double akp = a[k * n + p], akq = a[k * n + q];
          a[k * n + p] = c * akp - s * akq;
          a[k * n + q] = s * akp + c * akq;
        }
        for (int k = 0; k < n; ++k) {
          const double apk = a[p * n + k], aqk = a[q * n + k];
          a[p * n + k] = c * apk - s * aqk;
          a[q * n + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < n; ++k) {
          const double vkp = v[k * n + p], vkq = v[k * n + q];
          v[k * n + p] = c * vkp - s * vkq;
          v[k * n + q] = s * vkp + c * vkq;
        }
      }
    }
  }
  int order[12];
  for (int i = 0; i < n; ++i) order[i] = i;
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j)
      if (a[order[j] * n + order[j]] > a[order[i] * n + order[i]]) {
        int t = order[i];
        order[i] = order[j];
        order[j] = t;
      }
  for (int i = 0; i < n; ++i) {
    w[i] = a[order[i] * n + order[i]];
    for (int k = 0; k < n; ++k) vt[i * n + k] = v[k * n + order[i]];
  }
}

/* Least squares min |A x - b| for A m x n (m >= n, full column rank) by Householder QR:
 * the solution cvSolve(A, b, x, CV_SVD) returns for a full-rank system. */
static void lstsq(const double* A_, const double* b_, int m, int n, double* x) {
  double A[6 * 6], b[6];
  memcpy(A, A_, sizeof(double) * m * n);
  memcpy(b, b_, sizeof(double) * m);
  for (int k = 0; k < n; ++k) {
    double norm = 0.0;
    for (int i = k; i < m; ++i) norm += A[i * n + k] * A[i * n + k];
    norm = sqrt(norm);
    if (norm == 0.0) continue;
    const double alpha = A[k * n + k] > 0 ? -norm : norm;
    double v[6];
    for (int i = 0; i < m; ++i) v[i] = 0.0;
    for (int i = k; i < m; ++i) v[i] = A[i * n + k];
    v[k] -= alpha;
    double vv = 0.0;
    for (int i = k; i < m; ++i) vv += v[i] * v[i];
    if (vv == 0.0) continue;
    for (int j = k; j < n; ++j) {
      double s = 0.0;
      for (int i = k; i < m; ++i) s += v[i] * A[i * n + j];
      s = 2.0 * s / vv;
      for (int i = k; i < m; ++i) A[i * n + j] -= s * v[i];
    }
    double s = 0.0;
    for (int i = k; i < m; ++i) s += v[i] * b[i];
    s = 2.0 * s / vv;
    for (int i = k; i < m; ++i) b[i] -= s * v[i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    for (int j = i + 1; j < n; ++j) s -= A[i * n + j] * x[j];
    x[i] = (A[i * n + i] != 0.0) ? s / A[i * n + i] : 0.0;
  }
}

/* 3x3 inverse via the adjugate (cvInvert(CC, CC_inv, CV_SVD) for a non-singular CC). */
static void inv3(const double* m, double* r) {
  const double c00 = m[4] * m[8] - m[5] * m[7];
  const double c01 = m[5] * m[6] - m[3] * m[8];
  const double c02 = m[3] * m[7] - m[4] * m[6];
  const double det = m[0] * c00 + m[1] * c01 + m[2] * c02;
  const double id = 1.0 / det;
  r[0] = c00 * id;
  r[1] = (m[2] * m[7] - m[1] * m[8]) * id;
  r[2] = (m[1] * m[5] - m[2] * m[4]) * id;
  r[3] = c01 * id;
  r[4] = (m[0] * m[8] - m[2] * m[6]) * id;
  r[5] = (m[2] * m[3] - m[0] * m[5]) * id;
  r[6] = c02 * id;
  r[7] = (m[1] * m[6] - m[0] * m[7]) * id;
  r[8] = (m[0] * m[4] - m[1] * m[3]) * id;
}

/* Orthogonal polar factor U V^T of a 3x3 matrix (what estimate_R_and_t builds from
 * cvSVD(ABt)), via the eigen-decomposition of A^T A. */
static void polar3(const double* A, double* R) {
  double ata[9], w[3], vt[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
      for (int k = 0; k < 3; ++k) s += A[k * 3 + i] * A[k * 3 + j];
      ata[i * 3 + j] = s;
    }
  jacobi_eigen(ata, 3, w, vt);
  /* U columns = A v_i / sigma_i, third completed by a cross product when degenerate */
  double u[3][3];
  for (int i = 0; i < 3; ++i) {
    const double sig = sqrt(w[i] > 0 ? w[i] : 0);
    for (int r = 0; r < 3; ++r) {
      double s = 0.0;
      for (int k = 0; k < 3; ++k) s += A[r * 3 + k] * vt[i * 3 + k];
      u[i][r] = sig > 1e-300 ? s / sig : 0.0;
    }
  }
  if (!(w[2] > 1e-24 * w[0])) {
    u[2][0] = u[0][1] * u[1][2] - u[0][2] * u[1][1];
    u[2][1] = u[0][2] * u[1][0] - u[0][0] * u[1][2];
    u[2][2] = u[0][0] * u[1][1] - u[0][1] * u[1][0];
    /* keep sign consistent with v3 = v1 x v2 so that U V^T is the polar factor */
    double vc[3] = {vt[1] * vt[5] - vt[2] * vt[4], vt[2] * vt[3] - vt[0] * vt[5],
                    vt[0] * vt[4] - vt[1] * vt[3]};
    const double sgn = (vc[0] * vt[6] + vc[1] * vt[7] + vc[2] * vt[8]) >= 0 ? 1.0 : -1.0;
    for (int r = 0; r < 3; ++r) u[2][r] *= sgn;
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
      for (int k = 0; k < 3; ++k) s += u[k][i] * vt[k * 3 + j];
      R[i * 3 + j] = s;
    }
}

/* ----------------------------------------------------------------------------------- */
/* EPnP (epnp.cpp)                                                                       */
/* ----------------------------------------------------------------------------------- */
typedef struct {
  int n;
  const double* pws; /* [n][3] */
  const double* us;  /* [n][2] */
  double* alphas;    /* [n][4] */
  double* pcs;       /* [n][3] */
  double fu, fv, uc, vc;
  double cws[4][3], ccs[4][3];
} Epnp;

static double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static double dist2(const double* a, const double* b) {
  return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
}

static void choose_control_points(Epnp* e) {
  for (int j = 0; j < 3; ++j) e->cws[0][j] = 0;
  for (int i = 0; i < e->n; ++i)
    for (int j = 0; j < 3; ++j) e->cws[0][j] += e->pws[3 * i + j];
  for (int j = 0; j < 3; ++j) e->cws[0][j] /= e->n;
  double m[9] = {0}, dc[3], uct[9];
  for (int i = 0; i < e->n; ++i) {
    double p[3];
    for (int j = 0; j < 3; ++j) p[j] = e->pws[3 * i + j] - e->cws[0][j];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) m[r * 3 + c] += p[r] * p[c];
  }
  jacobi_eigen(m, 3, dc, uct);
  for (int i = 1; i < 4; ++i) {
    const double k = sqrt(dc[i - 1] / e->n);
    for (int j = 0; j < 3; ++j) e->cws[i][j] = e->cws[0][j] + k * uct[3 * (i - 1) + j];
  }
}

static void compute_barycentric(Epnp* e) {
  double cc[9], ci[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 1; j < 4; ++j) cc[3 * i + j - 1] = e->cws[j][i] - e->cws[0][i];
  inv3(cc, ci);
  for (int i = 0; i < e->n; ++i) {
    const double* pi = e->pws + 3 * i;
    double* a = e->alphas + 4 * i;
    for (int j = 0; j < 3; ++j)
      a[1 + j] = ci[3 * j] * (pi[0] - e->cws[0][0]) + ci[3 * j + 1] * (pi[1] - e->cws[0][1]) +
                 ci[3 * j + 2] * (pi[2] - e->cws[0][2]);
    a[0] = 1.0f - a[1] - a[2] - a[3];
  }
}

static void compute_L_6x10(const double* ut, double* l) {
  const double* v[4] = {ut + 12 * 11, ut + 12 * 10, ut + 12 * 9, ut + 12 * 8};
  double dv[4][6][3];
  for (int i = 0; i < 4; ++i) {
    int a = 0, b = 1;
    for (int j = 0; j < 6; ++j) {
      for (int k = 0; k < 3; ++k) dv[i][j][k] = v[i][3 * a + k] - v[i][3 * b + k];
      b++;
      if (b > 3) {
        a++;
        b = a + 1;
      }
    }
  }
  for (int i = 0; i < 6; ++i) {
    double* row = l + 10 * i;
    row[0] = dot3(dv[0][i], dv[0][i]);
    row[1] = 2.0f * dot3(dv[0][i], dv[1][i]);
    row[2] = dot3(dv[1][i], dv[1][i]);
    row[3] = 2.0f * dot3(dv[0][i], dv[2][i]);
    row[4] = 2.0f * dot3(dv[1][i], dv[2][i]);
    row[5] = dot3(dv[2][i], dv[2][i]);
    row[6] = 2.0f * dot3(dv[0][i], dv[3][i]);
    row[7] = 2.0f * dot3(dv[1][i], dv[3][i]);
    row[8] = 2.0f * dot3(dv[2][i], dv[3][i]);
    row[9] = dot3(dv[3][i], dv[3][i]);
  }
}

static void compute_rho(const Epnp* e, double* rho) {
  rho[0] = dist2(e->cws[0], e->cws[1]);
  rho[1] = dist2(e->cws[0], e->cws[2]);
  rho[2] = dist2(e->cws[0], e->cws[3]);
  rho[3] = dist2(e->cws[1], e->cws[2]);
  rho[4] = dist2(e->cws[1], e->cws[3]);
  rho[5] = dist2(e->cws[2], e->cws[3]);
}

static void betas_approx_1(const double* L, const double* rho, double* betas) {
  double l[24], b4[4];
  for (int i = 0; i < 6; ++i) {
    l[i * 4 + 0] = L[i * 10 + 0];
    l[i * 4 + 1] = L[i * 10 + 1];
    l[i * 4 + 2] = L[i * 10 + 3];
    l[i * 4 + 3] = L[i * 10 + 6];
  }
  lstsq(l, rho, 6, 4, b4);
  if (b4[0] < 0) {
    betas[0] = sqrt(-b4[0]);
    betas[1] = -b4[1] / betas[0];
    betas[2] = -b4[2] / betas[0];
    betas[3] = -b4[3] / betas[0];
  } else {
    betas[0] = sqrt(b4[0]);
    betas[1] = b4[1] / betas[0];
    betas[2] = b4[2] / betas[0];
    betas[3] = b4[3] / betas[0];
  }
}

static void betas_approx_2(const double* L, const double* rho, double* betas) {
  double l[18], b3[3];
  for (int i = 0; i < 6; ++i)
    for (int k = 0; k < 3; ++k) l[i * 3 + k] = L[i * 10 + k];
  lstsq(l, rho, 6, 3, b3);
  if (b3[0] < 0) {
    betas[0] = sqrt(-b3[0]);
    betas[1] = (b3[2] < 0) ? sqrt(-b3[2]) : 0.0;
  } else {
    betas[0] = sqrt(b3[0]);
    betas[1] = (b3[2] > 0) ? sqrt(b3[2]) : 0.0;
  }
  if (b3[1] < 0) betas[0] = -betas[0];
  betas[2] = 0.0;
  betas[3] = 0.0;
}

static void betas_approx_3(const double* L, const double* rho, double* betas) {
  double l[30], b5[5];
  for (int i = 0; i < 6; ++i)
    for (int k = 0; k < 5; ++k) l[i * 5 + k] = L[i * 10 + k];
  lstsq(l, rho, 6, 5, b5);
  if (b5[0] < 0) {
    betas[0] = sqrt(-b5[0]);
    betas[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0;
  } else {
    betas[0] = sqrt(b5[0]);
    betas[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0;
  }
  if (b5[1] < 0) betas[0] = -betas[0];
  betas[2] = b5[3] / betas[0];
  betas[3] = 0.0;
}

/* epnp::qr_solve (epnp.cpp): the Householder variant EPnP ships for Gauss-Newton */
static void qr_solve_6x4(double* A, double* b, double* X) {
  const int nr = 6, nc = 4;
  double A1[6], A2[6];
  double* pA = A;
  double* ppAkk = pA;
  for (int k = 0; k < nc; k++) {
    double *ppAik1 = ppAkk, eta = fabs(*ppAik1);
    for (int i = k + 1; i < nr; i++) {
      double elt = fabs(*ppAik1);
      if (eta < elt) eta = elt;
      ppAik1 += nc;
    }
    if (eta == 0) {
      A1[k] = A2[k] = 0.0;
      return;
    } else {
      double *ppAik2 = ppAkk, sum2 = 0.0, inv_eta = 1. / eta;
      for (int i = k; i < nr; i++) {
        *ppAik2 *= inv_eta;
        sum2 += *ppAik2 * *ppAik2;
        ppAik2 += nc;
      }
      double sigma = sqrt(sum2);
      if (*ppAkk < 0) sigma = -sigma;
      *ppAkk += sigma;
      A1[k] = sigma * *ppAkk;
      A2[k] = -eta * sigma;
      for (int j = k + 1; j < nc; j++) {
        double *ppAik = ppAkk, sum = 0;
        for (int i = k; i < nr; i++) {
          sum += *ppAik * ppAik[j - k];
          ppAik += nc;
        }
        double tau = sum / A1[k];
        ppAik = ppAkk;
        for (int i = k; i < nr; i++) {
          ppAik[j - k] -= tau * *ppAik;
          ppAik += nc;
        }
      }
    }
    ppAkk += nc + 1;
  }
  double *ppAjj = pA, *pb = b;
  for (int j = 0; j < nc; j++) {
    double *ppAij = ppAjj, tau = 0;
    for (int i = j; i < nr; i++) {
      tau += *ppAij * pb[i];
      ppAij += nc;
    }
    tau /= A1[j];
    ppAij = ppAjj;
    for (int i = j; i < nr; i++) {
      pb[i] -= tau * *ppAij;
      ppAij += nc;
    }
    ppAjj += nc + 1;
  }
  double* pX = X;
  pX[nc - 1] = pb[nc - 1] / A2[nc - 1];
  for (int i = nc - 2; i >= 0; i--) {
    double *ppAij = pA + i * nc + (i + 1), sum = 0;
    for (int j = i + 1; j < nc; j++) {
      sum += *ppAij * pX[j];
      ppAij++;
    }
    pX[i] = (pb[i] - sum) / A2[i];
  }
}

static void gauss_newton(const double* L, const double* rho, double* betas) {
  double x[4] = {0, 0, 0, 0}; /* declared outside the loop, as epnp.cpp does */
  for (int it = 0; it < 5; ++it) {
    double A[24], b[6];
    for (int i = 0; i < 6; ++i) {
      const double* r = L + i * 10;
      A[i * 4 + 0] = 2 * r[0] * betas[0] + r[1] * betas[1] + r[3] * betas[2] + r[6] * betas[3];
      A[i * 4 + 1] = r[1] * betas[0] + 2 * r[2] * betas[1] + r[4] * betas[2] + r[7] * betas[3];
      A[i * 4 + 2] = r[3] * betas[0] + r[4] * betas[1] + 2 * r[5] * betas[2] + r[8] * betas[3];
      A[i * 4 + 3] = r[6] * betas[0] + r[7] * betas[1] + r[8] * betas[2] + 2 * r[9] * betas[3];
      b[i] = rho[i] - (r[0] * betas[0] * betas[0] + r[1] * betas[0] * betas[1] +
                       r[2] * betas[1] * betas[1] + r[3] * betas[0] * betas[2] +
                       r[4] * betas[1] * betas[2] + r[5] * betas[2] * betas[2] +
                       r[6] * betas[0] * betas[3] + r[7] * betas[1] * betas[3] +
                       r[8] * betas[2] * betas[3] + r[9] * betas[3] * betas[3]);
    }
    qr_solve_6x4(A, b, x);
    for (int i = 0; i < 4; ++i) betas[i] += x[i];
  }
}

static double reprojection_error(const Epnp* e, const double R[3][3], const double t[3]) {
  double sum2 = 0.0;
  for (int i = 0; i < e->n; ++i) {
    const double* pw = e->pws + 3 * i;
    const double Xc = dot3(R[0], pw) + t[0];
    const double Yc = dot3(R[1], pw) + t[1];
    const double inv_Zc = 1.0 / (dot3(R[2], pw) + t[2]);
    const double ue = e->uc + e->fu * Xc * inv_Zc;
    const double ve = e->vc + e->fv * Yc * inv_Zc;
    const double u = e->us[2 * i], v = e->us[2 * i + 1];
    sum2 += sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
  }
  return sum2 / e->n;
}

static double compute_R_and_t(Epnp* e, const double* ut, const double* betas, double R[3][3],
                              double t[3]) {
  for (int i = 0; i < 4; ++i) e->ccs[i][0] = e->ccs[i][1] = e->ccs[i][2] = 0.0;
  for (int i = 0; i < 4; ++i) {
    const double* v = ut + 12 * (11 - i);
    for (int j = 0; j < 4; ++j)
      for (int k = 0; k < 3; ++k) e->ccs[j][k] += betas[i] * v[3 * j + k];
  }
  for (int i = 0; i < e->n; ++i) {
    const double* a = e->alphas + 4 * i;
    double* pc = e->pcs + 3 * i;
    for (int j = 0; j < 3; ++j)
      pc[j] = a[0] * e->ccs[0][j] + a[1] * e->ccs[1][j] + a[2] * e->ccs[2][j] + a[3] * e->ccs[3][j];
  }
  if (e->pcs[2] < 0.0) { /* solve_for_sign */
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 3; ++j) e->ccs[i][j] = -e->ccs[i][j];
    for (int i = 0; i < 3 * e->n; ++i) e->pcs[i] = -e->pcs[i];
  }
  /* estimate_R_and_t */
  double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
  for (int i = 0; i < e->n; ++i)
    for (int j = 0; j < 3; ++j) {
      pc0[j] += e->pcs[3 * i + j];
      pw0[j] += e->pws[3 * i + j];
    }
  for (int j = 0; j < 3; ++j) {
    pc0[j] /= e->n;
    pw0[j] /= e->n;
  }
  double abt[9] = {0};
  for (int i = 0; i < e->n; ++i) {
    const double* pc = e->pcs + 3 * i;
    const double* pw = e->pws + 3 * i;
    for (int j = 0; j < 3; ++j) {
      abt[3 * j + 0] += (pc[j] - pc0[j]) * (pw[0] - pw0[0]);
      abt[3 * j + 1] += (pc[j] - pc0[j]) * (pw[1] - pw0[1]);
      abt[3 * j + 2] += (pc[j] - pc0[j]) * (pw[2] - pw0[2]);
    }
  }
  double Rm[9];
  polar3(abt, Rm);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R[i][j] = Rm[i * 3 + j];
  const double det = R[0][0] * R[1][1] * R[2][2] + R[0][1] * R[1][2] * R[2][0] +
                     R[0][2] * R[1][0] * R[2][1] - R[0][2] * R[1][1] * R[2][0] -
                     R[0][1] * R[1][0] * R[2][2] - R[0][0] * R[1][2] * R[2][1];
  if (det < 0) {
    R[2][0] = -R[2][0];
    R[2][1] = -R[2][1];
    R[2][2] = -R[2][2];
  }
  t[0] = pc0[0] - dot3(R[0], pw0);
  t[1] = pc0[1] - dot3(R[1], pw0);
  t[2] = pc0[2] - dot3(R[2], pw0);
  return reprojection_error(e, R, t);
}

/* Exactly 4 correspondences give M (8 x 12) a 4-dimensional null space, so the basis an
 * eigensolver returns for it -- and with it EPnP's beta approximations -- is arbitrary (it
 * differs between eigensolvers and OpenCV versions).  For n == 4 both implementations here
 * use a canonical basis instead: the projector P = I - M^T (M M^T)^-1 M (Gauss-Jordan with
 * partial pivoting), then Gram-Schmidt of P's columns in index order, keeping residuals with
 * squared norm > 0.05.  v[i] is the null vector EPnP reads as its i-th (ut row 11 - i). */
static void null4_basis(const double M[8][12], double v[4][12]) {
  double G[8][8], X[8][12];
  for (int a = 0; a < 8; ++a) {
    for (int b = 0; b < 8; ++b) {
      double acc = 0;
      for (int k = 0; k < 12; ++k) acc += M[a][k] * M[b][k];
      G[a][b] = acc;
    }
    for (int k = 0; k < 12; ++k) X[a][k] = M[a][k];
  }
  for (int c = 0; c < 8; ++c) { /* G X = M, Gauss-Jordan with partial pivoting */
    int piv = c;
    for (int r = c + 1; r < 8; ++r)
      if (fabs(G[r][c]) > fabs(G[piv][c])) piv = r;
    if (piv != c) {
      for (int k = 0; k < 8; ++k) {
        const double tmp = G[c][k];
        G[c][k] = G[piv][k];
        G[piv][k] = tmp;
      }
      for (int k = 0; k < 12; ++k) {
        const double tmp = X[c][k];
        X[c][k] = X[piv][k];
        X[piv][k] = tmp;
      }
    }
    const double inv = 1.0 / G[c][c];
    for (int k = 0; k < 8; ++k) G[c][k] *= inv;
    for (int k = 0; k < 12; ++k) X[c][k] *= inv;
    for (int r = 0; r < 8; ++r) {
      if (r == c) continue;
      const double f = G[r][c];
      if (f == 0.0) continue;
      for (int k = 0; k < 8; ++k) G[r][k] -= f * G[c][k];
      for (int k = 0; k < 12; ++k) X[r][k] -= f * X[c][k];
    }
  }
  double P[12][12];
  for (int a = 0; a < 12; ++a)
    for (int b = 0; b < 12; ++b) {
      double acc = 0;
      for (int r = 0; r < 8; ++r) acc += M[r][a] * X[r][b];
      P[a][b] = (a == b ? 1.0 : 0.0) - acc;
    }
  int nq = 0;
  for (int pass = 0; pass < 2 && nq < 4; ++pass) {
    const double keep = pass == 0 ? 0.05 : 1e-12;
    for (int c = 0; c < 12 && nq < 4; ++c) {
      double w[12];
      for (int k = 0; k < 12; ++k) w[k] = P[k][c];
      for (int j = 0; j < nq; ++j) {
        double d = 0;
        for (int k = 0; k < 12; ++k) d += v[j][k] * w[k];
        for (int k = 0; k < 12; ++k) w[k] -= d * v[j][k];
      }
      double nn = 0;
      for (int k = 0; k < 12; ++k) nn += w[k] * w[k];
      if (nn <= keep) continue;
      nn = 1.0 / sqrt(nn);
      for (int k = 0; k < 12; ++k) v[nq][k] = w[k] * nn;
      ++nq;
    }
  }
}

/* epnp::compute_pose: R (3x3 row-major) and t from n >= 4 correspondences */
void oracle_epnp(const double* pws, const double* us, int n, const double* K, double* R_out,
                 double* t_out) {
  Epnp e;
  e.n = n;
  e.pws = pws;
  e.us = us;
  e.alphas = (double*)malloc(sizeof(double) * 4 * n);
  e.pcs = (double*)malloc(sizeof(double) * 3 * n);
  e.uc = K[2];
  e.vc = K[5];
  e.fu = K[0];
  e.fv = K[4];
  choose_control_points(&e);
  compute_barycentric(&e);
  double mtm[144] = {0};
  for (int i = 0; i < n; ++i) {
    const double* as = e.alphas + 4 * i;
    const double u = us[2 * i], v = us[2 * i + 1];
    double r1[12], r2[12];
    for (int k = 0; k < 4; ++k) {
      r1[3 * k] = as[k] * e.fu;
      r1[3 * k + 1] = 0.0;
      r1[3 * k + 2] = as[k] * (e.uc - u);
      r2[3 * k] = 0.0;
      r2[3 * k + 1] = as[k] * e.fv;
      r2[3 * k + 2] = as[k] * (e.vc - v);
    }
    for (int a = 0; a < 12; ++a)
      for (int b = 0; b < 12; ++b) mtm[a * 12 + b] += r1[a] * r1[b] + r2[a] * r2[b];
  }
  double d[12], ut[144];
  jacobi_eigen(mtm, 12, d, ut);
  if (n == 4) { /* canonical null-space basis (see null4_basis) */
    double M[8][12], v4[4][12];
    for (int i = 0; i < 4; ++i) {
      const double* as = e.alphas + 4 * i;
      const double u = us[2 * i], v = us[2 * i + 1];
      for (int k = 0; k < 4; ++k) {
        M[2 * i][3 * k] = as[k] * e.fu;
        M[2 * i][3 * k + 1] = 0.0;
        M[2 * i][3 * k + 2] = as[k] * (e.uc - u);
        M[2 * i + 1][3 * k] = 0.0;
        M[2 * i + 1][3 * k + 1] = as[k] * e.fv;
        M[2 * i + 1][3 * k + 2] = as[k] * (e.vc - v);
      }
    }
    null4_basis(M, v4);
    for (int i = 0; i < 4; ++i)
      for (int k = 0; k < 12; ++k) ut[12 * (11 - i) + k] = v4[i][k];
  }
  double L[60], rho[6];
  compute_L_6x10(ut, L);
  compute_rho(&e, rho);
  double Betas[4][4], errs[4], Rs[4][3][3], ts[4][3];
  betas_approx_1(L, rho, Betas[1]);
  gauss_newton(L, rho, Betas[1]);
  errs[1] = compute_R_and_t(&e, ut, Betas[1], Rs[1], ts[1]);
  betas_approx_2(L, rho, Betas[2]);
  gauss_newton(L, rho, Betas[2]);
  errs[2] = compute_R_and_t(&e, ut, Betas[2], Rs[2], ts[2]);
  betas_approx_3(L, rho, Betas[3]);
  gauss_newton(L, rho, Betas[3]);
  errs[3] = compute_R_and_t(&e, ut, Betas[3], Rs[3], ts[3]);
  int N = 1;
  if (errs[2] < errs[1]) N = 2;
  if (errs[3] < errs[N]) N = 3;
  for (int i = 0; i < 3; ++i) {
    t_out[i] = ts[N][i];
    for (int j = 0; j < 3; ++j) R_out[i * 3 + j] = Rs[N][i][j];
  }
  free(e.alphas);
  free(e.pcs);
}

/* cvRodrigues2, matrix -> vector (the SVD re-orthonormalisation is skipped: R is already
 * orthonormal to rounding) and vector -> matrix */
void oracle_rodrigues_m2v(const double* R, double* r) {
  double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
  double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
  double c = (R[0] + R[4] + R[8] - 1) * 0.5;
  c = c > 1. ? 1. : c < -1. ? -1. : c;
  double theta = acos(c);
  if (s < 1e-5) {
    if (c > 0) {
      rx = ry = rz = 0;
    } else {
      double t = (R[0] + 1) * 0.5;
      rx = sqrt(t > 0 ? t : 0.);
      t = (R[4] + 1) * 0.5;
      ry = sqrt(t > 0 ? t : 0.) * (R[1] < 0 ? -1. : 1.);
      t = (R[8] + 1) * 0.5;
      rz = sqrt(t > 0 ? t : 0.) * (R[2] < 0 ? -1. : 1.);
      if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
      theta /= sqrt(rx * rx + ry * ry + rz * rz);
      rx *= theta;
      ry *= theta;
      rz *= theta;
    }
  } else {
    double vth = 1 / (2 * s);
    vth *= theta;
    rx *= vth;
    ry *= vth;
    rz *= vth;
  }
  r[0] = rx;
  r[1] = ry;
  r[2] = rz;
}

void oracle_rodrigues_v2m(const double* r, double* R) {
  double theta = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
  if (theta < DBL_EPSILON) {
    for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
    return;
  }
  const double c = cos(theta), s = sin(theta), c1 = 1. - c;
  const double itheta = theta ? 1. / theta : 0.;
  const double x = r[0] * itheta, y = r[1] * itheta, z = r[2] * itheta;
  const double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
  const double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
  for (int i = 0; i < 9; ++i) R[i] = c * ((i % 4 == 0) ? 1.0 : 0.0) + c1 * rrt[i] + s * rx[i];
}

/* squared float reprojection errors of PnPRansacCallback::computeError */
static void reproj_errors(const float* p2, const float* p3, int n, const double* K,
                          const double* rvec, const double* tvec, float* err) {
  double R[9];
  oracle_rodrigues_v2m(rvec, R);
  const double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
  for (int i = 0; i < n; ++i) {
    const double X = p3[3 * i], Y = p3[3 * i + 1], Z = p3[3 * i + 2];
    const double x = R[0] * X + R[1] * Y + R[2] * Z + tvec[0];
    const double y = R[3] * X + R[4] * Y + R[5] * Z + tvec[1];
    double z = R[6] * X + R[7] * Y + R[8] * Z + tvec[2];
    z = z ? 1. / z : 1;
    const float u = (float)(x * z * fx + cx);
    const float v = (float)(y * z * fy + cy);
    const float du = p2[2 * i] - u, dv = p2[2 * i + 1] - v;
    const volatile float du2 = du * du, dv2 = dv * dv; /* no contraction */
    err[i] = du2 + dv2;
  }
}

static int update_num_iters(double p, double ep, int model_points, int max_iters) {
  p = p > 0 ? p : 0;
  p = p < 1 ? p : 1;
  ep = ep > 0 ? ep : 0;
  ep = ep < 1 ? ep : 1;
  double num = 1. - p > DBL_MIN ? 1. - p : DBL_MIN;
  double denom = 1. - pow(1. - ep, model_points);
  if (denom < DBL_MIN) return 0;
  num = log(num);
  denom = log(denom);
  return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)lrint(num / denom);
}

static void epnp_rt(const float* p2, const float* p3, const int* idx, int n, const double* K,
                    double* rvec, double* tvec) {
  double* pws = (double*)malloc(sizeof(double) * 3 * n);
  double* us = (double*)malloc(sizeof(double) * 2 * n);
  for (int i = 0; i < n; ++i) {
    const int j = idx ? idx[i] : i;
    for (int k = 0; k < 3; ++k) pws[3 * i + k] = p3[3 * j + k];
    for (int k = 0; k < 2; ++k) us[2 * i + k] = p2[2 * j + k];
  }
  double R[9];
  oracle_epnp(pws, us, n, K, R, tvec);
  oracle_rodrigues_m2v(R, rvec);
  free(pws);
  free(us);
}

/* ---- P3P (Gao et al. 2003, the kernel cv::solvePnPRansac switches to for exactly 4 points:
 * model_points = 4, ransac_kernel_method = SOLVEPNP_P3P).  With count == model_points the
 * RANSAC registrator runs the kernel once on all points and, when it yields a model, marks all
 * 4 inliers; the final refit is solvePnP(EPNP) over them.  So P3P only decides model / no
 * model; the pose is the EPnP of the 4 points.  Lengths follow Gao's law-of-cosines system
 * with x = |P0|/|P2|, y = |P1|/|P2|; y is eliminated linearly (b*Eq1 + (1-a)*Eq2) and the
 * quartic in x is Eq2 after substitution.  Real roots: recursive derivative bracketing +
 * bisection (deterministic; pnp.hip runs the same arithmetic). */
static double poly_eval(const double* c, int deg, double x) { /* c[0] + c[1] x + ... */
  double v = c[deg];
  for (int i = deg - 1; i >= 0; --i) v = v * x + c[i];
  return v;
}

static double bisect_root(const double* c, int deg, double lo, double hi) {
  double flo = poly_eval(c, deg, lo);
  for (int it = 0; it < 200; ++it) {
    const double mid = 0.5 * (lo + hi);
    if (mid <= lo || mid >= hi) break;
    const double fm = poly_eval(c, deg, mid);
    if (fm == 0.0) return mid;
    if ((fm < 0) == (flo < 0)) {
      lo = mid;
      flo = fm;
    } else {
      hi = mid;
    }
  }
  return 0.5 * (lo + hi);
}

/* real roots (ascending) of c[0..deg], deg <= 4, c[deg] != 0 */
static int real_roots(const double* c, int deg, double* roots) {
  if (deg == 1) {
    roots[0] = -c[0] / c[1];
    return 1;
  }
  double bound = 0.0; /* Cauchy bound */
  for (int i = 0; i < deg; ++i) {
    const double q = fabs(c[i] / c[deg]);
    bound = q > bound ? q : bound;
  }
  bound += 1.0;
  double dc[4], crit[4];
  for (int i = 1; i <= deg; ++i) dc[i - 1] = i * c[i];
  const int nc = real_roots(dc, deg - 1, crit);
  double pts[6];
  int np = 0;
  pts[np++] = -bound;
  for (int i = 0; i < nc; ++i)
    if (crit[i] > -bound && crit[i] < bound) pts[np++] = crit[i];
  pts[np++] = bound;
  int n = 0;
  for (int i = 0; i + 1 < np; ++i) {
    const double fa = poly_eval(c, deg, pts[i]), fb = poly_eval(c, deg, pts[i + 1]);
    if (fa == 0.0) {
      if (n == 0 || roots[n - 1] != pts[i]) roots[n++] = pts[i];
    } else if ((fa < 0) != (fb < 0) && fb != 0.0) {
      roots[n++] = bisect_root(c, deg, pts[i], pts[i + 1]);
    }
  }
  if (poly_eval(c, deg, pts[np - 1]) == 0.0) roots[n++] = pts[np - 1];
  return n;
}

/* number of P3P solutions from the first three correspondences (p3p::solve's lengths) */
int oracle_p3p_solutions(const float* p2, const float* p3, const double* K) {
  const double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
  double bear[3][3], P[3][3];
  for (int i = 0; i < 3; ++i) {
    double mu = (p2[2 * i] - cx) / fx, mv = (p2[2 * i + 1] - cy) / fy;
    const double mk = 1.0 / sqrt(mu * mu + mv * mv + 1.0);
    bear[i][0] = mu * mk;
    bear[i][1] = mv * mk;
    bear[i][2] = mk;
    for (int k = 0; k < 3; ++k) P[i][k] = p3[3 * i + k];
  }
  const double d0 = sqrt(dist2(P[1], P[2])), d1 = sqrt(dist2(P[0], P[2])),
               d2 = sqrt(dist2(P[0], P[1]));
  const double p = 2.0 * dot3(bear[1], bear[2]), q = 2.0 * dot3(bear[0], bear[2]),
               r = 2.0 * dot3(bear[0], bear[1]);
  if (p * p + q * q + r * r - p * q * r - 1.0 == 0.0) return 0; /* Gao's degenerate case */
  if (d2 == 0.0) return 0;
  const double a = (d0 * d0) / (d2 * d2), b = (d1 * d1) / (d2 * d2);
  /* y = N(x) / (b E(x)); quartic -N^2 + b r x N E + b Q E^2 = 0 */
  const double n2 = -(1.0 - a - b), n1 = (1.0 - a) * q, n0 = -(1.0 - a + b);
  const double e1 = r, e0 = -p;
  const double q2 = 1.0 - b, q1 = -q, q0 = 1.0;
  double c[5] = {0, 0, 0, 0, 0};
  /* -N^2 */
  c[4] -= n2 * n2;
  c[3] -= 2.0 * n2 * n1;
  c[2] -= n1 * n1 + 2.0 * n2 * n0;
  c[1] -= 2.0 * n1 * n0;
  c[0] -= n0 * n0;
  /* b r x N E:  N E = (n2 x^2 + n1 x + n0)(e1 x + e0) */
  const double ne3 = n2 * e1, ne2 = n2 * e0 + n1 * e1, ne1 = n1 * e0 + n0 * e1, ne0 = n0 * e0;
  c[4] += b * r * ne3;
  c[3] += b * r * ne2;
  c[2] += b * r * ne1;
  c[1] += b * r * ne0;
  /* b Q E^2 */
  const double ee2 = e1 * e1, ee1 = 2.0 * e1 * e0, ee0 = e0 * e0;
  c[4] += b * q2 * ee2;
  c[3] += b * (q2 * ee1 + q1 * ee2);
  c[2] += b * (q2 * ee0 + q1 * ee1 + q0 * ee2);
  c[1] += b * (q1 * ee0 + q0 * ee1);
  c[0] += b * q0 * ee0;
  if (c[4] == 0.0) return 0; /* Gao's A == 0 */
  double xs[4];
  const int nr = real_roots(c, 4, xs);
  int sols = 0;
  for (int i = 0; i < nr; ++i) {
    const double x = xs[i];
    if (x <= 0.0) continue;
    const double den = b * (e1 * x + e0);
    if (den == 0.0) continue;
    const double y = (n2 * x * x + n1 * x + n0) / den;
    if (y <= 0.0) continue;
    const double v = x * x + y * y - x * y * r;
    if (v <= 0.0) continue;
    ++sols; /* lengths (x Z, y Z, Z), Z = d2 / sqrt(v): a pose aligns the three points */
  }
  return sols;
}

/* Returns status (0 ok, 1 <4 points, 2 no model); pose34 = [R | t/scale]
 * with R = Rodrigues(rvec) as eval_utils.py:31-34 builds it. */
int oracle_pnp_ransac(const float* p2, const float* p3, int n, const double* K, double scale,
                      float reproj_error, int max_iters, double confidence, double* pose34,
                      unsigned char* mask, int* n_inliers, int* iters_run) {
  for (int i = 0; i < 12; ++i) pose34[i] = (i % 5 == 0) ? 1.0 : 0.0;
  for (int i = 0; i < n; ++i) mask[i] = 0;
  *n_inliers = 0;
  if (iters_run) *iters_run = 0;
  if (n < 4) return 1;
  double rvec[3], tvec[3];
  if (n == 4) { /* P3P kernel decides model / no model; refit EPnP over all four */
    if (oracle_p3p_solutions(p2, p3, K) == 0) return 2;
    epnp_rt(p2, p3, NULL, n, K, rvec, tvec);
    for (int i = 0; i < n; ++i) mask[i] = 1;
    *n_inliers = n;
  } else if (n == 5) { /* count == model_points: the EPnP kernel once, all inliers */
    epnp_rt(p2, p3, NULL, n, K, rvec, tvec);
    for (int i = 0; i < n; ++i) mask[i] = 1;
    *n_inliers = n;
  } else {
    const int model_points = 5;
    rng_state = 0xFFFFFFFFFFFFFFFFULL;
    const float thr = (float)((double)reproj_error * (double)reproj_error);
    int niters = max_iters > 1 ? max_iters : 1;
    int max_good = 0;
    double best_r[3] = {0}, best_t[3] = {0};
    float* err = (float*)malloc(sizeof(float) * n);
    unsigned char* m = (unsigned char*)malloc(n);
    int iter;
    for (iter = 0; iter < niters; ++iter) {
      int idx[5];
      for (int i = 0; i < model_points;) { /* getSubset; checkSubset is always true for PnP */
        int ii, j;
        for (;;) {
          ii = idx[i] = rng_uniform(0, n);
          for (j = 0; j < i; ++j)
            if (ii == idx[j]) break;
          if (j == i) break;
        }
        ++i;
      }
      epnp_rt(p2, p3, idx, model_points, K, rvec, tvec);
      reproj_errors(p2, p3, n, K, rvec, tvec, err);
      int good = 0;
      for (int i = 0; i < n; ++i) {
        m[i] = err[i] <= thr;
        good += m[i];
      }
      if (good > (max_good > model_points - 1 ? max_good : model_points - 1)) {
        memcpy(mask, m, n);
        memcpy(best_r, rvec, sizeof(rvec));
        memcpy(best_t, tvec, sizeof(tvec));
        max_good = good;
        niters = update_num_iters(confidence, (double)(n - good) / n, model_points, niters);
      }
    }
    if (iters_run) *iters_run = iter;
    free(err);
    free(m);
    if (max_good <= 0) {
      for (int i = 0; i < n; ++i) mask[i] = 0;
      return 2;
    }
    int* inl = (int*)malloc(sizeof(int) * n);
    int k = 0;
    for (int i = 0; i < n; ++i)
      if (mask[i]) inl[k++] = i;
    epnp_rt(p2, p3, inl, k, K, rvec, tvec);
    free(inl);
    *n_inliers = k;
  }
  double R[9];
  oracle_rodrigues_v2m(rvec, R);
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) pose34[i * 4 + j] = R[i * 3 + j];
    pose34[i * 4 + 3] = tvec[i] / scale;
  }
  return 0;
}
