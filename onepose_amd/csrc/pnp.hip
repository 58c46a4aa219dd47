// Batched RANSAC-EPnP on gfx950: cv2.solvePnPRansac(..., SOLVEPNP_EPNP) as OpenCV 4.4 runs
// it (see include/onepose_hip.h and oracle/epnp_ransac.c for the algorithm statement),
// one workgroup per frame.
//
// Per RANSAC round the workgroup takes the next 64 iterations of OpenCV's loop:
//   1. lane 0 draws the 64 subsets from the cv::RNG stream (sequential by definition:
//      duplicate indices are redrawn);
//   2. wave 0 solves one 5-point EPnP per lane (rvec, tvec);
//   3. all 256 threads count inliers of the 64 models over the frame's points (float32
//      squared reprojection error <= thr^2, as PnPRansacCallback::computeError);
//   4. lane 0 replays OpenCV's acceptance rule in iteration order (goodCount >
//      max(best, 4) -> new best, niters = RANSACUpdateNumIters(...)) and stops the loop
//      exactly where OpenCV would.
// Iterations evaluated beyond the stopping point are discarded, so the chosen model, the
// inlier mask and the iteration count are those of the sequential algorithm.  The final
// pose is a workgroup-parallel EPnP over the inliers.
#include "common.h"

// The pose kernels are compiled for one wave per SIMD (amdgpu_waves_per_eu(1)): a wave may use
// a whole SIMD's register file. 2 and 4 were measured slower or equal.
// "// @phase N" comments mark the pose kernels' phases; the pose probe's generated copy of
// this file (tools/probe_src.sh) turns them into stamps.

namespace onepose {
namespace {

constexpr int kModelPoints = 5;
constexpr int kRound = 64;
constexpr int kThreads = 256;
// cv::RNG (multiply-with-carry): state' = (state & 0xffffffff) * kMwcA + (state >> 32)
constexpr unsigned long long kMwcA = 4164903690ull;
constexpr unsigned long long kMwcM = kMwcA * 4294967296ull - 1ull;   // < 2^64
constexpr int kRngPrefix = 8, kRngPos = kRngPrefix + 6 * 64;   // draws generated per round

// A^(6 l) mod kMwcM, l = 0..63 (compile time)
constexpr unsigned long long mwc_mulmod_c(unsigned long long a, unsigned long long b) {
  return (unsigned long long)((unsigned __int128)a * b % kMwcM);
}
struct MwcJumps {
  unsigned long long v[64];
  constexpr MwcJumps() : v() {
    unsigned long long a6 = 1ull;
    for (int i = 0; i < 6; ++i) a6 = mwc_mulmod_c(a6, kMwcA);
    unsigned long long x = 1ull;
    for (int l = 0; l < 64; ++l) {
      v[l] = x;
      x = mwc_mulmod_c(x, a6);
    }
  }
};
__constant__ const MwcJumps kMwcJumps = MwcJumps();

// ---------------------------------------------------------------------------------------
// small dense linear algebra, double
// ---------------------------------------------------------------------------------------
// Cyclic Jacobi for the 3x3 symmetric matrices (PCA of the control points, polar factor):
// eigenvalues descending in w, eigenvectors as rows of vt.  Static indices only.
__device__ __forceinline__ void jacobi3(double* a, double* w, double* vt) {
  double v[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  for (int sweep = 0; sweep < 30; ++sweep) {
    const double off = a[1] * a[1] + a[2] * a[2] + a[5] * a[5];
    const double diag = a[0] * a[0] + a[4] * a[4] + a[8] * a[8];
    if (off <= 1e-30 * diag || off == 0.0) break;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int q = p + 1; q < 3; ++q) {
        const double apq = a[p * 3 + q];
        if (apq != 0.0) {
          const double theta = (a[q * 3 + q] - a[p * 3 + p]) / (2.0 * apq);
          const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
          const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const double akp = a[k * 3 + p], akq = a[k * 3 + q];
            a[k * 3 + p] = c * akp - s * akq;
            a[k * 3 + q] = s * akp + c * akq;
          }
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const double apk = a[p * 3 + k], aqk = a[q * 3 + k];
            a[p * 3 + k] = c * apk - s * aqk;
            a[q * 3 + k] = s * apk + c * aqk;
          }
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const double vkp = v[k * 3 + p], vkq = v[k * 3 + q];
            v[k * 3 + p] = c * vkp - s * vkq;
            v[k * 3 + q] = s * vkp + c * vkq;
          }
        }
      }
    }
  }
  double e[3] = {a[0], a[4], a[8]};
  double c0[3] = {v[0], v[3], v[6]}, c1[3] = {v[1], v[4], v[7]}, c2[3] = {v[2], v[5], v[8]};
  auto cswap = [](double& x, double& y, double* u, double* z) {
    if (y > x) {
      double t = x; x = y; y = t;
#pragma unroll
      for (int k = 0; k < 3; ++k) { t = u[k]; u[k] = z[k]; z[k] = t; }
    }
  };
  cswap(e[0], e[1], c0, c1);
  cswap(e[1], e[2], c1, c2);
  cswap(e[0], e[1], c0, c1);
  w[0] = e[0]; w[1] = e[1]; w[2] = e[2];
#pragma unroll
  for (int k = 0; k < 3; ++k) { vt[k] = c0[k]; vt[3 + k] = c1[k]; vt[6 + k] = c2[k]; }
}

// The four eigenvectors of the symmetric 12x12 matrix M^T M with the smallest eigenvalues,
// ascending (vec[0] = smallest) -- the rows 11, 10, 9, 8 of the U^T that epnp.cpp takes
// from cvSVD(MtM).  Register-resident (static indices only):
//   1. Householder tridiagonalisation T = Q^T A Q (reflectors kept in A's lower part);
//   2. block inverse iteration with 4 vectors on T + sigma I (LDL^T, sigma = 1e-9 |T|),
//      until the 4-dimensional subspace stops moving;
//   3. Rayleigh-Ritz on the 4x4 projection (Jacobi), then back-transform through Q.
// The invariant subspace is the same one any exact eigen-solver returns; inside a
// (numerically) degenerate cluster the basis is arbitrary, as it is for cvSVD.
#define LI(i, j) ((i) * ((i) + 1) / 2 + (j))
// hh: 55 doubles of per-lane scratch (LDS), element q at hh[q * hs], where the reflectors
// wait for the back-transform instead of occupying registers during the iteration.
template <int ITERS>
__device__ __forceinline__ void eig12_small4(double (&a)[78], double (&vec)[4][12], double* hh, int hs) {
  constexpr int n = 12;
  double tau[n - 2], e[n - 1], d[n];
#pragma unroll
  for (int k = 0; k < n - 2; ++k) {
    const double alpha = a[LI(k + 1, k)];
    double xn = 0.0;
#pragma unroll
    for (int i = k + 2; i < n; ++i) xn += a[LI(i, k)] * a[LI(i, k)];
    double beta = alpha, tk = 0.0;
    if (xn != 0.0) {
      beta = -copysign(sqrt(alpha * alpha + xn), alpha);
      tk = (beta - alpha) / beta;
      const double sc = 1.0 / (alpha - beta);
#pragma unroll
      for (int i = k + 2; i < n; ++i) a[LI(i, k)] *= sc;
    }
    tau[k] = tk;
    e[k] = beta;
    if (tk != 0.0) {
      // v = [1, a[k+2..][k]] on rows k+1..n-1;  p = tk * A22 v
      double pv[n];
#pragma unroll
      for (int i = k + 1; i < n; ++i) {
        double s = 0.0;
#pragma unroll
        for (int j = k + 1; j < n; ++j) {
          const double vj = (j == k + 1) ? 1.0 : a[LI(j, k)];
          const double aij = (i >= j) ? a[LI(i, j)] : a[LI(j, i)];
          s += aij * vj;
        }
        pv[i] = tk * s;
      }
      double pvv = 0.0;
#pragma unroll
      for (int i = k + 1; i < n; ++i) pvv += pv[i] * ((i == k + 1) ? 1.0 : a[LI(i, k)]);
      const double half = 0.5 * tk * pvv;
#pragma unroll
      for (int i = k + 1; i < n; ++i) pv[i] -= half * ((i == k + 1) ? 1.0 : a[LI(i, k)]);
#pragma unroll
      for (int i = k + 1; i < n; ++i) {
        const double vi = (i == k + 1) ? 1.0 : a[LI(i, k)];
#pragma unroll
        for (int j = k + 1; j <= i; ++j) {
          const double vj = (j == k + 1) ? 1.0 : a[LI(j, k)];
          a[LI(i, j)] -= vi * pv[j] + pv[i] * vj;
        }
      }
    }
  }
  e[n - 2] = a[LI(n - 1, n - 2)];
#pragma unroll
  for (int i = 0; i < n; ++i) d[i] = a[LI(i, i)];
  {
    int q = 0;
#pragma unroll
    for (int k = 0; k < n - 2; ++k) {
      hh[q++ * hs] = tau[k];
#pragma unroll
      for (int i = k + 2; i < n; ++i) hh[q++ * hs] = a[LI(i, k)];
    }
  }

  // LDL^T of T + sigma I
  double tn = 0.0;
#pragma unroll
  for (int i = 0; i < n; ++i) tn = fmax(tn, fabs(d[i]) + (i > 0 ? fabs(e[i - 1]) : 0.0) + (i < n - 1 ? fabs(e[i]) : 0.0));
  const double sigma = 1e-9 * tn + 1e-300;
  double ipiv[n], lo[n - 1];
  {
    double piv = d[0] + sigma;
#pragma unroll
    for (int i = 0; i < n - 1; ++i) {
      ipiv[i] = 1.0 / piv;
      lo[i] = e[i] * ipiv[i];
      piv = d[i + 1] + sigma - lo[i] * e[i];
    }
    ipiv[n - 1] = 1.0 / piv;
  }

  double x[4][n];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < n; ++i) x[j][i] = 1.0 + 0.37 * (double)(((i + 3) * (j + 5) * 7) % 11) - 0.13 * j;

  auto orthonormalize = [&](double (&y)[4][n]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {   // MGS, twice for stability
#pragma unroll
        for (int q = 0; q < j; ++q) {
          double dp = 0.0;
#pragma unroll
          for (int i = 0; i < n; ++i) dp += y[q][i] * y[j][i];
#pragma unroll
          for (int i = 0; i < n; ++i) y[j][i] -= dp * y[q][i];
        }
      }
      double nn = 0.0;
#pragma unroll
      for (int i = 0; i < n; ++i) nn += y[j][i] * y[j][i];
      const double inv = 1.0 / sqrt(nn);
#pragma unroll
      for (int i = 0; i < n; ++i) y[j][i] *= inv;
    }
  };
  orthonormalize(x);
  // fixed iteration count: the subspace error shrinks like ((l4+s)/(l5+s))^ITERS
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // x <- (T + sigma I)^-1 x, in place
      double z = x[j][0];
#pragma unroll
      for (int i = 1; i < n; ++i) {
        z = x[j][i] - lo[i - 1] * z;
        x[j][i] = z;
      }
#pragma unroll
      for (int i = 0; i < n; ++i) x[j][i] *= ipiv[i];
#pragma unroll
      for (int i = n - 2; i >= 0; --i) x[j][i] -= lo[i] * x[j][i + 1];
    }
    orthonormalize(x);
  }
  // Rayleigh-Ritz: H = X T X^T
  double h[16], hv[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      double dp = 0.0;
#pragma unroll
      for (int i = 0; i < n; ++i) {
        const double txq = d[i] * x[q][i] + (i > 0 ? e[i - 1] * x[q][i - 1] : 0.0) +
                           (i < n - 1 ? e[i] * x[q][i + 1] : 0.0);
        dp += x[p][i] * txq;
      }
      h[p * 4 + q] = dp;
    }
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int q = p + 1; q < 4; ++q) h[p * 4 + q] = h[q * 4 + p] = 0.5 * (h[p * 4 + q] + h[q * 4 + p]);
  for (int sweep = 0; sweep < 30; ++sweep) {
    double off = 0.0, dg = 0.0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      dg += h[p * 5] * h[p * 5];
#pragma unroll
      for (int q = p + 1; q < 4; ++q) off += h[p * 4 + q] * h[p * 4 + q];
    }
    if (off <= 1e-32 * dg || off == 0.0) break;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int q = p + 1; q < 4; ++q) {
        const double apq = h[p * 4 + q];
        if (apq != 0.0) {
          const double theta = (h[q * 5] - h[p * 5]) / (2.0 * apq);
          const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
          const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const double akp = h[k * 4 + p], akq = h[k * 4 + q];
            h[k * 4 + p] = c * akp - s * akq;
            h[k * 4 + q] = s * akp + c * akq;
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const double apk = h[p * 4 + k], aqk = h[q * 4 + k];
            h[p * 4 + k] = c * apk - s * aqk;
            h[q * 4 + k] = s * apk + c * aqk;
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const double vkp = hv[k * 4 + p], vkq = hv[k * 4 + q];
            hv[k * 4 + p] = c * vkp - s * vkq;
            hv[k * 4 + q] = s * vkp + c * vkq;
          }
        }
      }
  }
  // ascending order of the Ritz values (static sorting network on 4 slots)
  double ev[4] = {h[0], h[5], h[10], h[15]};
  int ord[4] = {0, 1, 2, 3};
  auto cs = [&](int i, int j) {
    if (ev[j] < ev[i]) {
      double t = ev[i]; ev[i] = ev[j]; ev[j] = t;
      int u = ord[i]; ord[i] = ord[j]; ord[j] = u;
    }
  };
  cs(0, 1); cs(2, 3); cs(0, 2); cs(1, 3); cs(1, 2);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    double c4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {   // column ord[r] of hv, selected statically
      c4[q] = hv[q * 4 + 0];
      c4[q] = (ord[r] == 1) ? hv[q * 4 + 1] : c4[q];
      c4[q] = (ord[r] == 2) ? hv[q * 4 + 2] : c4[q];
      c4[q] = (ord[r] == 3) ? hv[q * 4 + 3] : c4[q];
    }
    double y[n];
#pragma unroll
    for (int i = 0; i < n; ++i) y[i] = c4[0] * x[0][i] + c4[1] * x[1][i] + c4[2] * x[2][i] + c4[3] * x[3][i];
    // back-transform: y <- H_0 H_1 ... H_{n-3} y
#pragma unroll
    for (int k = n - 3; k >= 0; --k) {
      const int q0 = k * (2 * n - k - 1) / 2;   // start of reflector k in hh
      const double tk = hh[q0 * hs];
      if (tk != 0.0) {
        double s = y[k + 1];
#pragma unroll
        for (int i = k + 2; i < n; ++i) s += hh[(q0 + i - k - 1) * hs] * y[i];
        s *= tk;
        y[k + 1] -= s;
#pragma unroll
        for (int i = k + 2; i < n; ++i) y[i] -= s * hh[(q0 + i - k - 1) * hs];
      }
    }
#pragma unroll
    for (int i = 0; i < n; ++i) vec[r][i] = y[i];
  }
}

// least squares by Householder QR, m x n, m <= 6, full column rank
template <int M, int N>
__device__ __forceinline__ void lstsq(const double* A_, const double* b_, double* x) {
  double A[M * N], b[M];
#pragma unroll
  for (int i = 0; i < M * N; ++i) A[i] = A_[i];
#pragma unroll
  for (int i = 0; i < M; ++i) b[i] = b_[i];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    double norm = 0.0;
#pragma unroll
    for (int i = k; i < M; ++i) norm += A[i * N + k] * A[i * N + k];
    norm = sqrt(norm);
    if (norm == 0.0) continue;
    const double alpha = A[k * N + k] > 0 ? -norm : norm;
    double v[M];
#pragma unroll
    for (int i = 0; i < M; ++i) v[i] = (i >= k) ? A[i * N + k] : 0.0;
    v[k] -= alpha;
    double vv = 0.0;
#pragma unroll
    for (int i = k; i < M; ++i) vv += v[i] * v[i];
    if (vv == 0.0) continue;
#pragma unroll
    for (int j = k; j < N; ++j) {
      double s = 0.0;
#pragma unroll
      for (int i = k; i < M; ++i) s += v[i] * A[i * N + j];
      s = 2.0 * s / vv;
#pragma unroll
      for (int i = k; i < M; ++i) A[i * N + j] -= s * v[i];
    }
    double s = 0.0;
#pragma unroll
    for (int i = k; i < M; ++i) s += v[i] * b[i];
    s = 2.0 * s / vv;
#pragma unroll
    for (int i = k; i < M; ++i) b[i] -= s * v[i];
  }
#pragma unroll
  for (int i = N - 1; i >= 0; --i) {
    double s = b[i];
#pragma unroll
    for (int j = i + 1; j < N; ++j) s -= A[i * N + j] * x[j];
    x[i] = (A[i * N + i] != 0.0) ? s / A[i * N + i] : 0.0;
  }
}

__device__ __forceinline__ void inv3(const double* m, double* r) {
  const double c00 = m[4] * m[8] - m[5] * m[7];
  const double c01 = m[5] * m[6] - m[3] * m[8];
  const double c02 = m[3] * m[7] - m[4] * m[6];
  const double id = 1.0 / (m[0] * c00 + m[1] * c01 + m[2] * c02);
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

// orthogonal polar factor of a 3x3 matrix (U V^T of its SVD)
__device__ __forceinline__ void polar3(const double* A, double* R) {
  double ata[9], w[3], vt[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      ata[i * 3 + j] = A[i] * A[j] + A[3 + i] * A[3 + j] + A[6 + i] * A[6 + j];
  jacobi3(ata, w, vt);
  double u[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double sig = sqrt(w[i] > 0 ? w[i] : 0.0);
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const double s = A[r * 3] * vt[i * 3] + A[r * 3 + 1] * vt[i * 3 + 1] + A[r * 3 + 2] * vt[i * 3 + 2];
      u[i][r] = sig > 1e-300 ? s / sig : 0.0;
    }
  }
  if (!(w[2] > 1e-24 * w[0])) {
    u[2][0] = u[0][1] * u[1][2] - u[0][2] * u[1][1];
    u[2][1] = u[0][2] * u[1][0] - u[0][0] * u[1][2];
    u[2][2] = u[0][0] * u[1][1] - u[0][1] * u[1][0];
    const double vc0 = vt[1] * vt[5] - vt[2] * vt[4], vc1 = vt[2] * vt[3] - vt[0] * vt[5],
                 vc2 = vt[0] * vt[4] - vt[1] * vt[3];
    const double sgn = (vc0 * vt[6] + vc1 * vt[7] + vc2 * vt[8]) >= 0 ? 1.0 : -1.0;
#pragma unroll
    for (int r = 0; r < 3; ++r) u[2][r] *= sgn;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) R[i * 3 + j] = u[0][i] * vt[j] + u[1][i] * vt[3 + j] + u[2][i] * vt[6 + j];
}

__device__ __forceinline__ double dot3(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

// ---------------------------------------------------------------------------------------
// EPnP pieces that do not depend on the point count (epnp.cpp)
// ---------------------------------------------------------------------------------------
// vs: the four eigenvectors, vs + 12*i = i-th smallest (epnp.cpp's ut + 12*(11-i))
__device__ __forceinline__ void compute_L_6x10(const double* vs, double* l) {
  const double* v[4] = {vs, vs + 12, vs + 24, vs + 36};
  double dv[4][6][3];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int a = 0, b = 1;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
#pragma unroll
      for (int k = 0; k < 3; ++k) dv[i][j][k] = v[i][3 * a + k] - v[i][3 * b + k];
      b++;
      if (b > 3) {
        a++;
        b = a + 1;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double* row = l + 10 * i;
    row[0] = dot3(dv[0][i], dv[0][i]);
    row[1] = 2.0 * dot3(dv[0][i], dv[1][i]);
    row[2] = dot3(dv[1][i], dv[1][i]);
    row[3] = 2.0 * dot3(dv[0][i], dv[2][i]);
    row[4] = 2.0 * dot3(dv[1][i], dv[2][i]);
    row[5] = dot3(dv[2][i], dv[2][i]);
    row[6] = 2.0 * dot3(dv[0][i], dv[3][i]);
    row[7] = 2.0 * dot3(dv[1][i], dv[3][i]);
    row[8] = 2.0 * dot3(dv[2][i], dv[3][i]);
    row[9] = dot3(dv[3][i], dv[3][i]);
  }
}

__device__ __forceinline__ void compute_rho(const double (*cws)[3], double* rho) {
  auto d2 = [](const double* a, const double* b) {
    return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
  };
  rho[0] = d2(cws[0], cws[1]);
  rho[1] = d2(cws[0], cws[2]);
  rho[2] = d2(cws[0], cws[3]);
  rho[3] = d2(cws[1], cws[2]);
  rho[4] = d2(cws[1], cws[3]);
  rho[5] = d2(cws[2], cws[3]);
}

__device__ __forceinline__ void betas_approx(int which, const double* L, const double* rho, double* betas) {
  if (which == 1) {
    double l[24], b4[4];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      l[i * 4 + 0] = L[i * 10 + 0];
      l[i * 4 + 1] = L[i * 10 + 1];
      l[i * 4 + 2] = L[i * 10 + 3];
      l[i * 4 + 3] = L[i * 10 + 6];
    }
    lstsq<6, 4>(l, rho, b4);
    const double sg = b4[0] < 0 ? -1.0 : 1.0;
    betas[0] = sqrt(sg * b4[0]);
    betas[1] = sg * b4[1] / betas[0];
    betas[2] = sg * b4[2] / betas[0];
    betas[3] = sg * b4[3] / betas[0];
  } else if (which == 2) {
    double l[18], b3[3];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int k = 0; k < 3; ++k) l[i * 3 + k] = L[i * 10 + k];
    lstsq<6, 3>(l, rho, b3);
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
  } else {
    double l[30], b5[5];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int k = 0; k < 5; ++k) l[i * 5 + k] = L[i * 10 + k];
    lstsq<6, 5>(l, rho, b5);
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
}

// epnp::qr_solve for the 6x4 Gauss-Newton system
__device__ __forceinline__ void qr_solve_6x4(double* A, double* b, double* X) {
  constexpr int nr = 6, nc = 4;
  double A1[nc], A2[nc];
#pragma unroll
  for (int k = 0; k < nc; k++) {
    double eta = fabs(A[k * nc + k]);
#pragma unroll
    // epnp.cpp reads the pivot column before advancing, so rows k..nr-2 are scanned
    for (int i = k + 1; i < nr; i++) eta = fmax(eta, fabs(A[(i - 1) * nc + k]));
    if (eta == 0) return;   // X keeps its previous value, as in epnp.cpp
    double sum2 = 0.0;
    const double inv_eta = 1. / eta;
#pragma unroll
    for (int i = k; i < nr; i++) {
      A[i * nc + k] *= inv_eta;
      sum2 += A[i * nc + k] * A[i * nc + k];
    }
    double sigma = sqrt(sum2);
    if (A[k * nc + k] < 0) sigma = -sigma;
    A[k * nc + k] += sigma;
    A1[k] = sigma * A[k * nc + k];
    A2[k] = -eta * sigma;
#pragma unroll
    for (int j = k + 1; j < nc; j++) {
      double sum = 0;
#pragma unroll
      for (int i = k; i < nr; i++) sum += A[i * nc + k] * A[i * nc + j];
      const double tau = sum / A1[k];
#pragma unroll
      for (int i = k; i < nr; i++) A[i * nc + j] -= tau * A[i * nc + k];
    }
  }
#pragma unroll
  for (int j = 0; j < nc; j++) {
    double tau = 0;
#pragma unroll
    for (int i = j; i < nr; i++) tau += A[i * nc + j] * b[i];
    tau /= A1[j];
#pragma unroll
    for (int i = j; i < nr; i++) b[i] -= tau * A[i * nc + j];
  }
  X[nc - 1] = b[nc - 1] / A2[nc - 1];
#pragma unroll
  for (int i = nc - 2; i >= 0; i--) {
    double sum = 0;
#pragma unroll
    for (int j = i + 1; j < nc; j++) sum += A[i * nc + j] * X[j];
    X[i] = (b[i] - sum) / A2[i];
  }
}

__device__ __forceinline__ void gauss_newton(const double* L, const double* rho, double* betas) {
  double x[4] = {0.0, 0.0, 0.0, 0.0};
  for (int it = 0; it < 5; ++it) {
    double A[24], b[6];
#pragma unroll
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
#pragma unroll
    for (int i = 0; i < 4; ++i) betas[i] += x[i];
  }
}

__device__ __forceinline__ void ccs_from_betas(const double* vs, const double* betas, double (*ccs)[3]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) ccs[j][0] = ccs[j][1] = ccs[j][2] = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const double* v = vs + 12 * i;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < 3; ++k) ccs[j][k] += betas[i] * v[3 * j + k];
  }
}

__device__ __forceinline__ void finish_R(const double* abt, double* R) {
  polar3(abt, R);
  const double det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] -
                     R[2] * R[4] * R[6] - R[1] * R[3] * R[8] - R[0] * R[5] * R[7];
  if (det < 0) {
    R[6] = -R[6];
    R[7] = -R[7];
    R[8] = -R[8];
  }
}

__device__ __forceinline__ void rodrigues_m2v(const double* R, double* r) {
  double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
  const double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
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
    const double vth = theta * (1 / (2 * s));
    rx *= vth;
    ry *= vth;
    rz *= vth;
  }
  r[0] = rx;
  r[1] = ry;
  r[2] = rz;
}

__device__ __forceinline__ void rodrigues_v2m(const double* r, double* R) {
  const double theta = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
  if (theta < 2.220446049250313e-16) {
#pragma unroll
    for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
    return;
  }
  const double c = cos(theta), s = sin(theta), c1 = 1. - c;
  const double it = 1. / theta;
  const double x = r[0] * it, y = r[1] * it, z = r[2] * it;
  const double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
  const double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
#pragma unroll
  for (int i = 0; i < 9; ++i) R[i] = c * ((i % 4 == 0) ? 1.0 : 0.0) + c1 * rrt[i] + s * rx[i];
}

// ---------------------------------------------------------------------------------------
// 5-point EPnP (RANSAC kernel): epnp::compute_pose with n = 5, one hypothesis per lane, in
// two stages so that the workgroup's waves share the work:
//   epnp5_eig     (wave 0, lane h)      control points, M^T M, its four smallest eigenvectors,
//                                       handed over in LDS (HypState, lane h's column);
//   epnp5_approx  (wave w = 1..3)       approximation `w` (betas, Gauss-Newton, R, t, mean
//                                       reprojection error) for every hypothesis -- the three
//                                       run concurrently instead of one after another;
// then the smallest error picks the model, as compute_pose's sequential comparison does.
// Each piece is the arithmetic of the one-lane version, so the models are the same.  The
// points are read from the workgroup's LDS copy through `sub` whenever needed (volatile
// reads), so they do not occupy registers across the eigen-solve.
// ---------------------------------------------------------------------------------------
// Per-hypothesis state between the stages, SoA rows of kRound doubles (element h = lane h):
// it overlays eig12_small4's per-lane Householder scratch (Shared::hh), dead by then.
constexpr int kHsVs = 0, kHsRho = 48, kHsCw0 = 54, kHsCi = 57, kHsRows = 66;

__device__ __forceinline__ void epnp5_eig(const volatile int* sub, const volatile float* p2,
                                          const volatile float* p3, const double* K4, double* hh,
                                          int hs) {
  constexpr int n = kModelPoints;
  const double fu = K4[0], fv = K4[1], uc = K4[2], vc = K4[3];
  auto PW = [&](int i, int j) { return (double)p3[3 * sub[i] + j]; };
  auto US = [&](int i, int j) { return (double)p2[2 * sub[i] + j]; };
  double cw0[3], ci[9], rho[6];
  double mtm[78];
  {
    double cws[4][3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
#pragma unroll
      for (int i = 0; i < n; ++i) s += PW(i, j);
      cws[0][j] = s / n;
    }
    double m[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, dc[3], uct[9];
#pragma unroll
    for (int i = 0; i < n; ++i) {
      double p[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) p[j] = PW(i, j) - cws[0][j];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) m[r * 3 + c] += p[r] * p[c];
    }
    jacobi3(m, dc, uct);
#pragma unroll
    for (int i = 1; i < 4; ++i) {
      const double k = sqrt(dc[i - 1] / n);
#pragma unroll
      for (int j = 0; j < 3; ++j) cws[i][j] = cws[0][j] + k * uct[3 * (i - 1) + j];
    }
    double cc[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 1; j < 4; ++j) cc[3 * i + j - 1] = cws[j][i] - cws[0][i];
    inv3(cc, ci);
#pragma unroll
    for (int j = 0; j < 3; ++j) cw0[j] = cws[0][j];
    compute_rho(cws, rho);
#pragma unroll
    for (int i = 0; i < 78; ++i) mtm[i] = 0.0;
#pragma unroll
    for (int i = 0; i < n; ++i) {
      double as[4];
#pragma unroll
      for (int j = 0; j < 3; ++j)
        as[1 + j] = ci[3 * j] * (PW(i, 0) - cw0[0]) + ci[3 * j + 1] * (PW(i, 1) - cw0[1]) +
                    ci[3 * j + 2] * (PW(i, 2) - cw0[2]);
      as[0] = 1.0 - as[1] - as[2] - as[3];
      const double u = US(i, 0), v = US(i, 1);
      double r1[12], r2[12];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        r1[3 * k] = as[k] * fu;
        r1[3 * k + 1] = 0.0;
        r1[3 * k + 2] = as[k] * (uc - u);
        r2[3 * k] = 0.0;
        r2[3 * k + 1] = as[k] * fv;
        r2[3 * k + 2] = as[k] * (vc - v);
      }
#pragma unroll
      for (int a = 0; a < 12; ++a)
#pragma unroll
        for (int b = 0; b <= a; ++b) mtm[LI(a, b)] += r1[a] * r1[b] + r2[a] * r2[b];
    }
  }
  double ev4[4][12];
  eig12_small4<28>(mtm, ev4, hh, hs);
  // hand over (the Householder scratch is dead: eig12_small4 has back-transformed)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 12; ++k) hh[(kHsVs + 12 * i + k) * hs] = ev4[i][k];
#pragma unroll
  for (int i = 0; i < 6; ++i) hh[(kHsRho + i) * hs] = rho[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) hh[(kHsCw0 + i) * hs] = cw0[i];
#pragma unroll
  for (int i = 0; i < 9; ++i) hh[(kHsCi + i) * hs] = ci[i];
}

// Approximation `which` (1..3) of compute_pose for the hypothesis whose state is at hh
// (stride hs): R, t and the mean reprojection error over its five points.
__device__ __forceinline__ void epnp5_approx(int which, const volatile int* sub,
                                             const volatile float* p2, const volatile float* p3,
                                             const double* K4, const double* hh, int hs,
                                             double* R, double* t, double* err_out) {
  constexpr int n = kModelPoints;
  const double fu = K4[0], fv = K4[1], uc = K4[2], vc = K4[3];
  auto PW = [&](int i, int j) { return (double)p3[3 * sub[i] + j]; };
  auto US = [&](int i, int j) { return (double)p2[2 * sub[i] + j]; };
  double ut[48], rho[6], cw0[3], ci[9];
#pragma unroll
  for (int i = 0; i < 48; ++i) ut[i] = hh[(kHsVs + i) * hs];
#pragma unroll
  for (int i = 0; i < 6; ++i) rho[i] = hh[(kHsRho + i) * hs];
#pragma unroll
  for (int i = 0; i < 3; ++i) cw0[i] = hh[(kHsCw0 + i) * hs];
#pragma unroll
  for (int i = 0; i < 9; ++i) ci[i] = hh[(kHsCi + i) * hs];
  double L[60];
  compute_L_6x10(ut, L);
  double betas[4], ccs[4][3], pcs[n * 3];
  betas_approx(which, L, rho, betas);
  gauss_newton(L, rho, betas);
  ccs_from_betas(ut, betas, ccs);
#pragma unroll
  for (int i = 0; i < n; ++i) {
    double a[4];
#pragma unroll
    for (int j = 0; j < 3; ++j)
      a[1 + j] = ci[3 * j] * (PW(i, 0) - cw0[0]) + ci[3 * j + 1] * (PW(i, 1) - cw0[1]) +
                 ci[3 * j + 2] * (PW(i, 2) - cw0[2]);
    a[0] = 1.0 - a[1] - a[2] - a[3];
#pragma unroll
    for (int j = 0; j < 3; ++j)
      pcs[3 * i + j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
  }
  if (pcs[2] < 0.0) {
#pragma unroll
    for (int i = 0; i < 3 * n; ++i) pcs[i] = -pcs[i];
  }
  double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
#pragma unroll
  for (int i = 0; i < n; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      pc0[j] += pcs[3 * i + j];
      pw0[j] += PW(i, j);
    }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    pc0[j] /= n;
    pw0[j] /= n;
  }
  double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < n; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int k = 0; k < 3; ++k) abt[3 * j + k] += (pcs[3 * i + j] - pc0[j]) * (PW(i, k) - pw0[k]);
  finish_R(abt, R);
#pragma unroll
  for (int j = 0; j < 3; ++j) t[j] = pc0[j] - dot3(R + 3 * j, pw0);
  double err = 0.0;
#pragma unroll
  for (int i = 0; i < n; ++i) {
    const double pw[3] = {PW(i, 0), PW(i, 1), PW(i, 2)};
    const double Xc = dot3(R, pw) + t[0], Yc = dot3(R + 3, pw) + t[1];
    const double iz = 1.0 / (dot3(R + 6, pw) + t[2]);
    const double ue = uc + fu * Xc * iz, ve = vc + fv * Yc * iz;
    const double du = US(i, 0) - ue, dv = US(i, 1) - ve;
    err += sqrt(du * du + dv * dv);
  }
  *err_out = err / n;
}

// RANSACUpdateNumIters (ptsetreg.cpp)
__device__ __forceinline__ int update_num_iters(double p, double ep, int model_points, int max_iters) {
  p = fmin(fmax(p, 0.0), 1.0);
  ep = fmin(fmax(ep, 0.0), 1.0);
  double num = fmax(1. - p, 2.2250738585072014e-308);
  double denom = 1. - pow(1. - ep, (double)model_points);
  if (denom < 2.2250738585072014e-308) return 0;
  num = log(num);
  denom = log(denom);
  return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : __double2int_rn(num / denom);
}

// squared float reprojection error of one point (computeError; no fp contraction)
__device__ __forceinline__ float reproj_err2(const double* R, const double* t, const double* K4,
                                             float X, float Y, float Z, float u, float v) {
#pragma clang fp contract(off)
  const double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
  const double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
  double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
  z = z != 0.0 ? 1. / z : 1.0;
  const float pu = (float)(x * z * K4[0] + K4[2]);
  const float pv = (float)(y * z * K4[1] + K4[3]);
  const float du = u - pu, dv = v - pv;
  return du * du + dv * dv;
}

// ---------------------------------------------------------------------------------------
// workgroup reductions (double)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// sum `cnt` per-thread values across the workgroup; every thread gets the totals
template <int CNT>
__device__ __forceinline__ void block_sum(double* vals, double* scratch /* [4][CNT] */) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < CNT; ++i) {
    const double s = wave_sum_d(vals[i]);
    if (lane == 0) scratch[wave * CNT + i] = s;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < CNT; ++i)
    vals[i] = scratch[i] + scratch[CNT + i] + scratch[2 * CNT + i] + scratch[3 * CNT + i];
  __syncthreads();
}

struct Shared {
  double hh[kHsRows * kRound];   // per-lane Householder scratch of eig12_small4 (65 rows),
                                 // then the hypotheses' HypState rows (epnp5_eig -> epnp5_approx)
  double herr[4][kRound];         // mean reprojection error of approximation w (1..3)
  // RANSAC round
  int subset[kRound][kModelPoints];
  double hypR[kRound][9];
  double hypT[kRound][3];
  double hypRvec[kRound][3];
  int count[kRound];
  // RNG positions of a round, generated in parallel: state after each draw, draw % n
  unsigned long long rst[kRngPos];
  int rii[kRngPos];
  short rend[kRngPos], rstart[kRound];
  unsigned long long rz;
  int rk, rP, rdealt, rpos;
  // control
  int iter, niters, max_good, done, p3p;
  double bestRvec[3], bestT[3];
  unsigned long long rng;
  // refit
  double red[4 * 78];
  double cws[4][3];
  double ci[9];
  double vs[48];
  double L[60], rho[6];
  double betas[4];
  double ccs[4][3];
  double sol_R[4][9], sol_t[4][3], sol_err[4];
  double flip;
  double wccs[3][4][3], wflip[3];   // per approximation wave (refit, n >= 6)
  double S40[40];                    // M^T M's distinct sums (refit, n >= 6)
  int ord[4];
  int wave_cnt[4];
  int n_inl;
  // refit eigensolver (jacobi12_wave)
  double jA[144], jV[144];
};

// Eigenvectors of the four smallest eigenvalues of the symmetric 12x12 M^T M (in sh.jA),
// ascending -> sh.vs (48 doubles), for the EPnP refit.  Cyclic Jacobi in parallel rounds:
// the circle method pairs the 12 indices into 6 disjoint (p, q) per round, 11 rounds per
// sweep.  One wave runs it (the caller's wave 0), lane I * 6 + J (I, J < 6) owning the 2 x 2
// block of rows (p_I, q_I) and columns (p_J, q_J) of A and of V in the round: it computes
// the rotations of pairs I and J from the round's diagonal entries (every lane the same
// formulas, so the same values), then A's block as J^T (A J) -- the column pass, then the
// row pass, the arithmetic of the round-4 workgroup version -- and V's block as V J.  A and V
// stay in LDS in full 12 x 12 layout; within one wave a round needs no workgroup barrier (its
// reads precede its writes in the wave's LDS order), which is what the workgroup version
// paid three of per round.  EPnP's result does not depend on the eigenvectors' signs, and
// any accurate eigensolver gives the oracle's vectors up to sign when the eigenvalues are
// separated.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void jacobi_rot(double app, double aqq, double apq, double& c, double& sn) {
  c = 1.0;
  sn = 0.0;
  if (apq != 0.0) {   // t = sgn(theta) / (|theta| + sqrt(theta^2 + 1)), theta = a / b, without
                       // the division for theta: t = sgn(a) b / (|a| + sqrt(a^2 + b^2))
    const double a = aqq - app, b = 2.0 * apq;
    const double tt = (a >= 0.0 ? b : -b) / (fabs(a) + sqrt(a * a + b * b));
    c = 1.0 / sqrt(tt * tt + 1.0);
    sn = tt * c;
  }
}
// pair k of round r (circle method), p < q
__device__ __forceinline__ void jacobi_pair(int r, int k, int& p, int& q) {
  const int a = r + k, c = r - k + 11;   // (r + k) % 11, (r - k + 11) % 11
  p = k == 0 ? r : (a >= 11 ? a - 11 : a);
  q = k == 0 ? 11 : (c >= 11 ? c - 11 : c);
  if (p > q) {
    const int x = p;
    p = q;
    q = x;
  }
}
__device__ void jacobi12_wave(Shared& sh) {
  const int lane = threadIdx.x & 63;
  for (int i = lane; i < 144; i += 64) sh.jV[i] = (i / 12 == i % 12) ? 1.0 : 0.0;
  double tr = 0.0;   // trace: the scale of "converged" off-diagonals (M^T M is PSD)
  for (int i = 0; i < 12; ++i) tr += fabs(sh.jA[i * 13]);
  const double thr = 1e-22 * tr;
  const int I = min(lane / 6, 5), J = lane % 6;   // lanes >= 36 shadow block (5, J): no writes
  const bool own = lane < 36;
  double* A = sh.jA;
  double* V = sh.jV;
  wave_lds_sync();
  for (int sweep = 0; sweep < 12; ++sweep) {
    bool big = false;
    for (int round = 0; round < 11; ++round) {
      int pI, qI, pJ, qJ;
      jacobi_pair(round, I, pI, qI);
      jacobi_pair(round, J, pJ, qJ);
      // pair J's rotation; pair I's is lane I's pair J (lane I = block (0, I))
      const double apqJ = A[pJ * 12 + qJ];
      double cJ, sJ;
      jacobi_rot(A[pJ * 13], A[qJ * 13], apqJ, cJ, sJ);
      const double cI = __shfl(cJ, I, 64), sI = __shfl(sJ, I, 64);
      big |= fabs(apqJ) > thr;   // (every pair is some lane's J)
      const double app = A[pI * 12 + pJ], apq = A[pI * 12 + qJ];
      const double aqp = A[qI * 12 + pJ], aqq = A[qI * 12 + qJ];
      const double vpp = V[pI * 12 + pJ], vpq = V[pI * 12 + qJ];
      const double vqp = V[qI * 12 + pJ], vqq = V[qI * 12 + qJ];
      wave_lds_sync();   // every read of the round before any write
      // A J (columns pJ, qJ), then J^T (A J) (rows pI, qI)
      const double xpp = cJ * app - sJ * apq, xpq = sJ * app + cJ * apq;
      const double xqp = cJ * aqp - sJ * aqq, xqq = sJ * aqp + cJ * aqq;
      if (own) {
        A[pI * 12 + pJ] = cI * xpp - sI * xqp;
        A[qI * 12 + pJ] = sI * xpp + cI * xqp;
        A[pI * 12 + qJ] = cI * xpq - sI * xqq;
        A[qI * 12 + qJ] = sI * xpq + cI * xqq;
        V[pI * 12 + pJ] = cJ * vpp - sJ * vpq;
        V[pI * 12 + qJ] = sJ * vpp + cJ * vpq;
        V[qI * 12 + pJ] = cJ * vqp - sJ * vqq;
        V[qI * 12 + qJ] = sJ * vqp + cJ * vqq;
      }
      wave_lds_sync();
    }
    if (__ballot(big) == 0ull) break;   // a sweep without a rotation: converged
  }
  if (lane == 0) {   // the four smallest eigenvalues, ascending (ties by index)
    int order[12];
    for (int i = 0; i < 12; ++i) order[i] = i;
    for (int i = 0; i < 4; ++i)
      for (int j = i + 1; j < 12; ++j)
        if (A[order[j] * 13] < A[order[i] * 13]) {
          const int x = order[i];
          order[i] = order[j];
          order[j] = x;
        }
    for (int i = 0; i < 4; ++i) sh.ord[i] = order[i];
  }
  wave_lds_sync();
  if (lane < 48) sh.vs[lane] = V[(lane % 12) * 12 + sh.ord[lane / 12]];
}

// Canonical basis of the 4-dimensional EPnP null space of exactly 4 correspondences (M is
// 8 x 12): P = I - M^T (M M^T)^-1 M, Gram-Schmidt of P's columns in index order.  Same
// arithmetic as null4_basis in oracle/epnp_ransac.c (see there for why).
__device__ void null4_basis(const double (&M)[8][12], double (&v)[4][12]) {
#pragma clang fp contract(off)
  double G[8][8], X[8][12];
  for (int a = 0; a < 8; ++a) {
    for (int b = 0; b < 8; ++b) {
      double acc = 0;
      for (int k = 0; k < 12; ++k) acc += M[a][k] * M[b][k];
      G[a][b] = acc;
    }
    for (int k = 0; k < 12; ++k) X[a][k] = M[a][k];
  }
  for (int c = 0; c < 8; ++c) {
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

// Workgroup-parallel EPnP over the points p2 / p3 [0, n) (epnp::compute_pose): the kernel's LDS
// copy of the inliers, in inlier order.

__device__ __forceinline__ void epnp_refit(Shared& sh, const float* p2, const float* p3, int n,
                           const double* K4, double* R_out, double* t_out) {
  const int t = threadIdx.x;
  const double fu = K4[0], fv = K4[1], uc = K4[2], vc = K4[3];
  // centroid
  double v3[3] = {0, 0, 0};
  for (int i = t; i < n; i += kThreads) {
    const int j = i;
    v3[0] += (double)p3[3 * j];
    v3[1] += (double)p3[3 * j + 1];
    v3[2] += (double)p3[3 * j + 2];
  }
  block_sum<3>(v3, sh.red);
  const double c0[3] = {v3[0] / n, v3[1] / n, v3[2] / n};
  // PCA
  double m6[6] = {0, 0, 0, 0, 0, 0};
  for (int i = t; i < n; i += kThreads) {
    const int j = i;
    const double p0 = (double)p3[3 * j] - c0[0], p1 = (double)p3[3 * j + 1] - c0[1],
                 p2_ = (double)p3[3 * j + 2] - c0[2];
    m6[0] += p0 * p0;
    m6[1] += p0 * p1;
    m6[2] += p0 * p2_;
    m6[3] += p1 * p1;
    m6[4] += p1 * p2_;
    m6[5] += p2_ * p2_;
  }
  block_sum<6>(m6, sh.red);
  // @phase 9
  if (t == 0) {
    double m[9] = {m6[0], m6[1], m6[2], m6[1], m6[3], m6[4], m6[2], m6[4], m6[5]}, dc[3], uct[9];
    jacobi3(m, dc, uct);
    for (int j = 0; j < 3; ++j) sh.cws[0][j] = c0[j];
    for (int i = 1; i < 4; ++i) {
      const double k = sqrt(dc[i - 1] / n);
      for (int j = 0; j < 3; ++j) sh.cws[i][j] = c0[j] + k * uct[3 * (i - 1) + j];
    }
    double cc[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 1; j < 4; ++j) cc[3 * i + j - 1] = sh.cws[j][i] - sh.cws[0][i];
    inv3(cc, sh.ci);
  }
  __syncthreads();
  auto alphas = [&](int j, double* a) {
    const double d0 = (double)p3[3 * j] - sh.cws[0][0], d1 = (double)p3[3 * j + 1] - sh.cws[0][1],
                 d2 = (double)p3[3 * j + 2] - sh.cws[0][2];
#pragma unroll
    for (int k = 0; k < 3; ++k) a[1 + k] = sh.ci[3 * k] * d0 + sh.ci[3 * k + 1] * d1 + sh.ci[3 * k + 2] * d2;
    a[0] = 1.0 - a[1] - a[2] - a[3];
  };
  const int lane = t & 63, wave = t >> 6;
  if (n >= 6) {
    // M^T M from its 40 distinct sums: with r1 = [a_k fu, 0, a_k (uc - u)] and
    // r2 = [0, a_k fv, a_k (vc - v)], entry (3k+i, 3l+j) is G_ij summed with a_k a_l:
    //   (0,0) fu^2 S,  (1,1) fv^2 S,  (0,2) fu Su,  (1,2) fv Sv,  (2,2) Sw,  (0,1) 0,
    // S / Su / Sv / Sw = sum a_k a_l x {1, uc - u, vc - v, (uc - u)^2 + (vc - v)^2}, k <= l.
    // Wave 0 accumulates (lane = point stride), then a transposed reduction through LDS.
    if (wave == 0) {
      double S[40];
#pragma unroll
      for (int e = 0; e < 40; ++e) S[e] = 0.0;
      for (int i = lane; i < n; i += 64) {
        const int j = i;
        double as[4];
        alphas(j, as);
        const double du = uc - (double)p2[2 * j], dv = vc - (double)p2[2 * j + 1];
        const double dw = du * du + dv * dv;
        int q = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int l = k; l < 4; ++l, ++q) {
            const double aa = as[k] * as[l];
            S[4 * q] += aa;
            S[4 * q + 1] += aa * du;
            S[4 * q + 2] += aa * dv;
            S[4 * q + 3] += aa * dw;
          }
      }
      double* red = sh.hh;   // [40][64], free in this kernel
#pragma unroll
      for (int e = 0; e < 40; ++e) red[e * 64 + lane] = S[e];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (lane < 40) {
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        for (int l = 0; l < 64; l += 4) {
          a0 += red[lane * 64 + l];
          a1 += red[lane * 64 + l + 1];
          a2 += red[lane * 64 + l + 2];
          a3 += red[lane * 64 + l + 3];
        }
        sh.S40[lane] = (a0 + a1) + (a2 + a3);
      }
    }
    __syncthreads();
    for (int i = t; i < 144; i += kThreads) {
      const int r = i / 12, c = i - r * 12;
      const int k = r / 3, ii = r - 3 * k, l = c / 3, jj = c - 3 * l;
      const int lo = k < l ? k : l, hi = k < l ? l : k;
      const int q = lo * 4 - lo * (lo - 1) / 2 + (hi - lo);   // pair index of (lo, hi), k <= l
      const int a = ii < jj ? ii : jj, b = ii < jj ? jj : ii;
      const double* Sq = sh.S40 + 4 * q;
      double v = 0.0;
      if (a == 0 && b == 0) v = fu * fu * Sq[0];
      else if (a == 1 && b == 1) v = fv * fv * Sq[0];
      else if (a == 0 && b == 2) v = fu * Sq[1];
      else if (a == 1 && b == 2) v = fv * Sq[2];
      else if (a == 2 && b == 2) v = Sq[3];
      sh.jA[i] = v;
    }
    __syncthreads();
    // @phase 10
    if (wave == 0) jacobi12_wave(sh);   // -> sh.vs
    __syncthreads();
    // @phase 11
    if (t < 60) {   // compute_L_6x10, one entry per thread
      constexpr int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
      constexpr int cp[10] = {0, 0, 1, 0, 1, 2, 0, 1, 2, 3}, cq[10] = {0, 1, 1, 2, 2, 2, 3, 3, 3, 3};
      const int i = t / 10, c = t - 10 * i;
      const double* vp = sh.vs + 12 * cp[c];
      const double* vq = sh.vs + 12 * cq[c];
      double dp[3], dq[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        dp[k] = vp[3 * pa[i] + k] - vp[3 * pb[i] + k];
        dq[k] = vq[3 * pa[i] + k] - vq[3 * pb[i] + k];
      }
      const double d = dot3(dp, dq);
      sh.L[t] = cp[c] == cq[c] ? d : 2.0 * d;
    } else if (t == 64) {
      compute_rho(sh.cws, sh.rho);
    }
  } else {
    // n = 4 / 5: M^T M per thread, summed over the workgroup (the arithmetic the oracle's
    // test scenes pin for these rank-deficient cases), then thread 0's basis
    double acc[78];
#pragma unroll
    for (int i = 0; i < 78; ++i) acc[i] = 0.0;
    for (int i = t; i < n; i += kThreads) {
      const int j = i;
      double as[4];
      alphas(j, as);
      const double u = (double)p2[2 * j], v = (double)p2[2 * j + 1];
      double r1[12], r2[12];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        r1[3 * k] = as[k] * fu;
        r1[3 * k + 1] = 0.0;
        r1[3 * k + 2] = as[k] * (uc - u);
        r2[3 * k] = 0.0;
        r2[3 * k + 1] = as[k] * fv;
        r2[3 * k + 2] = as[k] * (vc - v);
      }
#pragma unroll
      for (int a = 0; a < 12; ++a)
#pragma unroll
        for (int b = 0; b <= a; ++b) acc[LI(a, b)] += r1[a] * r1[b] + r2[a] * r2[b];
    }
    block_sum<78>(acc, sh.red);
    if (t == 0) {
      double ev4[4][12];
      if (n == 4) {   // canonical null-space basis (null4_basis), no eigensolver
        double M[8][12];
        for (int i = 0; i < 4; ++i) {
          double as[4];
          alphas(i, as);
          const double u = (double)p2[2 * i], v = (double)p2[2 * i + 1];
          for (int k = 0; k < 4; ++k) {
            M[2 * i][3 * k] = as[k] * fu;
            M[2 * i][3 * k + 1] = 0.0;
            M[2 * i][3 * k + 2] = as[k] * (uc - u);
            M[2 * i + 1][3 * k] = 0.0;
            M[2 * i + 1][3 * k + 1] = as[k] * fv;
            M[2 * i + 1][3 * k + 2] = as[k] * (vc - v);
          }
        }
        null4_basis(M, ev4);
      } else {
        eig12_small4<100>(acc, ev4, sh.hh, 1);
      }
      for (int i = 0; i < 48; ++i) sh.vs[i] = (&ev4[0][0])[i];
      compute_L_6x10(sh.vs, sh.L);
      compute_rho(sh.cws, sh.rho);
    }
  }
  __syncthreads();
  // @phase 12
  // compute_pose's three approximations, one per wave (waves 0..2), each reducing over the
  // points with wave-level sums; wave 3 waits
  if (wave < 3) {
    const int which = wave + 1;
    double(*ccs)[3] = sh.wccs[wave];
    if (lane == 0) {
      double betas[4];
      betas_approx(which, sh.L, sh.rho, betas);
      gauss_newton(sh.L, sh.rho, betas);
      ccs_from_betas(sh.vs, betas, ccs);
      // solve_for_sign looks at the first point's camera-frame depth
      double a[4];
      alphas(0, a);
      const double z0 = a[0] * ccs[0][2] + a[1] * ccs[1][2] + a[2] * ccs[2][2] + a[3] * ccs[3][2];
      sh.wflip[wave] = z0 < 0.0 ? -1.0 : 1.0;
    }
    // @phase 16
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const double fl = sh.wflip[wave];
    auto pc_of = [&](int j, double* pc) {
      double a[4];
      alphas(j, a);
#pragma unroll
      for (int k = 0; k < 3; ++k)
        pc[k] = fl * (a[0] * ccs[0][k] + a[1] * ccs[1][k] + a[2] * ccs[2][k] + a[3] * ccs[3][k]);
    };
    double s6[6] = {0, 0, 0, 0, 0, 0};
    for (int i = lane; i < n; i += 64) {
      const int j = i;
      double pc[3];
      pc_of(j, pc);
      s6[0] += pc[0];
      s6[1] += pc[1];
      s6[2] += pc[2];
      s6[3] += (double)p3[3 * j];
      s6[4] += (double)p3[3 * j + 1];
      s6[5] += (double)p3[3 * j + 2];
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) s6[k] = wave_sum_d(s6[k]);
    const double pc0[3] = {s6[0] / n, s6[1] / n, s6[2] / n}, pw0[3] = {s6[3] / n, s6[4] / n, s6[5] / n};
    double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = lane; i < n; i += 64) {
      const int j = i;
      double pc[3];
      pc_of(j, pc);
      const double pw[3] = {(double)p3[3 * j] - pw0[0], (double)p3[3 * j + 1] - pw0[1],
                            (double)p3[3 * j + 2] - pw0[2]};
#pragma unroll
      for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) abt[3 * a + b] += (pc[a] - pc0[a]) * pw[b];
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) abt[k] = wave_sum_d(abt[k]);
    // @phase 17
    double R[9], tt[3];
    finish_R(abt, R);   // every lane (identical inputs): no hand-over needed
    // @phase 18
#pragma unroll
    for (int j = 0; j < 3; ++j) tt[j] = pc0[j] - dot3(R + 3 * j, pw0);
    double err = 0.0;
    for (int i = lane; i < n; i += 64) {
      const int j = i;
      const double pw[3] = {(double)p3[3 * j], (double)p3[3 * j + 1], (double)p3[3 * j + 2]};
      const double Xc = dot3(R, pw) + tt[0], Yc = dot3(R + 3, pw) + tt[1];
      const double iz = 1.0 / (dot3(R + 6, pw) + tt[2]);
      const double ue = uc + fu * Xc * iz, ve = vc + fv * Yc * iz;
      const double du = (double)p2[2 * j] - ue, dv = (double)p2[2 * j + 1] - ve;
      err += sqrt(du * du + dv * dv);
    }
    err = wave_sum_d(err);
    if (lane == 0) {
      for (int k = 0; k < 9; ++k) sh.sol_R[which][k] = R[k];
      for (int k = 0; k < 3; ++k) sh.sol_t[which][k] = tt[k];
      sh.sol_err[which] = err / n;
    }
  }
  __syncthreads();
  // @phase 13
  int N = 1;
  if (sh.sol_err[2] < sh.sol_err[1]) N = 2;
  if (sh.sol_err[3] < sh.sol_err[N]) N = 3;
  for (int i = 0; i < 9; ++i) R_out[i] = sh.sol_R[N][i];
  for (int i = 0; i < 3; ++i) t_out[i] = sh.sol_t[N][i];
}

// ---- P3P gate for exactly 4 points (solvePnPRansac: model_points = 4, P3P kernel; with
// count == model_points the kernel runs once on all points and, when it yields a model, all 4
// are inliers and the final refit is EPnP over them).  Same arithmetic as the oracle's
// oracle_p3p_solutions (oracle/epnp_ransac.c): Gao's law-of-cosines system, y eliminated
// linearly, the quartic's real roots by derivative bracketing + bisection.
__device__ double p3p_poly(const double* c, int deg, double x) {
#pragma clang fp contract(off)
  double v = c[deg];
  for (int i = deg - 1; i >= 0; --i) v = v * x + c[i];
  return v;
}

__device__ double p3p_bisect(const double* c, int deg, double lo, double hi) {
#pragma clang fp contract(off)
  double flo = p3p_poly(c, deg, lo);
  for (int it = 0; it < 200; ++it) {
    const double mid = 0.5 * (lo + hi);
    if (mid <= lo || mid >= hi) break;
    const double fm = p3p_poly(c, deg, mid);
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

// real roots (ascending) of c[0..deg]; iterative over degrees 1..deg (no recursion on device)
__device__ int p3p_real_roots(const double* c4, double* roots) {
#pragma clang fp contract(off)
  double cs[5][5];   // cs[d] = the (4-d)-th derivative of the quartic, degree d
  for (int i = 0; i <= 4; ++i) cs[4][i] = c4[i];
  for (int d = 3; d >= 1; --d)
    for (int i = 1; i <= d + 1; ++i) cs[d][i - 1] = i * cs[d + 1][i];
  double r[4];
  int nr = 1;
  r[0] = -cs[1][0] / cs[1][1];
  for (int deg = 2; deg <= 4; ++deg) {
    const double* c = cs[deg];
    double bound = 0.0;
    for (int i = 0; i < deg; ++i) {
      const double q = fabs(c[i] / c[deg]);
      bound = q > bound ? q : bound;
    }
    bound += 1.0;
    double pts[6];
    int np = 0;
    pts[np++] = -bound;
    for (int i = 0; i < nr; ++i)
      if (r[i] > -bound && r[i] < bound) pts[np++] = r[i];
    pts[np++] = bound;
    double out[4];
    int n = 0;
    for (int i = 0; i + 1 < np; ++i) {
      const double fa = p3p_poly(c, deg, pts[i]), fb = p3p_poly(c, deg, pts[i + 1]);
      if (fa == 0.0) {
        if (n == 0 || out[n - 1] != pts[i]) out[n++] = pts[i];
      } else if ((fa < 0) != (fb < 0) && fb != 0.0) {
        out[n++] = p3p_bisect(c, deg, pts[i], pts[i + 1]);
      }
    }
    if (p3p_poly(c, deg, pts[np - 1]) == 0.0) out[n++] = pts[np - 1];
    for (int i = 0; i < n; ++i) r[i] = out[i];
    nr = n;
  }
  for (int i = 0; i < nr; ++i) roots[i] = r[i];
  return nr;
}

__device__ int p3p_solutions(const float* p2, const float* p3, const double* K4) {
#pragma clang fp contract(off)
  const double fx = K4[0], fy = K4[1], cx = K4[2], cy = K4[3];
  double bear[3][3], P[3][3];
  for (int i = 0; i < 3; ++i) {
    const double mu = ((double)p2[2 * i] - cx) / fx, mv = ((double)p2[2 * i + 1] - cy) / fy;
    const double mk = 1.0 / sqrt(mu * mu + mv * mv + 1.0);
    bear[i][0] = mu * mk;
    bear[i][1] = mv * mk;
    bear[i][2] = mk;
    for (int k = 0; k < 3; ++k) P[i][k] = p3[3 * i + k];
  }
  auto d2f = [](const double* a, const double* b) {
    return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
  };
  auto dotf = [](const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
  const double d0 = sqrt(d2f(P[1], P[2])), d1 = sqrt(d2f(P[0], P[2])), d2 = sqrt(d2f(P[0], P[1]));
  const double p = 2.0 * dotf(bear[1], bear[2]), q = 2.0 * dotf(bear[0], bear[2]),
               r = 2.0 * dotf(bear[0], bear[1]);
  if (p * p + q * q + r * r - p * q * r - 1.0 == 0.0) return 0;
  if (d2 == 0.0) return 0;
  const double a = (d0 * d0) / (d2 * d2), b = (d1 * d1) / (d2 * d2);
  const double n2 = -(1.0 - a - b), n1 = (1.0 - a) * q, n0 = -(1.0 - a + b);
  const double e1 = r, e0 = -p;
  const double q2 = 1.0 - b, q1 = -q, q0 = 1.0;
  double c[5] = {0, 0, 0, 0, 0};
  c[4] -= n2 * n2;
  c[3] -= 2.0 * n2 * n1;
  c[2] -= n1 * n1 + 2.0 * n2 * n0;
  c[1] -= 2.0 * n1 * n0;
  c[0] -= n0 * n0;
  const double ne3 = n2 * e1, ne2 = n2 * e0 + n1 * e1, ne1 = n1 * e0 + n0 * e1, ne0 = n0 * e0;
  c[4] += b * r * ne3;
  c[3] += b * r * ne2;
  c[2] += b * r * ne1;
  c[1] += b * r * ne0;
  const double ee2 = e1 * e1, ee1 = 2.0 * e1 * e0, ee0 = e0 * e0;
  c[4] += b * q2 * ee2;
  c[3] += b * (q2 * ee1 + q1 * ee2);
  c[2] += b * (q2 * ee0 + q1 * ee1 + q0 * ee2);
  c[1] += b * (q1 * ee0 + q0 * ee1);
  c[0] += b * q0 * ee0;
  if (c[4] == 0.0) return 0;
  double xs[4];
  const int nr = p3p_real_roots(c, xs);
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
    ++sols;
  }
  return sols;
}

__device__ __forceinline__ unsigned rng_next(unsigned long long& s) {
  s = (unsigned long long)(unsigned)s * 4164903690ull + (unsigned)(s >> 32);
  return (unsigned)s;
}

// cv::RNG is a lag-1 multiply-with-carry generator: for a state z = c * 2^32 + x below
// m = A * 2^32 - 1, the next state A x + c equals A z mod m (A 2^32 = 1 mod m), so the state
// k draws ahead is A^k z mod m -- lane l of a wave starts its 6 draws at A^(6 l) z.
__device__ __forceinline__ unsigned long long mwc_mulmod(unsigned long long a,
                                                         unsigned long long b) {
  // a b mod m for a, b < m: fold the high word with 2^64 = r (mod m), r = (2^32 - A) 2^32 + 1
  constexpr unsigned long long r = ((4294967296ull - kMwcA) << 32) | 1ull;
  unsigned long long lo = a * b, hi = __umul64hi(a, b);
  while (hi != 0ull) {
    const unsigned long long l2 = hi * r, h2 = __umul64hi(hi, r);
    lo += l2;
    hi = h2 + (lo < l2 ? 1ull : 0ull);
  }
  return lo >= kMwcM ? lo - kMwcM : lo;
}

// Correspondence selection fused into the RANSAC kernel (onepose_pose_stage): the frame's
// valid matches compacted in ascending 2D-index order (select_kernel's rule) straight into
// the LDS point copy, and into pts2d / pts3d / counts for the refit and the caller.
struct SelArgs {
  const int64_t* matches0;   // null: the points are given (onepose_pnp_ransac)
  const float* kp2;
  int64_t kp2_bs;
  const float* kp3;
  int64_t kp3_bs;
  int n1, n3;
  double scale3d;
};

__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1)))
void pnp_ransac_kernel(
    const float* __restrict__ pts2d, const float* __restrict__ pts3d, const int* __restrict__ counts,
    int max_points, const double* __restrict__ Kmat, int64_t K_bs, double scale, float reproj,
    int max_iters, double confidence, double* __restrict__ pose34, uint8_t* __restrict__ mask_out,
    int* __restrict__ n_inliers, int* __restrict__ status, int* __restrict__ idx_ws, SelArgs sel,
    float* __restrict__ sel_p2, float* __restrict__ sel_p3, int* __restrict__ sel_counts) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
  Shared& sh = *reinterpret_cast<Shared*>(dyn);
  float* p2 = reinterpret_cast<float*>(dyn + ((sizeof(Shared) + 15) / 16) * 16);
  float* p3 = p2 + 2 * max_points;
  const int b = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  // @phase 0
  int n;
  if (sel.matches0 != nullptr) {   // select: compact the valid matches (block-wide scan)
    const int64_t* m = sel.matches0 + (int64_t)b * sel.n1;
    const float* k2 = sel.kp2 + b * sel.kp2_bs;
    const float* k3 = sel.kp3 + b * sel.kp3_bs;
    float* o2 = sel_p2 + (int64_t)b * max_points * 2;
    float* o3 = sel_p3 + (int64_t)b * max_points * 3;
    int base = 0;
    for (int start = 0; start < sel.n1; start += kThreads) {
      const int i = start + t;
      const int64_t j = (i < sel.n1) ? m[i] : -1;
      const bool valid = j > -1 && j < sel.n3;
      const unsigned long long bal = __ballot(valid);
      if (lane == 0) sh.wave_cnt[wave] = __popcll(bal);
      __syncthreads();
      int off = base;
      for (int w2 = 0; w2 < wave; ++w2) off += sh.wave_cnt[w2];
      if (valid) {
        const int q = off + __popcll(bal & ((1ull << lane) - 1ull));
        const float u = k2[(int64_t)i * 2], v = k2[(int64_t)i * 2 + 1];
        const float X = (float)((double)k3[j * 3] * sel.scale3d);
        const float Y = (float)((double)k3[j * 3 + 1] * sel.scale3d);
        const float Z = (float)((double)k3[j * 3 + 2] * sel.scale3d);
        p2[2 * q] = u;
        p2[2 * q + 1] = v;
        p3[3 * q] = X;
        p3[3 * q + 1] = Y;
        p3[3 * q + 2] = Z;
        o2[2 * q] = u;
        o2[2 * q + 1] = v;
        o3[3 * q] = X;
        o3[3 * q + 1] = Y;
        o3[3 * q + 2] = Z;
      }
      base += sh.wave_cnt[0] + sh.wave_cnt[1] + sh.wave_cnt[2] + sh.wave_cnt[3];
      __syncthreads();
    }
    n = base;
    if (t == 0) sel_counts[b] = n;
  } else {
    n = min(counts[b], max_points);
  }
  const double* K = Kmat + b * K_bs;
  const double K4[4] = {K[0], K[4], K[2], K[5]};
  uint8_t* mask = mask_out + (int64_t)b * max_points;
  int* idx = idx_ws + (int64_t)b * max_points;
  double* pose = pose34 + (int64_t)b * 12;

  for (int i = t; i < max_points; i += kThreads) mask[i] = 0;
  auto identity = [&](int st) {
    if (t < 12) pose[t] = (t % 5 == 0) ? 1.0 : 0.0;
    if (t == 0) {
      n_inliers[b] = 0;
      status[b] = st;
    }
  };
  if (n < 4) {
    identity(1);
    return;
  }
  if (sel.matches0 == nullptr) {
    for (int i = t; i < n; i += kThreads) {
      p2[2 * i] = pts2d[((int64_t)b * max_points + i) * 2];
      p2[2 * i + 1] = pts2d[((int64_t)b * max_points + i) * 2 + 1];
      p3[3 * i] = pts3d[((int64_t)b * max_points + i) * 3];
      p3[3 * i + 1] = pts3d[((int64_t)b * max_points + i) * 3 + 1];
      p3[3 * i + 2] = pts3d[((int64_t)b * max_points + i) * 3 + 2];
    }
  }
  const float thr = (float)((double)reproj * (double)reproj);
  // @phase 1
  if (t == 0) {
    sh.iter = 0;
    sh.niters = max(max_iters, 1);
    sh.max_good = 0;
    sh.done = (n == kModelPoints) ? 1 : 0;
    sh.rng = 0xFFFFFFFFFFFFFFFFull;
  }
  __syncthreads();
  if (n == 4) {   // solvePnPRansac's 4-point branch: P3P gate, then EPnP over all four
    if (t == 0) sh.p3p = p3p_solutions(p2, p3, K4);
    __syncthreads();
    if (sh.p3p == 0) {
      identity(2);
      return;
    }
    for (int i = t; i < 4; i += kThreads) {
      idx[i] = i;
      mask[i] = 1;
    }
    if (t == 0) {
      n_inliers[b] = 4;
      status[b] = 0;
    }
    return;
  }

  while (!sh.done) {
    // getSubset x 64, in iteration order.  The round's draws are generated in parallel by
    // jump-ahead (see mwc_mulmod; states at or above m -- the first draws from
    // RNG((uint64)-1) -- are stepped by lane 0 first).  A subset takes draws until it has 5
    // distinct indices, so the subset starting at draw s ends at a draw e(s) that depends on
    // the draws alone: every thread evaluates e(s) for its positions, thread 0 chains
    // s_{h+1} = e(s_h), and lane h deals subset h from s_h.  A chain that runs past the
    // generated draws continues sequentially (rng_next) from that subset on.
    if (wave == 0) {
      if (lane == 0) {
        unsigned long long z = sh.rng;
        int k = 0;
        while (z >= kMwcM && k < kRngPrefix) {
          const unsigned v = rng_next(z);
          sh.rst[k] = z;
          sh.rii[k] = (int)(v % (unsigned)n);
          ++k;
        }
        sh.rk = k;
        sh.rz = z;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int k = sh.rk;
      const unsigned long long z0 = sh.rz;
      if (z0 < kMwcM) {
        unsigned long long z = mwc_mulmod(z0, kMwcJumps.v[lane]);
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const unsigned v = rng_next(z);
          sh.rst[k + 6 * lane + i] = z;
          sh.rii[k + 6 * lane + i] = (int)(v % (unsigned)n);
        }
      }
      if (lane == 0) sh.rP = z0 < kMwcM ? k + 6 * 64 : k;
    }
    __syncthreads();
    {
      const int P = sh.rP;
      // the 5 distinct draws from position s: their positions' end (one past the 5th) or -1
      auto deal = [&](int s0, int* out) __attribute__((always_inline)) {
        int c0 = -1, c1 = -1, c2 = -1, c3 = -1, got = 0, q = s0;
        while (got < kModelPoints && q < P) {
          const int v = sh.rii[q++];
          if (v == c0 || v == c1 || v == c2 || v == c3) continue;
          if (out) out[got] = v;
          if (got == 0) c0 = v;
          else if (got == 1) c1 = v;
          else if (got == 2) c2 = v;
          else if (got == 3) c3 = v;
          ++got;
        }
        return got == kModelPoints ? q : -1;
      };
      for (int q = t; q < P; q += kThreads) sh.rend[q] = (short)deal(q, nullptr);
      __syncthreads();
      if (t == 0) {   // the chain of subset starts
        int q = 0, h = 0;
        for (; h < kRound && q >= 0 && q < P; ++h) {
          sh.rstart[h] = (short)q;
          q = sh.rend[q];
        }
        sh.rdealt = q < 0 ? h - 1 : h;   // subsets with all 5 draws among the generated ones
        sh.rpos = q;
      }
      __syncthreads();
      const int dealt = sh.rdealt;
      if (t < dealt) deal(sh.rstart[t], sh.subset[t]);
      if (t == 0) {
        unsigned long long st;
        if (dealt == kRound) {   // the state after the last draw dealt
          st = sh.rst[sh.rpos - 1];
        } else {   // sequential from subset `dealt`, at its start draw
          const int q0 = dealt > 0 ? sh.rend[sh.rstart[dealt - 1]] : 0;
          st = q0 > 0 ? sh.rst[q0 - 1] : sh.rng;
          int pos = q0;
          for (int h = dealt; h < kRound; ++h) {
            for (int i = 0; i < kModelPoints;) {
              int ii, j;
              for (;;) {
                if (pos < P) {
                  st = sh.rst[pos];
                  ii = sh.rii[pos];
                } else {
                  ii = (int)(rng_next(st) % (unsigned)n);
                }
                ++pos;
                for (j = 0; j < i; ++j)
                  if (ii == sh.subset[h][j]) break;
                if (j == i) break;
              }
              sh.subset[h][i] = ii;
              ++i;
            }
          }
        }
        sh.rng = st;
      }
    }
    __syncthreads();
    // @phase 2
    // one EPnP model per hypothesis: wave 0 the eigenvectors (lane h = hypothesis h), then
    // waves 1..3 one approximation each for every hypothesis; the smallest mean error wins
    // (ties to the earlier approximation, as compute_pose's sequential comparison)
    if (wave == 0) {
      epnp5_eig(sh.subset[lane], p2, p3, K4, sh.hh + lane, kRound);
      sh.count[lane] = 0;
    }
    __syncthreads();
    // @phase 3
    double Rw[9], tw[3];
    if (wave > 0) {
      epnp5_approx(wave, sh.subset[lane], p2, p3, K4, sh.hh + lane, kRound, Rw, tw,
                   &sh.herr[wave][lane]);
    }
    __syncthreads();
    if (wave > 0) {
      int best = 1;
      if (sh.herr[2][lane] < sh.herr[best][lane]) best = 2;
      if (sh.herr[3][lane] < sh.herr[best][lane]) best = 3;
      if (best == wave) {   // Rodrigues(R) -> rvec -> R, as solvePnP hands the model over
        double rvec[3], R[9];
        rodrigues_m2v(Rw, rvec);
        rodrigues_v2m(rvec, R);
        for (int i = 0; i < 9; ++i) sh.hypR[lane][i] = R[i];
        for (int i = 0; i < 3; ++i) {
          sh.hypT[lane][i] = tw[i];
          sh.hypRvec[lane][i] = rvec[i];
        }
      }
    }
    __syncthreads();
    // @phase 4
    // inlier counts and OpenCV's acceptance rule, 16 iterations at a time: iterations past
    // the stopping point are neither counted nor accepted (wave w counts w, w + 4, ...;
    // lanes sweep the points)
    for (int hb = 0; hb < kRound; hb += 16) {
      for (int h = hb + wave; h < hb + 16; h += 4) {
        int c = 0;
        for (int i = lane; i < n; i += 64)
          c += reproj_err2(sh.hypR[h], sh.hypT[h], K4, p3[3 * i], p3[3 * i + 1], p3[3 * i + 2],
                           p2[2 * i], p2[2 * i + 1]) <= thr;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
        if (lane == 0) sh.count[h] = c;
      }
      __syncthreads();
      if (t == 0) {  // in iteration order
        int iter = sh.iter, niters = sh.niters, best = sh.max_good;
        for (int h = hb; h < hb + 16 && iter < niters; ++h, ++iter) {
          const int good = sh.count[h];
          if (good > max(best, kModelPoints - 1)) {
            best = good;
            for (int i = 0; i < 3; ++i) {
              sh.bestRvec[i] = sh.hypRvec[h][i];
              sh.bestT[i] = sh.hypT[h][i];
            }
            niters = update_num_iters(confidence, (double)(n - good) / n, kModelPoints, niters);
          }
        }
        sh.iter = iter;
        sh.niters = niters;
        sh.max_good = best;
        sh.done = iter >= niters;
      }
      __syncthreads();
      if (sh.done) break;
    }
    // @phase 5
  }

  int nin;
  if (n == kModelPoints) {
    for (int i = t; i < n; i += kThreads) idx[i] = i;
    nin = n;
  } else {
    if (sh.max_good <= 0) {
      identity(2);
      return;
    }
    // inlier mask of the best model, compacted in point order
    double R[9];
    rodrigues_v2m(sh.bestRvec, R);
    if (t == 0) sh.n_inl = 0;
    __syncthreads();
    for (int base = 0; base < n; base += kThreads) {
      const int i = base + t;
      bool in = false;
      if (i < n)
        in = reproj_err2(R, sh.bestT, K4, p3[3 * i], p3[3 * i + 1], p3[3 * i + 2], p2[2 * i],
                         p2[2 * i + 1]) <= thr;
      const unsigned long long bal = __ballot(in);
      if (lane == 0) sh.wave_cnt[wave] = __popcll(bal);
      __syncthreads();
      int off = sh.n_inl;
      for (int w = 0; w < wave; ++w) off += sh.wave_cnt[w];
      if (in) {
        idx[off + __popcll(bal & ((1ull << lane) - 1ull))] = i;
        mask[i] = 1;
      }
      __syncthreads();
      if (t == 0) sh.n_inl += sh.wave_cnt[0] + sh.wave_cnt[1] + sh.wave_cnt[2] + sh.wave_cnt[3];
      __syncthreads();
    }
    nin = sh.n_inl;
  }
  // @phase 6
  if (n == kModelPoints)
    for (int i = t; i < n; i += kThreads) mask[i] = 1;
  if (t == 0) {   // the refit kernel reads these
    n_inliers[b] = nin;
    status[b] = 0;
  }
}

// EPnP on the RANSAC inliers (solvePnPRansac's final solvePnP call), then
// Rodrigues(R) -> rvec -> Rodrigues(rvec) as eval_utils.py:31 rebuilds R, t / scale.
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1)))
void pnp_refit_kernel(
    const float* __restrict__ pts2d, const float* __restrict__ pts3d, int max_points,
    const double* __restrict__ Kmat, int64_t K_bs, double scale, double* __restrict__ pose34,
    const int* __restrict__ n_inliers, const int* __restrict__ status,
    const int* __restrict__ idx_ws, const double* __restrict__ pose_gt, int64_t gt_bs,
    double* __restrict__ rerr, double* __restrict__ terr, uint8_t* __restrict__ cmd) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
  Shared& sh = *reinterpret_cast<Shared*>(dyn);
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  double* pose = pose34 + (int64_t)b * 12;
  // @phase 8
  // pose_gt (onepose_pose_stage): query_pose_error of the frame's final pose, fused
  auto errors = [&]() {
    if (pose_gt != nullptr && t == 0)
      pose_error_one(pose, pose_gt + b * gt_bs, rerr + b, terr + b, cmd + b * 3);
  };
  if (status[b] != 0) {   // identity pose (written by the RANSAC kernel)
    errors();
    return;
  }
  const int nin = n_inliers[b];
  const double* K = Kmat + b * K_bs;
  const double K4[4] = {K[0], K[4], K[2], K[5]};
  // the inliers, compacted into LDS once: every pass of the refit reads them from there (from
  // global memory each pass's loads sat behind the index load, one round trip after another)
  float* p2 = reinterpret_cast<float*>(dyn + ((sizeof(Shared) + 15) / 16) * 16);
  float* p3 = p2 + 2 * max_points;
  {
    const float* g2 = pts2d + (int64_t)b * max_points * 2;
    const float* g3 = pts3d + (int64_t)b * max_points * 3;
    const int* idx = idx_ws + (int64_t)b * max_points;
    for (int i = t; i < nin; i += kThreads) {
      const int j = idx[i];
      p2[2 * i] = g2[2 * j];
      p2[2 * i + 1] = g2[2 * j + 1];
      p3[3 * i] = g3[3 * j];
      p3[3 * i + 1] = g3[3 * j + 1];
      p3[3 * i + 2] = g3[3 * j + 2];
    }
    __syncthreads();
  }
  double Rf[9], tf[3], rv[3], Rr[9];
  epnp_refit(sh, p2, p3, nin, K4, Rf, tf);
  // @phase 14
  rodrigues_m2v(Rf, rv);
  rodrigues_v2m(rv, Rr);
  if (t == 0) {
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) pose[i * 4 + j] = Rr[i * 3 + j];
      pose[i * 4 + 3] = tf[i] / scale;
    }
  }
  errors();
}

}  // namespace
}  // namespace onepose

using namespace onepose;

extern "C" {

size_t onepose_pnp_workspace_bytes(int batch, int max_points, int max_iters) {
  (void)max_iters;
  if (batch <= 0 || max_points <= 0) return 0;
  return align_up((size_t)batch * max_points * sizeof(int), 256);
}

int onepose_pnp_ransac(const float* pts2d, const float* pts3d, const int* counts, int max_points,
                       const double* K, int64_t K_bstride, int batch, double scale,
                       float reproj_error, int max_iters, double confidence, double* pose34,
                       uint8_t* inlier_mask, int* n_inliers, int* status, void* workspace,
                       size_t workspace_bytes, void* stream) {
  clear_error();
  OP_REQUIRE(pts2d && pts3d && counts && K && pose34 && inlier_mask && n_inliers && status,
             "pnp: null pointer");
  OP_REQUIRE(batch >= 1 && max_points >= 1 && max_points <= 8192, "pnp: batch=%d max_points=%d",
             batch, max_points);
  OP_REQUIRE(confidence > 0 && confidence < 1, "pnp: confidence %f not in (0,1)", confidence);
  OP_REQUIRE(scale != 0.0, "pnp: scale 0");
  const size_t need = onepose_pnp_workspace_bytes(batch, max_points, max_iters);
  if (!workspace || workspace_bytes < need) {
    set_error("pnp: workspace %zu < %zu bytes", workspace_bytes, need);
    return ONEPOSE_ERR_WORKSPACE;
  }
  const size_t lds = ((sizeof(Shared) + 15) / 16) * 16 + (size_t)max_points * 5 * sizeof(float);
  OP_REQUIRE(lds <= 160 * 1024, "pnp: max_points=%d needs %zu B of LDS", max_points, lds);
  static bool attr_set = false;
  if (!attr_set) {
    OP_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(pnp_ransac_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    OP_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(pnp_refit_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  SelArgs none{};
  OP_LAUNCH(K_PNP, st, pnp_ransac_kernel, dim3(batch), dim3(kThreads), lds, st, pts2d, pts3d,
            counts, max_points, K, K_bstride, scale, reproj_error, max_iters, confidence, pose34,
            inlier_mask, n_inliers, status, static_cast<int*>(workspace), none, nullptr, nullptr,
            nullptr);
  OP_LAUNCH(K_PNP_REFIT, st, pnp_refit_kernel, dim3(batch), dim3(kThreads), lds, st, pts2d, pts3d,
            max_points, K, K_bstride, scale, pose34, n_inliers, status,
            static_cast<const int*>(workspace), nullptr, (int64_t)0, nullptr, nullptr, nullptr);
  return ONEPOSE_OK;
}

int onepose_pose_stage(const int64_t* matches0, const float* kpts2d, int64_t kpts2d_bstride,
                       const float* kpts3d, int64_t kpts3d_bstride, int batch, int n1, int n3,
                       double scale, const double* K, int64_t K_bstride, float reproj_error,
                       int max_iters, double confidence, const double* pose_gt,
                       int64_t gt_bstride, float* pts2d, float* pts3d, int* counts,
                       double* pose34, uint8_t* inlier_mask, int* n_inliers, int* status,
                       double* R_err_deg, double* t_err_cm, uint8_t* cmd, void* workspace,
                       size_t workspace_bytes, void* stream) {
  clear_error();
  OP_REQUIRE(matches0 && kpts2d && kpts3d && K && pts2d && pts3d && counts && pose34 &&
                 inlier_mask && n_inliers && status,
             "pose_stage: null pointer");
  OP_REQUIRE(!pose_gt || (R_err_deg && t_err_cm && cmd), "pose_stage: null error output");
  OP_REQUIRE(batch >= 1 && n1 >= 1 && n1 <= 8192 && n3 >= 1, "pose_stage: batch=%d n1=%d n3=%d",
             batch, n1, n3);
  OP_REQUIRE(confidence > 0 && confidence < 1, "pose_stage: confidence %f not in (0,1)",
             confidence);
  OP_REQUIRE(scale != 0.0, "pose_stage: scale 0");
  const int max_points = n1;
  const size_t need = onepose_pnp_workspace_bytes(batch, max_points, max_iters);
  if (!workspace || workspace_bytes < need) {
    set_error("pose_stage: workspace %zu < %zu bytes", workspace_bytes, need);
    return ONEPOSE_ERR_WORKSPACE;
  }
  const size_t lds = ((sizeof(Shared) + 15) / 16) * 16 + (size_t)max_points * 5 * sizeof(float);
  OP_REQUIRE(lds <= 160 * 1024, "pose_stage: n1=%d needs %zu B of LDS", n1, lds);
  static bool attr_set = false;
  if (!attr_set) {
    OP_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(pnp_ransac_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    OP_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(pnp_refit_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  const SelArgs sel{matches0, kpts2d, kpts2d_bstride, kpts3d, kpts3d_bstride, n1, n3, scale};
  OP_LAUNCH(K_PNP, st, pnp_ransac_kernel, dim3(batch), dim3(kThreads), lds, st, nullptr, nullptr,
            nullptr, max_points, K, K_bstride, scale, reproj_error, max_iters, confidence, pose34,
            inlier_mask, n_inliers, status, static_cast<int*>(workspace), sel, pts2d, pts3d,
            counts);
  OP_LAUNCH(K_PNP_REFIT, st, pnp_refit_kernel, dim3(batch), dim3(kThreads), lds, st, pts2d, pts3d,
            max_points, K, K_bstride, scale, pose34, n_inliers, status,
            static_cast<const int*>(workspace), pose_gt, gt_bstride, R_err_deg, t_err_cm, cmd);
  return ONEPOSE_OK;
}

}  // extern "C"
