/* Sanitizer driver (test infrastructure): runs the C RANSAC-EPnP oracle (oracle/epnp_ransac.c)
 * over synthetic scenes -- exact, noisy, with outliers, degenerate sizes 0-6, duplicated points
 * -- so that an -fsanitize=address,undefined build reports any out-of-bounds access, leak or
 * undefined behaviour.  Built and run by tests/test_sanitize.py; exit status 0 = every scene ran. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oracle_pnp_ransac(const float* p2, const float* p3, int n, const double* K, double scale,
                      float reproj_error, int max_iters, double confidence, double* pose34,
                      unsigned char* mask, int* n_inliers, int* iters_run);
void oracle_epnp(const double* pws, const double* us, int n, const double* K, double* R_out,
                 double* t_out);
void oracle_rng_draws(unsigned* out, int count);

static unsigned s = 12345u;
static double urand(void) {
  s = s * 1664525u + 1013904223u;
  return (double)(s >> 8) / 16777216.0;
}

static int scene(int n, double noise, double outlier_frac, int dup) {
  const double K[9] = {600, 0, 256, 0, 600, 256, 0, 0, 1};
  const double R[9] = {0.936, -0.275, 0.218, 0.289, 0.956, -0.036, -0.199, 0.098, 0.975};
  const double t[3] = {0.05, -0.03, 1.2};
  float* p3 = (float*)malloc(sizeof(float) * 3 * (n > 0 ? n : 1));
  float* p2 = (float*)malloc(sizeof(float) * 2 * (n > 0 ? n : 1));
  unsigned char* mask = (unsigned char*)malloc(n > 0 ? n : 1);
  for (int i = 0; i < n; ++i) {
    const int src = dup && i > 0 && (i % 3 == 0) ? i - 1 : i;
    if (src != i) {
      memcpy(p3 + 3 * i, p3 + 3 * src, 12);
    } else {
      for (int k = 0; k < 3; ++k) p3[3 * i + k] = (float)(urand() - 0.5) * 0.2f;
    }
    double pc[3];
    for (int r = 0; r < 3; ++r)
      pc[r] = R[3 * r] * p3[3 * i] + R[3 * r + 1] * p3[3 * i + 1] + R[3 * r + 2] * p3[3 * i + 2] + t[r];
    p2[2 * i] = (float)(K[0] * pc[0] / pc[2] + K[2] + noise * (urand() - 0.5));
    p2[2 * i + 1] = (float)(K[4] * pc[1] / pc[2] + K[5] + noise * (urand() - 0.5));
    if (urand() < outlier_frac) {
      p2[2 * i] = (float)(urand() * 512);
      p2[2 * i + 1] = (float)(urand() * 512);
    }
  }
  double pose[12];
  int ninl = 0, iters = 0;
  const int st = oracle_pnp_ransac(p2, p3, n, K, 1.0, 8.0f, 10000, 0.99, pose, mask, &ninl, &iters);
  for (int i = 0; i < 12; ++i)
    if (!isfinite(pose[i])) {
      fprintf(stderr, "non-finite pose (n=%d)\n", n);
      return 1;
    }
  if (n >= 4) {   /* EPnP on every correspondence, through the public entry point */
    double* pw = (double*)malloc(sizeof(double) * 3 * n);
    double* us = (double*)malloc(sizeof(double) * 2 * n);
    for (int i = 0; i < 3 * n; ++i) pw[i] = p3[i];
    for (int i = 0; i < 2 * n; ++i) us[i] = p2[i];
    double Ro[9], to[3];
    oracle_epnp(pw, us, n, K, Ro, to);
    free(pw);
    free(us);
  }
  printf("n=%d noise=%.1f outliers=%.2f dup=%d: status %d, %d inliers, %d iterations\n", n, noise,
         outlier_frac, dup, st, ninl, iters);
  free(p3);
  free(p2);
  free(mask);
  return 0;
}

int main(void) {
  unsigned draws[64];
  oracle_rng_draws(draws, 64);
  int bad = 0;
  for (int n = 0; n <= 6; ++n) bad |= scene(n, 0.0, 0.0, 0);
  bad |= scene(50, 0.0, 0.0, 0);
  bad |= scene(300, 1.0, 0.2, 0);
  bad |= scene(300, 2.0, 0.6, 0);
  bad |= scene(120, 0.5, 0.3, 1);
  bad |= scene(1024, 1.0, 0.5, 0);
  return bad;
}
