// Where does the pose stage's time go?  Wraps pnp.hip's kernels with phase stamps (thread 0 of
// workgroup 0 records s_memtime at each "// @phase" marker) and runs onepose_pnp_ransac on
// one synthetic frame (tests/test_pnp_gpu.py's scene: cube of points 0.35-0.55 m away, 0.5 px
// noise, a fraction of uniform outliers), serially, reporting per phase the median cycles.
//
//   bash tools/probe_src.sh   (generates _gen/pnp.hip with the stamps, then builds)
//   ./tools/pnp_probe [n] [outlier_frac]
__device__ unsigned long long g_pph[24];
__device__ unsigned g_pcnt[24];
#define ONEPOSE_PNP_PHASE(i)                                   \
  if (threadIdx.x == 0 && blockIdx.x == 0) {                   \
    g_pph[(i)] = __builtin_amdgcn_s_memtime();                 \
    g_pcnt[(i)] += 1u;                                         \
  }
#include "_gen/pnp.hip"   // tools/probe_src.sh
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <random>
#include <vector>

namespace onepose {
void set_error(const char* fmt, ...) { va_list ap; va_start(ap, fmt); vprintf(fmt, ap); va_end(ap); printf("\n"); }
void clear_error() {}
void prof_pre(int, hipStream_t) {}
void prof_post(int, hipStream_t) {}
StampAcc* prof_stamp_slot(int) { return nullptr; }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 700;
  const double out_frac = argc > 2 ? atof(argv[2]) : 0.3;
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  std::normal_distribution<double> N01(0.0, 1.0);
  const double K[9] = {600, 0, 256, 0, 600, 256, 0, 0, 1};
  double ax[3] = {N01(rng), N01(rng), N01(rng)};
  const double an = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]), th = 2.0 * U(rng);
  double R[9];

  {
    const double k0 = ax[0] / an, k1 = ax[1] / an, k2 = ax[2] / an, c = std::cos(th), s = std::sin(th);
    const double C = 1 - c;
    const double r[9] = {c + k0 * k0 * C, k0 * k1 * C - k2 * s, k0 * k2 * C + k1 * s,
                         k1 * k0 * C + k2 * s, c + k1 * k1 * C, k1 * k2 * C - k0 * s,
                         k2 * k0 * C - k1 * s, k2 * k1 * C + k0 * s, c + k2 * k2 * C};
    for (int i = 0; i < 9; ++i) R[i] = r[i];
  }
  const double t[3] = {0.03 * (2 * U(rng) - 1), 0.03 * (2 * U(rng) - 1), 0.35 + 0.2 * U(rng)};
  std::vector<float> p2(2 * n), p3(3 * n);
  for (int i = 0; i < n; ++i) {
    double X[3];
    for (int k = 0; k < 3; ++k) X[k] = (float)(0.2 * U(rng) - 0.1);
    const double Xc = R[0] * X[0] + R[1] * X[1] + R[2] * X[2] + t[0];
    const double Yc = R[3] * X[0] + R[4] * X[1] + R[5] * X[2] + t[1];
    const double Zc = R[6] * X[0] + R[7] * X[1] + R[8] * X[2] + t[2];
    double u = K[0] * Xc / Zc + K[2] + 0.5 * N01(rng), v = K[4] * Yc / Zc + K[5] + 0.5 * N01(rng);
    if (U(rng) < out_frac) {
      u = 512 * U(rng);
      v = 512 * U(rng);
    }
    p2[2 * i] = (float)u;
    p2[2 * i + 1] = (float)v;
    for (int k = 0; k < 3; ++k) p3[3 * i + k] = (float)(X[k] * 1000.0);
  }
  float *d2, *d3;
  int *dcnt, *dnin, *dst;
  double *dK, *dpose;
  uint8_t* dmask;
  void* ws;
  const size_t wsb = onepose_pnp_workspace_bytes(1, n, 1000);
  CK(hipMalloc(&d2, 8 * n));
  CK(hipMalloc(&d3, 12 * n));
  CK(hipMalloc(&dcnt, 4));
  CK(hipMalloc(&dnin, 4));
  CK(hipMalloc(&dst, 4));
  CK(hipMalloc(&dK, 72));
  CK(hipMalloc(&dpose, 96));
  CK(hipMalloc(&dmask, n));
  CK(hipMalloc(&ws, wsb));
  CK(hipMemcpy(d2, p2.data(), 8 * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(d3, p3.data(), 12 * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(dcnt, &n, 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dK, K, 72, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 30;
  std::vector<std::vector<double>> ph(20);
  std::vector<double> ev;
  unsigned cnt0[24] = {0}, cnt1[24];
  int nin = 0;
  for (int r = 0; r < reps; ++r) {
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_pcnt), cnt0, sizeof(cnt0)));
    CK(hipEventRecord(e0, 0));
    if (onepose_pnp_ransac(d2, d3, dcnt, n, dK, 0, 1, 1000.0, 5.0f, 1000, 0.99, dpose, dmask, dnin,
                           dst, ws, wsb, 0) != 0)
      return 1;
    CK(hipEventRecord(e1, 0));
    CK(hipDeviceSynchronize());
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ev.push_back(ms * 1e3);
    unsigned long long st[24];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_pph), sizeof(st)));
    CK(hipMemcpyFromSymbol(cnt1, HIP_SYMBOL(g_pcnt), sizeof(cnt1)));
    for (int i = 1; i < 16; ++i)
      if (cnt1[i] && cnt1[i - 1]) ph[i].push_back((double)(long long)(st[i] - st[i - 1]));
    for (int i = 16; i < 20; ++i)   // markers inside the refit's approximations: since phase 12
      if (cnt1[i] && cnt1[12]) ph[i].push_back((double)(long long)(st[i] - st[12]));
    CK(hipMemcpy(&nin, dnin, 4, hipMemcpyDeviceToHost));
  }
  auto med = [](std::vector<double> v) {
    if (v.empty()) return -1.0;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  printf("n %d outliers %.2f inliers %d ransac rounds %u (hook 2 count)\n", n, out_frac, nin, cnt1[2]);
  printf("both kernels, event-timed: median %.1f us\n", med(ev));
  const char* names[16] = {"", "ransac: load / select", "ransac: deal subsets (last round)",
                           "ransac: eig (last round)", "ransac: 3 approximations (last round)",
                           "ransac: counts + accept (last round)", "ransac: inlier mask",
                           "", "", "refit: centroid + PCA", "refit: M^T M sums", "refit: jacobi12",
                           "refit: L, rho", "refit: 3 approximations", "refit: rest of epnp_refit", ""};
  for (int i = 1; i < 15; ++i)
    if (names[i][0]) printf("  %-40s %8.0f cycles (s_memtime)\n", names[i], med(ph[i]));
  const char* inner[4] = {"refit approx 1: betas + GN + ccs (lane 0)", "  + centroid / abt sums",
                          "  + finish_R", ""};
  for (int i = 16; i < 19; ++i)
    if (!ph[i].empty()) printf("  %-40s %8.0f cycles since phase 12\n", inner[i - 16], med(ph[i]));
  return 0;
}
