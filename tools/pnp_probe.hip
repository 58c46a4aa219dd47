// Dev tool (not shipped): phase timeline of the EPnP refit kernel on one synthetic frame.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/pnp_probe.hip -o tools/pnp_probe
#define ONEPOSE_PNP_PHASES 1
#include "../onepose_amd/csrc/pnp.hip"
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
int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 700;
  const double outl = argc > 2 ? atof(argv[2]) : 0.0;   // fraction of gross outliers
  std::uniform_real_distribution<float> U01(0.f, 1.f), UI(0.f, 512.f);
  std::mt19937 rng(3);
  std::uniform_real_distribution<float> U(-100.f, 100.f);
  std::normal_distribution<float> N(0.f, 0.5f);
  const double K[9] = {600, 0, 256, 0, 600, 256, 0, 0, 1};
  const double R[9] = {0.36, 0.48, -0.8, -0.8, 0.6, 0, 0.48, 0.64, 0.6}, t[3] = {10, -20, 450};
  std::vector<float> p2(2 * n), p3(3 * n);
  for (int i = 0; i < n; ++i) {
    for (int k = 0; k < 3; ++k) p3[3 * i + k] = U(rng);
    double X[3];
    for (int r = 0; r < 3; ++r) X[r] = R[3 * r] * p3[3 * i] + R[3 * r + 1] * p3[3 * i + 1] + R[3 * r + 2] * p3[3 * i + 2] + t[r];
    p2[2 * i] = (float)(600 * X[0] / X[2] + 256) + N(rng);
    p2[2 * i + 1] = (float)(600 * X[1] / X[2] + 256) + N(rng);
    if (U01(rng) < outl) {
      p2[2 * i] = UI(rng);
      p2[2 * i + 1] = UI(rng);
    }
  }
  float *d2, *d3; double *dK, *pose; int *cnt, *nin, *st; uint8_t* mask; void* ws;
  hipMalloc(&d2, 8 * n); hipMalloc(&d3, 12 * n); hipMalloc(&dK, 72); hipMalloc(&pose, 96);
  hipMalloc(&cnt, 4); hipMalloc(&nin, 4); hipMalloc(&st, 4); hipMalloc(&mask, n);
  const size_t wsb = onepose_pnp_workspace_bytes(1, n, 10000); hipMalloc(&ws, wsb);
  hipMemcpy(d2, p2.data(), 8 * n, hipMemcpyHostToDevice); hipMemcpy(d3, p3.data(), 12 * n, hipMemcpyHostToDevice);
  hipMemcpy(dK, K, 72, hipMemcpyHostToDevice); hipMemcpy(cnt, &n, 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int it = 0; it < 3; ++it) {
    hipEventRecord(e0);
    onepose_pnp_ransac(d2, d3, cnt, n, dK, 0, 1, 1.0, 5.0f, 10000, 0.99, pose, mask, nin, st, ws, wsb, nullptr);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long ph[16]; hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_pnp_phase), sizeof(ph));
    int ni; hipMemcpy(&ni, nin, 4, hipMemcpyDeviceToHost);
    printf("n=%d inliers=%d ransac+refit %.1f us | refit phases (us): MtM+reduce %.1f  assemble %.1f  eig+L %.1f  approx %.1f  total %.1f\n",
           n, ni, ms * 1e3, (ph[1] - ph[0]) / 100.0, (ph[2] - ph[1]) / 100.0, (ph[3] - ph[2]) / 100.0,
           (ph[4] - ph[3]) / 100.0, (ph[5] - ph[0]) / 100.0);
    printf("  ransac phases (us, last round): load %.1f  subsets %.1f  epnp5 x64 %.1f  count %.1f  accept %.1f  mask %.1f\n",
           (ph[8] - 0) * 0.0, (ph[9] - ph[8]) / 100.0, (ph[10] - ph[9]) / 100.0, (ph[11] - ph[10]) / 100.0,
           (ph[12] - ph[11]) / 100.0, (ph[13] - ph[12]) / 100.0);
  }
  return 0;
}
