// Dev tool (not shipped): sample the core clock of one CU while another process (bench.py)
// runs: each sample is a one-workgroup kernel spinning ~40 us on s_memtime (shader clock) vs
// s_memrealtime (100 MHz); N samples, ~1 ms apart.
//   hipcc -O3 --offload-arch=gfx950 tools/clock_sampler.hip -o tools/clock_sampler
#include <hip/hip_runtime.h>
#include <unistd.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void sample(double* out, int i) {
  if (threadIdx.x != 0) return;
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = r0, c1 = c0;
  while (r1 - r0 < 4000) {
    r1 = __builtin_amdgcn_s_memrealtime();
    c1 = __builtin_amdgcn_s_memtime();
  }
  out[i] = (double)(c1 - c0) / (double)(r1 - r0) * 0.1;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 100;
  double* d;
  (void)hipMalloc(&d, n * sizeof(double));
  for (int i = 0; i < n; ++i) {
    sample<<<1, 64>>>(d, i);
    (void)hipDeviceSynchronize();
    usleep(1000);
  }
  std::vector<double> h(n);
  (void)hipMemcpy(h.data(), d, n * sizeof(double), hipMemcpyDeviceToHost);
  double s = 0, mn = 1e9, mx = 0;
  for (double v : h) { s += v; mn = v < mn ? v : mn; mx = v > mx ? v : mx; }
  printf("clock samples %d: mean %.3f GHz min %.3f max %.3f\n", n, s / n, mn, mx);
  for (int i = 0; i < n; ++i) printf("%.2f%c", h[i], i % 20 == 19 ? '\n' : ' ');
  printf("\n");
  return 0;
}
