// Dev tool (not shipped): cycles per v_mfma_f32_32x32x2_f32 for one wave per SIMD with 1, 2 or 4
// independent accumulator chains (operands in registers).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -w tools/mfma_chain.hip -o tools/mfma_chain
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(256) void chain(float* out, unsigned long long* cyc, int n) {
  floatx16 acc[NACC];
  for (int j = 0; j < NACC; ++j)
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
  float x = threadIdx.x * 1e-3f, y = 1.0001f;
  const unsigned long long c0 = clock64();
  for (int it = 0; it < n; it += NACC) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, acc[j], 0, 0, 0);
  }
  const unsigned long long c1 = clock64();
  float s = 0.f;
  for (int j = 0; j < NACC; ++j)
    for (int i = 0; i < 16; ++i) s += acc[j][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
}

template <int NACC>
void run(float* out, unsigned long long* cyc, int n) {
  hipLaunchKernelGGL(chain<NACC>, dim3(256), dim3(256), 0, 0, out, cyc, n);
  hipLaunchKernelGGL(chain<NACC>, dim3(256), dim3(256), 0, 0, out, cyc, n);
  hipDeviceSynchronize();
  unsigned long long h[256];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < 256; ++i) s += h[i];
  printf("accumulators %d: %.1f cycles per MFMA (one wave per SIMD)\n", NACC, s / 256 / n);
}

int main() {
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 256 * 4);
  hipMalloc(&cyc, 256 * 8);
  run<1>(out, cyc, 4096);
  run<2>(out, cyc, 4096);
  run<4>(out, cyc, 4096);
  return 0;
}
