// Dev tool (not shipped): cycles per GEMM stage (16 MFMA 32x32x2 f32 per wave) for one
// 256-thread workgroup per CU, adding the GEMM loop's ingredients one at a time:
//   0: MFMA on LDS fragments (2 ds_read_b128 per 4 MFMAs)   1: + barrier per stage
//   2: + 4 ds_write_b128 per thread per stage              3: + 4 global float4 loads per stage
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -w tools/stage_probe.hip -o tools/stage_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int MODE>
__global__ __launch_bounds__(256) void stage_loop(const float4* g, float* out, unsigned long long* cyc,
                                                  int stages) {
  __shared__ __attribute__((aligned(16))) float lds[2 * 128 * 36];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, wm = wave >> 1, wn = wave & 1;
  for (int i = t; i < 2 * 128 * 36; i += 256) lds[i] = (i % 7) * 0.01f;
  __syncthreads();
  floatx16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  float4 st[4];
  for (int i = 0; i < 4; ++i) st[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4* gp = g + (blockIdx.x * 256 + t) % 65536;
  const unsigned long long c0 = clock64();
  for (int s = 0; s < stages; ++s) {
    const float* la = lds + (s & 1) * 128 * 36;
    if (MODE >= 3) {
#pragma unroll
      for (int i = 0; i < 4; ++i) st[i] = gp[((s * 4 + i) * 4096) % 65536];
    }
    const float* pa = la + (wm * 32 + (lane & 31)) * 36 + (lane >> 5) * 4;
    const float* pw = la + 64 * 36 + (wn * 32 + (lane & 31)) * 36 + (lane >> 5) * 4;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const float4 a = *reinterpret_cast<const float4*>(pa + kk * 8);
      const float4 w = *reinterpret_cast<const float4*>(pw + kk * 8);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, w.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, w.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, w.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, w.w, acc, 0, 0, 0);
    }
    if (MODE >= 2) {
      float* na = lds + ((s + 1) & 1) * 128 * 36;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<float4*>(na + ((t >> 3) + 32 * i) * 36 + (t & 7) * 4) = st[i];
    }
    if (MODE >= 1) __syncthreads();
  }
  const unsigned long long c1 = clock64();
  float sum = 0.f;
  for (int i = 0; i < 16; ++i) sum += acc[i];
  out[blockIdx.x * 256 + t] = sum + st[0].x + st[3].w;
  if (t == 0) cyc[blockIdx.x] = c1 - c0;
}

template <int MODE>
void run(const float4* g, float* out, unsigned long long* cyc, int wgs) {
  const int stages = 256;
  for (int r = 0; r < 2; ++r)
    hipLaunchKernelGGL(stage_loop<MODE>, dim3(wgs), dim3(256), 0, 0, g, out, cyc, stages);
  hipDeviceSynchronize();
  static unsigned long long h[2048];
  hipMemcpy(h, cyc, wgs * 8, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < wgs; ++i) s += h[i];
  printf("mode %d, %4d WGs: %7.1f cycles per stage (MFMA floor 1024)\n", MODE, wgs, s / wgs / stages);
}

int main() {
  float4* g;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&g, 65536 * 16);
  hipMemset(g, 0, 65536 * 16);
  hipMalloc(&out, 2048 * 256 * 4);
  hipMalloc(&cyc, 2048 * 8);
  for (int wgs : {256, 512, 768}) {
    run<0>(g, out, cyc, wgs);
    run<1>(g, out, cyc, wgs);
    run<2>(g, out, cyc, wgs);
    run<3>(g, out, cyc, wgs);
  }
  return 0;
}
