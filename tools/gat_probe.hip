// Dev tool (not shipped): GAT kernel variants at config 2 (n3 = 4096, L = 8, stored leaf
// logits), HIP events over 200 launches each; the leaves (33.5 MB) are re-read every launch as
// in the frame.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -w tools/gat_probe.hip -o tools/gat_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

constexpr int kDim = 256, kLogitStride = 16;
__device__ __forceinline__ float elu1(float x) { return x > 0.f ? x : (expf(x) - 1.0f); }
__device__ __forceinline__ float gat_dot(float4 a, float4 w) {
  return fmaf(a.w, w.w, fmaf(a.z, w.z, fmaf(a.y, w.y, a.x * w.x)));
}

// NT: non-temporal leaf loads; PPW: points per wave (loads of all points issued first)
template <int NT, int PPW, int WPB>
__global__ __launch_bounds__(64 * WPB) void gat_v(const float* __restrict__ x3,
                                                  const float* __restrict__ leaves_pm,
                                                  const float* __restrict__ wa,
                                                  const float* __restrict__ slog,
                                                  float* __restrict__ y3, int n3) {
  constexpr int L = 8;
  const int lane = threadIdx.x & 63;
  const int p0 = (blockIdx.x * WPB + (threadIdx.x >> 6)) * PPW;
  if (p0 >= n3) return;
  const float4 wh = reinterpret_cast<const float4*>(wa + 256)[lane];
  float4 h[PPW], lf[PPW][L];
#pragma unroll
  for (int q = 0; q < PPW; ++q) {
    const int p = p0 + q;
    h[q] = reinterpret_cast<const float4*>(x3 + (int64_t)p * kDim)[lane];
    typedef float fv4 __attribute__((ext_vector_type(4)));
    const fv4* lp = reinterpret_cast<const fv4*>(leaves_pm + (int64_t)p * L * kDim) + lane;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const fv4 v = NT ? __builtin_nontemporal_load(lp + j * 64) : lp[j * 64];
      lf[q][j] = make_float4(v.x, v.y, v.z, v.w);
    }
  }
#pragma unroll
  for (int q = 0; q < PPW; ++q) {
    const int p = p0 + q;
    float d0 = gat_dot(h[q], wh);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) d0 += __shfl_xor(d0, o, 64);
    const float* sl = slog + (int64_t)__builtin_amdgcn_readfirstlane(p) * kLogitStride;
    float e[L + 1];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j <= L; ++j) {
      float v = d0 + (j == 0 ? d0 : sl[j - 1]);
      v = v > 0.f ? v : v * 0.2f;
      e[j] = v;
      mx = fmaxf(mx, v);
    }
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j <= L; ++j) { e[j] = expf(e[j] - mx); sum += e[j]; }
    const float a0 = e[0] / sum;
    float4 acc = make_float4(a0 * h[q].x, a0 * h[q].y, a0 * h[q].z, a0 * h[q].w);
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const float a = e[j + 1] / sum;
      acc.x += a * lf[q][j].x; acc.y += a * lf[q][j].y; acc.z += a * lf[q][j].z; acc.w += a * lf[q][j].w;
    }
    reinterpret_cast<float4*>(y3 + (int64_t)p * kDim)[lane] =
        make_float4(elu1(acc.x), elu1(acc.y), elu1(acc.z), elu1(acc.w));
  }
}

template <int NT, int PPW, int WPB>
void run(const char* name, const float* x, const float* lv, const float* wa, const float* sl, float* y, int n3) {
  const int grid = (n3 / PPW + WPB - 1) / WPB;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 20; ++w)
    hipLaunchKernelGGL((gat_v<NT, PPW, WPB>), dim3(grid), dim3(64 * WPB), 0, 0, x, lv, wa, sl, y, n3);
  hipEventRecord(e0);
  const int it = 200;
  for (int w = 0; w < it; ++w)
    hipLaunchKernelGGL((gat_v<NT, PPW, WPB>), dim3(grid), dim3(64 * WPB), 0, 0, x, lv, wa, sl, y, n3);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / it, bytes = (double)n3 * 256 * 4 * 10;
  printf("%-22s pts/wave %d waves/wg %2d grid %5d  %6.2f us  %5.2f TB/s\n", name, PPW, WPB, grid, us,
         bytes / (us * 1e-6) / 1e12);
}

int main() {
  const int n3 = 4096, L = 8;
  std::mt19937 rng(1);
  std::normal_distribution<float> N(0.f, 0.06f);
  std::vector<float> x((size_t)n3 * 256), lv((size_t)n3 * L * 256), wa(512), sl((size_t)n3 * 16);
  for (auto& v : x) v = N(rng);
  for (auto& v : lv) v = N(rng);
  for (auto& v : wa) v = N(rng);
  for (auto& v : sl) v = N(rng);
  float *dx, *dl, *dw, *ds, *dy;
  hipMalloc(&dx, x.size() * 4); hipMalloc(&dl, lv.size() * 4); hipMalloc(&dw, 2048);
  hipMalloc(&ds, sl.size() * 4); hipMalloc(&dy, x.size() * 4);
  hipMemcpy(dx, x.data(), x.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dl, lv.data(), lv.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dw, wa.data(), 2048, hipMemcpyHostToDevice);
  hipMemcpy(ds, sl.data(), sl.size() * 4, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep) {
    run<0, 1, 4>("as built", dx, dl, dw, ds, dy, n3);
    run<1, 1, 4>("nontemporal leaves", dx, dl, dw, ds, dy, n3);
    run<0, 2, 4>("2 points per wave", dx, dl, dw, ds, dy, n3);
    run<0, 1, 8>("8 waves per wg", dx, dl, dw, ds, dy, n3);
    run<0, 1, 2>("2 waves per wg", dx, dl, dw, ds, dy, n3);
    run<0, 1, 1>("1 wave per wg", dx, dl, dw, ds, dy, n3);
    run<1, 2, 2>("nt, 2 pts, 2 waves", dx, dl, dw, ds, dy, n3);
  }
  return 0;
}
