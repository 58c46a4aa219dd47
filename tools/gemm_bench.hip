// Microbenchmark for tile configurations of the fp32-MFMA token GEMM (dev tool, not shipped).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gemm_bench.hip -o /tmp/gemm_bench
// Shapes: the four per-layer GEMMs of config 2 (2D side 1024 tokens + 3D side 4096 tokens in
// one launch).  Reports mean kernel time over 50 launches and TFLOP/s.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float floatx16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

struct Prob {
  const float* A;
  const float* W;
  float* Y;
  int M, N, K, mtiles, ntiles, tiles;
};
struct Args {
  Prob p[2];
};

// BM x BN tile, BK deep, WM x WN waves; each wave owns (BM/WM) x (BN/WN) = FM*32 x FN*32.
template <int BM, int BN, int BK, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void gemm_v(Args args) {
  constexpr int NT = 64 * WM * WN;
  constexpr int P = BK + 4;
  constexpr int FM = BM / WM / 32, FN = BN / WN / 32;
  constexpr int A4 = BM * BK / 4 / NT, W4 = BN * BK / 4 / NT;   // float4 per thread per stage
  static_assert(A4 >= 1 && W4 >= 1, "tile too small for the thread count");
  __shared__ __attribute__((aligned(16))) float lds[2 * (BM + BN) * P];
  int bid = blockIdx.x;
  const bool second = bid >= args.p[0].tiles;
  const Prob& pr = second ? args.p[1] : args.p[0];
  if (second) bid -= args.p[0].tiles;
  const int mt = bid / pr.ntiles, nt = bid - mt * pr.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int M = pr.M, N = pr.N, K = pr.K;
  const float* A = pr.A;
  const float* W = pr.W;
  constexpr int KQ = BK / 4;   // float4 per row
  float4 ra[A4], rw[W4];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A4; ++i) {
      const int e = t + NT * i, r = e / KQ, c = (e % KQ) * 4;
      ra[i] = (m0 + r < M) ? *reinterpret_cast<const float4*>(A + (int64_t)(m0 + r) * K + k0 + c)
                           : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < W4; ++i) {
      const int e = t + NT * i, r = e / KQ, c = (e % KQ) * 4;
      rw[i] = (n0 + r < N) ? *reinterpret_cast<const float4*>(W + (int64_t)(n0 + r) * K + k0 + c)
                           : make_float4(0, 0, 0, 0);
    }
  };
  auto store = [&](int buf) {
    float* la = lds + buf * (BM + BN) * P;
    float* lw = la + BM * P;
#pragma unroll
    for (int i = 0; i < A4; ++i) {
      const int e = t + NT * i, r = e / KQ, c = (e % KQ) * 4;
      *reinterpret_cast<float4*>(la + r * P + c) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < W4; ++i) {
      const int e = t + NT * i, r = e / KQ, c = (e % KQ) * 4;
      *reinterpret_cast<float4*>(lw + r * P + c) = rw[i];
    }
  };
  floatx16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = K / BK;
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load((kt + 1) * BK);
    const float* la = lds + (kt & 1) * (BM + BN) * P;
    const float* lw = la + BM * P;
#pragma unroll
    for (int kk = 0; kk < BK / 8; ++kk) {
      float4 a[FM], w[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        a[i] = *reinterpret_cast<const float4*>(la + (wm * FM * 32 + i * 32 + (lane & 31)) * P + kk * 8 + (lane >> 5) * 4);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        w[j] = *reinterpret_cast<const float4*>(lw + (wn * FN * 32 + j * 32 + (lane & 31)) * P + kk * 8 + (lane >> 5) * 4);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, w[j].x, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, w[j].y, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, w[j].z, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, w[j].w, acc[i][j], 0, 0, 0);
        }
    }
    if (kt + 1 < nk) store((kt + 1) & 1);
    __syncthreads();
  }
  float* Y = pr.Y;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * FM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int col = n0 + wn * FN * 32 + j * 32 + (lane & 31);
        if (row < M && col < N) Y[(int64_t)row * N + col] = acc[i][j][r];
      }
}

template <int BM, int BN, int BK, int WM, int WN>
void run(const char* name, float* A2, float* A3, float* W, float* Y2, float* Y3, int N, int K) {
  Args a;
  const int Ms[2] = {1024, 4096};
  float* As[2] = {A2, A3};
  float* Ys[2] = {Y2, Y3};
  int grid = 0;
  for (int i = 0; i < 2; ++i) {
    a.p[i] = {As[i], W, Ys[i], Ms[i], N, K, (Ms[i] + BM - 1) / BM, (N + BN - 1) / BN, 0};
    a.p[i].tiles = a.p[i].mtiles * a.p[i].ntiles;
    grid += a.p[i].tiles;
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i)
    hipLaunchKernelGGL((gemm_v<BM, BN, BK, WM, WN>), dim3(grid), dim3(64 * WM * WN), 0, 0, a);
  CHECK(hipEventRecord(e0));
  const int reps = 50;
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((gemm_v<BM, BN, BK, WM, WN>), dim3(grid), dim3(64 * WM * WN), 0, 0, a);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  const double flop = 2.0 * 5120 * N * K;
  printf("%-28s N=%4d K=%4d grid=%5d  %8.2f us  %6.1f TF/s\n", name, N, K, grid, us,
         flop / us * 1e-6);
}

int main() {
  float *A2, *A3, *W, *Y2, *Y3;
  CHECK(hipMalloc(&A2, 1024 * 512 * 4));
  CHECK(hipMalloc(&A3, 4096 * 512 * 4));
  CHECK(hipMalloc(&W, 768 * 512 * 4));
  CHECK(hipMalloc(&Y2, 1024 * 768 * 4));
  CHECK(hipMalloc(&Y3, 4096 * 768 * 4));
  std::vector<float> h(4096 * 768);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  CHECK(hipMemcpy(A2, h.data(), 1024 * 512 * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(A3, h.data(), 4096 * 512 * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(W, h.data(), 768 * 512 * 4, hipMemcpyHostToDevice));
  const int shapes[4][2] = {{768, 256}, {256, 256}, {512, 512}, {256, 512}};
  for (auto& s : shapes) {
    const int N = s[0], K = s[1];
    run<64, 64, 32, 2, 2>("64x64x32 w2x2", A2, A3, W, Y2, Y3, N, K);
    run<64, 64, 64, 2, 2>("64x64x64 w2x2", A2, A3, W, Y2, Y3, N, K);
    run<128, 64, 32, 2, 2>("128x64x32 w2x2", A2, A3, W, Y2, Y3, N, K);
    run<64, 128, 32, 2, 2>("64x128x32 w2x2", A2, A3, W, Y2, Y3, N, K);
    run<128, 128, 32, 2, 2>("128x128x32 w2x2", A2, A3, W, Y2, Y3, N, K);
    run<128, 64, 32, 4, 2>("128x64x32 w4x2", A2, A3, W, Y2, Y3, N, K);
    run<64, 128, 32, 2, 4>("64x128x32 w2x4", A2, A3, W, Y2, Y3, N, K);
    run<32, 64, 64, 1, 2>("32x64x64 w1x2", A2, A3, W, Y2, Y3, N, K);
    run<32, 32, 64, 1, 1>("32x32x64 w1x1", A2, A3, W, Y2, Y3, N, K);
    run<64, 32, 64, 2, 1>("64x32x64 w2x1", A2, A3, W, Y2, Y3, N, K);
    printf("\n");
  }
  return 0;
}
