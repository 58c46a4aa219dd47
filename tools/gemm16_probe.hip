// Dev tool (not shipped): an fp32 GEMM main loop on v_mfma_f32_16x16x4_f32 with large
// per-wave tiles (the shape hipBLASLt picks for these sizes: MT128x128x32, MI16x16, 64x64 per
// wave), timed on the matcher's GEMM shapes against the production kernel's alone times.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gemm16_probe.hip -o tools/gemm16_probe
//
// Y[m][n] = sum_k A[m][k] W[n][k] + bias[n].  Workgroup: WMW x WNW waves, wave tile
// (BM / WMW) x (BN / WNW) of 16x16 blocks.  K in stages of 32 through double-buffered LDS
// images [row][36]; one ds_read_b128 per operand block feeds four MFMAs: lane group g = l >> 4
// carries k = 16 q + 4 g + j into MFMA j of 16-deep group q (a re-ordering of the k sum).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int BM_, int BN_, int WMW_, int WNW_>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, WMW = WMW_, WNW = WNW_;
  static constexpr int NW = WMW * WNW, NT = 64 * NW;
  static constexpr int TM = BM / WMW / 16, TN = BN / WNW / 16;   // 16x16 blocks per wave
  static constexpr int BK = 32, PITCH = 36;
  static constexpr int A4 = BM * (BK / 4) / NT, W4 = BN * (BK / 4) / NT;   // float4 per thread
  static constexpr int STAGE = (BM + BN) * PITCH;
  static_assert(A4 >= 1 && W4 >= 1 && TM >= 1 && TN >= 1, "shape");
};

template <class C>
struct StageT {
  float4 a[C::A4], w[C::W4];
};
template <class C>
struct FragT {
  floatx4 a[C::TM], w[C::TN];
};

__device__ __forceinline__ int xcd_contig(int bid, int grid) {
  const int xcd = bid & 7, idx = bid >> 3;
  const int per = grid >> 3, rem = grid & 7;
  return xcd < rem ? xcd * (per + 1) + idx : rem * (per + 1) + (xcd - rem) * per + idx;
}

template <class C>
__global__ __launch_bounds__(C::NT) __attribute__((amdgpu_waves_per_eu(1, 2))) void g16_kernel(const float* __restrict__ A,
                                                    const float* __restrict__ W,
                                                    const float* __restrict__ bias,
                                                    float* __restrict__ Y, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) float lds[2 * C::STAGE];
  const int ntn = (N + C::BN - 1) / C::BN;
  const int bid = xcd_contig(blockIdx.x, gridDim.x);
  const int mt = bid / ntn, nt = bid - mt * ntn;
  const int m0 = mt * C::BM, n0 = nt * C::BN;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave / C::WNW, wn = wave % C::WNW;
  const int g = lane >> 4, r16 = lane & 15;

  floatx4 acc[C::TM][C::TN];
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = (floatx4)(0.f);

  using Stage = StageT<C>;
  auto load = [&](int k0, Stage& s) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < C::A4; ++i) {
      const int e = t + C::NT * i, row = min(m0 + e / 8, M - 1), kq = (e % 8) * 4;
      s.a[i] = *reinterpret_cast<const float4*>(A + (int64_t)row * K + k0 + kq);
    }
#pragma unroll
    for (int i = 0; i < C::W4; ++i) {
      const int e = t + C::NT * i, row = min(n0 + e / 8, N - 1), kq = (e % 8) * 4;
      s.w[i] = *reinterpret_cast<const float4*>(W + (int64_t)row * K + k0 + kq);
    }
  };
  auto store = [&](float* buf, const Stage& s) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < C::A4; ++i) {
      const int e = t + C::NT * i;
      *reinterpret_cast<float4*>(buf + (e / 8) * C::PITCH + (e % 8) * 4) = s.a[i];
    }
#pragma unroll
    for (int i = 0; i < C::W4; ++i) {
      const int e = t + C::NT * i;
      *reinterpret_cast<float4*>(buf + (C::BM + e / 8) * C::PITCH + (e % 8) * 4) = s.w[i];
    }
  };
  using Frag = FragT<C>;
  const int aoff = (wm * C::TM * 16 + r16) * C::PITCH + 4 * g;
  const int woff = (C::BM + wn * C::TN * 16 + r16) * C::PITCH + 4 * g;
  auto frag = [&](const float* buf, int q, Frag& f) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
      f.a[i] = *reinterpret_cast<const floatx4*>(buf + aoff + i * 16 * C::PITCH + 16 * q);
#pragma unroll
    for (int j = 0; j < C::TN; ++j)
      f.w[j] = *reinterpret_cast<const floatx4*>(buf + woff + j * 16 * C::PITCH + 16 * q);
  };
  auto mma = [&](const Frag& f) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < C::TM; ++i)
#pragma unroll
        for (int j = 0; j < C::TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[i][s], f.w[j][s], acc[i][j], 0, 0, 0);
        }
  };

  const int nk = K / C::BK;
  Stage s0, s1;
  Frag f0, f1;
  load(0, s0);
  load(C::BK, s1);
  store(lds, s0);
  __syncthreads();
  frag(lds, 0, f0);
  // two steps per iteration with fixed register roles (a runtime-selected Stage reference
  // would put both stages in scratch); nk is even
  auto step = [&](int kt, Stage& next, Stage& spare) __attribute__((always_inline)) {
    float* cur = lds + (kt & 1) * C::STAGE;
    float* nxt = lds + ((kt + 1) & 1) * C::STAGE;
    load(min(kt + 2, nk - 1) * C::BK, spare);
    frag(cur, 1, f1);
    mma(f0);                                   // group 0 of stage kt
    store(nxt, next);                          // (unused after the last step)
    __syncthreads();
    frag(nxt, 0, f0);
    mma(f1);                                   // group 1 of stage kt
  };
  for (int kt = 0; kt < nk; kt += 2) {
    step(kt, s1, s0);
    step(kt + 1, s0, s1);
  }
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      const int col = n0 + wn * C::TN * 16 + j * 16 + r16;
      const float bb = col < N ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * C::TM * 16 + i * 16 + 4 * g + r;
        if (row < M && col < N) Y[(int64_t)row * N + col] = acc[i][j][r] + bb;
      }
    }
}

template <class C>
float run(const float* A, const float* W, const float* b, float* Y, int M, int N, int K, int it) {
  const int grid = ((M + C::BM - 1) / C::BM) * ((N + C::BN - 1) / C::BN);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(g16_kernel<C>, dim3(grid), dim3(C::NT), 0, 0, A, W, b, Y, M, N, K);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  for (int i = 0; i < it; ++i)
    hipLaunchKernelGGL(g16_kernel<C>, dim3(grid), dim3(C::NT), 0, 0, A, W, b, Y, M, N, K);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / it;
}

template <class C>
void check(const char* name) {
  const int M = 300, N = 200, K = 128;
  std::vector<float> a(M * K), w(N * K), b(N), y(M * N);
  for (auto& v : a) v = (float)(rand() % 17 - 8);
  for (auto& v : w) v = (float)(rand() % 13 - 6);
  for (auto& v : b) v = (float)(rand() % 5);
  float *dA, *dW, *dB, *dY;
  (void)hipMalloc(&dA, a.size() * 4);
  (void)hipMalloc(&dW, w.size() * 4);
  (void)hipMalloc(&dB, b.size() * 4);
  (void)hipMalloc(&dY, y.size() * 4);
  (void)hipMemcpy(dA, a.data(), a.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dW, w.data(), w.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, b.data(), b.size() * 4, hipMemcpyHostToDevice);
  const int grid = ((M + C::BM - 1) / C::BM) * ((N + C::BN - 1) / C::BN);
  hipLaunchKernelGGL(g16_kernel<C>, dim3(grid), dim3(C::NT), 0, 0, dA, dW, dB, dY, M, N, K);
  (void)hipMemcpy(y.data(), dY, y.size() * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int m = 0; m < M; ++m)
    for (int n = 0; n < N; ++n) {
      double s = b[n];
      for (int k = 0; k < K; ++k) s += (double)a[m * K + k] * w[n * K + k];
      if (std::fabs(s - y[m * N + n]) > 1e-3) ++bad;
    }
  printf("check %-10s %s (%d bad)\n", name, bad ? "FAIL" : "ok", bad);
  (void)hipFree(dA); (void)hipFree(dW); (void)hipFree(dB); (void)hipFree(dY);
}

int main() {
  check<Cfg<128, 128, 2, 2>>("128x128");
  check<Cfg<64, 64, 2, 2>>("64x64");
  check<Cfg<128, 64, 2, 2>>("128x64");
  check<Cfg<64, 128, 2, 2>>("64x128");
  const int MM = 8192, KK = 4096;
  float *A, *W, *B, *Y;
  (void)hipMalloc(&A, (size_t)MM * 512 * 4);
  (void)hipMalloc(&W, (size_t)KK * 512 * 4);
  (void)hipMalloc(&B, KK * 4);
  (void)hipMalloc(&Y, (size_t)MM * KK * 4);
  std::vector<float> h((size_t)KK * 512);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
  (void)hipMemcpy(A, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(W, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemset(B, 0, KK * 4);
  struct Shape { const char* name; int M, N, K; };
  const Shape shapes[] = {{"qkv 5120x768x256", 5120, 768, 256}, {"mlp1 5120x512x512", 5120, 512, 512},
                          {"mlp2 5120x256x512", 5120, 256, 512}, {"score 1024x4096x256", 1024, 4096, 256}};
  for (const Shape& s : shapes) {
    const double fl = 2.0 * s.M * s.N * s.K;
    const float t1 = run<Cfg<128, 128, 2, 2>>(A, W, B, Y, s.M, s.N, s.K, 100);
    const float t2 = run<Cfg<64, 64, 2, 2>>(A, W, B, Y, s.M, s.N, s.K, 100);
    const float t3 = run<Cfg<128, 64, 2, 2>>(A, W, B, Y, s.M, s.N, s.K, 100);
    const float t4 = run<Cfg<64, 128, 2, 2>>(A, W, B, Y, s.M, s.N, s.K, 100);
    const float t5 = run<Cfg<64, 32, 2, 2>>(A, W, B, Y, s.M, s.N, s.K, 100);
    printf("%-22s 128x128 %6.2f us (%5.1f TF/s) | 64x64 %6.2f (%5.1f) | 128x64 %6.2f (%5.1f) | 64x128 %6.2f (%5.1f) | 64x32 %6.2f (%5.1f)\n",
           s.name, t1, fl / t1 * 1e-6, t2, fl / t2 * 1e-6, t3, fl / t3 * 1e-6, t4, fl / t4 * 1e-6, t5, fl / t5 * 1e-6);
  }
  return 0;
}
