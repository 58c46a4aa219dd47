// Dev tool (not shipped): LDS-free fp32 MFMA GEMM experiment.  Every wave streams its own
// MFMA operand fragments from global memory (L1/L2) straight into a register ring of D
// 8-deep k-groups, so the main loop has no LDS traffic and no workgroup barrier; waves of a
// workgroup that share A rows / W rows meet in the CU's L1.  Fragment k-order is the
// production kernel's (lane half h carries k = 8 g + 4 h + j into MFMA j), so the output is
// bit-identical to gemm_kernel's.  Compared against the production 64x64 LDS-staged tile on
// the config-2 mlp1 / mlp2 / qkv shapes (5120 tokens).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -w tools/gemm_direct.hip -o tools/gemm_direct
#include "../onepose_amd/csrc/gemm.hip"
#include <cstdarg>
#include <cstring>
#include <vector>
namespace onepose {
void set_error(const char* fmt, ...) { va_list ap; va_start(ap, fmt); vprintf(fmt, ap); va_end(ap); printf("\n"); }
void clear_error() {}
void prof_pre(int, hipStream_t) {}
void prof_post(int, hipStream_t) {}
StampAcc* prof_stamp_slot(int) { return nullptr; }
}
using namespace onepose;

typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int WM, int WN, int FN, int D>
__global__ __launch_bounds__(64 * WM * WN) void gemm_direct(const float* __restrict__ A, int lda,
                                                           const float* __restrict__ W, int ldw,
                                                           const float* __restrict__ bias,
                                                           float* __restrict__ Y, int ldy, int M,
                                                           int N, int K, int ntiles) {
  constexpr int BM = 32 * WM, BN = 32 * FN * WN;
  const int bid = xcd_contiguous(blockIdx.x, gridDim.x);
  const int mt = bid / ntiles, nt = bid - mt * ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int kh = (lane >> 5) * 4;
  const float* pa = A + (int64_t)min(m0 + wm * 32 + (lane & 31), M - 1) * lda + kh;
  const float* pw[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j)
    pw[j] = W + (int64_t)min(n0 + (wn * FN + j) * 32 + (lane & 31), N - 1) * ldw + kh;

  floatx16 acc[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;

  const int ng = K / 8;   // 8-deep k-groups (K % (8 D) == 0)
  float4 ra[D], rw[D][FN];
#pragma unroll
  for (int s = 0; s < D; ++s) {
    ra[s] = *reinterpret_cast<const float4*>(pa + s * 8);
#pragma unroll
    for (int j = 0; j < FN; ++j) rw[s][j] = *reinterpret_cast<const float4*>(pw[j] + s * 8);
  }
  for (int g0 = 0; g0 < ng; g0 += D) {
#pragma unroll
    for (int s = 0; s < D; ++s) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[s].x, rw[s][j].x, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[s].y, rw[s][j].y, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[s].z, rw[s][j].z, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[s].w, rw[s][j].w, acc[j], 0, 0, 0);
      }
      // refill this slot with group g0 + s + D (past the end: re-read the last group)
      const int gn = min(g0 + s + D, ng - 1) * 8;
      ra[s] = *reinterpret_cast<const float4*>(pa + gn);
#pragma unroll
      for (int j = 0; j < FN; ++j) rw[s][j] = *reinterpret_cast<const float4*>(pw[j] + gn);
    }
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int gn = n0 + (wn * FN + j) * 32 + (lane & 31);
    const float b = gn < N ? bias[gn] : 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int gm = m0 + wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
      if (gm < M && gn < N) Y[(int64_t)gm * ldy + gn] = acc[j][i] + b;
    }
  }
}

static float time_ref(float* A, float* W, float* Y, float* bias, int N, int K, int iters,
                      int m0 = 1024, int m1 = 4096) {
  using T = Tile<64, 64, 1, 4, 32>;
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.nprob = 2;
  const int Ms[2] = {m0, m1};
  int grid = 0;
  for (int i = 0; i < 2; ++i) {
    GemmProb& p = a.p[i];
    p = gemm_prob(A + (i ? (int64_t)1024 * K : 0), K, W, K, bias, Y + (i ? (int64_t)1024 * N : 0),
                  N, Ms[i], N, K, 1);
    p.mtiles = (Ms[i] + T::BM - 1) / T::BM;
    p.ntiles = (N + T::BN - 1) / T::BN;
    p.tiles = p.mtiles * p.ntiles;
    grid += p.tiles;
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) launch_one<EPI_BIAS, PRO_PLAIN, T, false>(a, grid, nullptr);
  hipEventRecord(e0);
  for (int it = 0; it < iters; ++it) launch_one<EPI_BIAS, PRO_PLAIN, T, false>(a, grid, nullptr);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / iters;
}

template <int WM, int WN, int FN, int D>
static float time_direct(float* A, float* W, float* Y, float* bias, int N, int K, int iters) {
  constexpr int BM = 32 * WM, BN = 32 * FN * WN;
  const int M = 5120, mt = (M + BM - 1) / BM, nt = (N + BN - 1) / BN;
  auto go = [&]() {
    hipLaunchKernelGGL((gemm_direct<WM, WN, FN, D>), dim3(mt * nt), dim3(64 * WM * WN), 0, 0, A, K,
                       W, K, bias, Y, N, M, N, K, nt);
  };
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) go();
  hipEventRecord(e0);
  for (int it = 0; it < iters; ++it) go();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / iters;
}

static const int kShapes[3][2] = {{512, 512}, {256, 512}, {768, 256}};   // (N, K)

template <int WM, int WN, int FN, int D>
static void row(const char* name, float* A, float* W, float* Y, float* Yr, float* bias) {
  printf("%-36s", name);
  for (auto& sh : kShapes) {
    const int N = sh[0], K = sh[1];
    if (K % (8 * D)) {
      printf("        -          ");
      continue;
    }
    const float us = time_direct<WM, WN, FN, D>(A, W, Y, bias, N, K, 50);
    time_ref(A, W, Yr, bias, N, K, 1);
    hipDeviceSynchronize();
    std::vector<float> a((size_t)5120 * N), b((size_t)5120 * N);
    hipMemcpy(a.data(), Y, a.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(b.data(), Yr, b.size() * 4, hipMemcpyDeviceToHost);
    size_t diff = 0;
    for (size_t i = 0; i < a.size(); ++i) diff += a[i] != b[i];
    printf(" %7.2f us %5.1fTF%s", us, 2.0 * 5120 * N * K / us * 1e-6, diff ? "!" : " ");
  }
  printf("\n");
}

int main() {
  float *A, *W, *Y, *Yr, *bias;
  hipMalloc(&A, 16384 * 512 * 4);
  hipMalloc(&W, 768 * 512 * 4);
  hipMalloc(&Y, 5120 * 768 * 4);
  hipMalloc(&Yr, 16384 * 768 * 4);
  hipMalloc(&bias, 768 * 4);
  std::vector<float> h(5120 * 512);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
  hipMemcpy(A, h.data(), 5120 * 512 * 4, hipMemcpyHostToDevice);
  hipMemcpy(W, h.data(), 768 * 512 * 4, hipMemcpyHostToDevice);
  hipMemset(bias, 0, 768 * 4);
  printf("%-36s %-19s %-19s %-19s\n", "variant", "mlp1 512x512", "mlp2 256x512", "qkv 768x256");
  printf("%-36s", "LDS 64x64 4w (production)");
  for (auto& sh : kShapes) {
    const float us = time_ref(A, W, Yr, bias, sh[0], sh[1], 50);
    printf(" %7.2f us %5.1fTF ", us, 2.0 * 5120 * sh[0] * sh[1] / us * 1e-6);
  }
  printf("\n");
  // wave quantisation: 64x64 tiles of the mlp1 shape at M = 2048 .. 16384 tokens
  for (int m : {2048, 3072, 4096, 5120, 6144, 8192, 10240, 12288, 16384}) {
    const float us = time_ref(A, W, Yr, bias, 512, 512, 30, 1024, m - 1024);
    printf("mlp1 shape M=%5d tiles=%5d  %7.2f us %5.1f TF  %.3f us/tile-round\n", m, m / 64 * 8, us,
           2.0 * m * 512 * 512 / us * 1e-6, us / ((m / 64 * 8 + 255) / 256));
  }
  row<2, 2, 1, 4>("direct 64x64 2x2w FN1 D4", A, W, Y, Yr, bias);
  row<2, 2, 1, 8>("direct 64x64 2x2w FN1 D8", A, W, Y, Yr, bias);
  row<2, 2, 1, 16>("direct 64x64 2x2w FN1 D16", A, W, Y, Yr, bias);
  row<2, 1, 2, 4>("direct 64x64 2x1w FN2 D4", A, W, Y, Yr, bias);
  row<2, 1, 2, 8>("direct 64x64 2x1w FN2 D8", A, W, Y, Yr, bias);
  row<1, 2, 1, 8>("direct 32x64 1x2w FN1 D8", A, W, Y, Yr, bias);
  row<1, 1, 2, 8>("direct 32x64 1w FN2 D8", A, W, Y, Yr, bias);
  row<2, 2, 2, 4>("direct 64x128 2x2w FN2 D4", A, W, Y, Yr, bias);
  row<2, 2, 2, 8>("direct 64x128 2x2w FN2 D8", A, W, Y, Yr, bias);
  row<4, 1, 2, 8>("direct 128x64 4x1w FN2 D8", A, W, Y, Yr, bias);
  row<1, 4, 1, 8>("direct 32x128 1x4w FN1 D8", A, W, Y, Yr, bias);
  return 0;
}
