// Dev tool (not shipped): is v_mfma_f32_16x16x4_f32 with a permuted k assignment bit-identical to
// the production v_mfma_f32_32x32x2_f32 sequence (gemm.hip: within each 8-deep group, MFMA j takes
// k = 8 kk + j from lane half 0 and 8 kk + 4 + j from lane half 1)?  Both are compared with a CPU
// fmaf chain in the order 0, 4, 1, 5, 2, 6, 3, 7 of every 8-group.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -w tools/mfma_order.hip -o tools/mfma_order
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int K = 512;

// D[r][c] = sum_k A[r][k] * W[c][k], 32 x 32, one wave
__global__ void k32(const float* A, const float* W, float* D) {
  const int l = threadIdx.x;
  floatx16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  for (int kk = 0; kk < K / 8; ++kk)
    for (int j = 0; j < 4; ++j) {
      const int k = 8 * kk + 4 * (l >> 5) + j;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[(l & 31) * K + k], W[(l & 31) * K + k], acc, 0, 0, 0);
    }
  for (int i = 0; i < 16; ++i) {
    const int r = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5);
    D[r * 32 + (l & 31)] = acc[i];
  }
}

__global__ void k16(const float* A, const float* W, float* D) {
  const int l = threadIdx.x, g = l >> 4;
  const int pat[2][4] = {{0, 4, 1, 5}, {2, 6, 3, 7}};
  for (int rb = 0; rb < 2; ++rb)
    for (int cb = 0; cb < 2; ++cb) {
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int kk = 0; kk < K / 8; ++kk)
        for (int m = 0; m < 2; ++m) {
          const int k = 8 * kk + pat[m][g];
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[(16 * rb + (l & 15)) * K + k],
                                                     W[(16 * cb + (l & 15)) * K + k], acc, 0, 0, 0);
        }
      for (int v = 0; v < 4; ++v) D[(16 * rb + 4 * g + v) * 32 + 16 * cb + (l & 15)] = acc[v];
    }
}

static float rnd(unsigned& s) {
  s = s * 1664525u + 1013904223u;
  const float u = (float)((s >> 8) & 0xffffff) / 16777216.f - 0.5f;
  s = s * 1664525u + 1013904223u;
  const int e = (int)((s >> 24) % 9) - 4;
  return ldexpf(u, e);
}

int main() {
  std::vector<float> A(32 * K), W(32 * K), D32(1024), D16(1024), C(1024), C2(1024);
  unsigned s = 12345u;
  for (auto& x : A) x = rnd(s);
  for (auto& x : W) x = rnd(s);
  const int ord[8] = {0, 4, 1, 5, 2, 6, 3, 7};
  for (int r = 0; r < 32; ++r)
    for (int c = 0; c < 32; ++c) {
      float acc = 0.f, acc2 = 0.f;
      for (int kk = 0; kk < K / 8; ++kk)
        for (int j = 0; j < 8; ++j) {
          const int k = 8 * kk + ord[j];
          acc = fmaf(A[r * K + k], W[c * K + k], acc);
        }
      for (int k = 0; k < K; ++k) acc2 = fmaf(A[r * K + k], W[c * K + k], acc2);
      C[r * 32 + c] = acc;
      C2[r * 32 + c] = acc2;
    }
  float *dA, *dW, *dD;
  hipMalloc(&dA, A.size() * 4);
  hipMalloc(&dW, W.size() * 4);
  hipMalloc(&dD, 4096);
  hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dW, W.data(), W.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, dA, dW, dD);
  hipMemcpy(D32.data(), dD, 4096, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, dA, dW, dD);
  hipMemcpy(D16.data(), dD, 4096, hipMemcpyDeviceToHost);
  int d32c = 0, d16c = 0, d1632 = 0, d32c2 = 0;
  for (int i = 0; i < 1024; ++i) {
    d32c += memcmp(&D32[i], &C[i], 4) != 0;
    d16c += memcmp(&D16[i], &C[i], 4) != 0;
    d1632 += memcmp(&D16[i], &D32[i], 4) != 0;
    d32c2 += memcmp(&D32[i], &C2[i], 4) != 0;
  }
  printf("mfma_order K=%d: 32x32x2 vs cpu chain(0,4,1,5..) %d/1024 differ; 16x16x4(perm) vs cpu %d; "
         "16x16x4 vs 32x32x2 %d; 32x32x2 vs cpu plain order %d\n",
         K, d32c, d16c, d1632, d32c2);
  return 0;
}
