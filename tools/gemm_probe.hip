// Dev tool (not shipped): what bounds the production 64x64 GEMM loop on the config-2 mlp1
// shape (M = 1024 + 4096, N = 512, K = 512, plain BIAS epilogue): fp32 MFMA vs the exact
// 3-way bf16 split (PM_SPLIT3), each with and without its in-loop global loads
// (ONEPOSE_GEMM_PROBE_NOLOAD: every stage re-stores the first two stages' registers), and
// at 1 / 2 / 3 / 4 tiles per CU (M scaled).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gemm_probe.hip -o tools/gemm_probe
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -DONEPOSE_GEMM_PROBE_NOLOAD tools/gemm_probe.hip -o tools/gemm_probe_noload
#include "../onepose_amd/csrc/gemm.hip"
#include <cstdarg>
#include <cstdlib>
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

template <class T, int PM>
float run(float* A, float* W, float* Y, float* bias, int M0, int M1, int N, int K, int iters) {
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.nprob = 2;
  const int Ms[2] = {M0, M1};
  int grid = 0;
  for (int i = 0; i < 2; ++i) {
    GemmProb& p = a.p[i];
    p = gemm_prob(A, K, W, K, bias, Y, N, Ms[i], N, K, 1);
    p.mtiles = (Ms[i] + T::BM - 1) / T::BM;
    p.ntiles = (N + T::BN - 1) / T::BN;
    p.tiles = p.mtiles * p.ntiles;
    grid += p.tiles;
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) launch_one<EPI_BIAS, PRO_PLAIN, T, PM>(a, grid, nullptr);
  hipEventRecord(e0);
  for (int it = 0; it < iters; ++it) launch_one<EPI_BIAS, PRO_PLAIN, T, PM>(a, grid, nullptr);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / iters;
}

// Clock sampler: one workgroup spins ~40 us reading the shader-clock counter (s_memtime) and
// the 100 MHz real-time counter; their ratio is the core clock of the CU it lands on.
__global__ void clock_sampler(double* out, int i) {
  if (threadIdx.x != 0) return;
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = r0, c1 = c0;
  while (r1 - r0 < 4000) {
    r1 = __builtin_amdgcn_s_memrealtime();
    c1 = __builtin_amdgcn_s_memtime();
  }
  out[i] = (double)(c1 - c0) / (double)(r1 - r0) * 0.1;   // GHz
}

template <class T, int PM>
void clock_under_load(float* A, float* W, float* Y, float* bias) {
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.nprob = 2;
  const int Ms[2] = {1024, 4096};
  int grid = 0;
  for (int i = 0; i < 2; ++i) {
    GemmProb& p = a.p[i];
    p = gemm_prob(A, 512, W, 512, bias, Y, 512, Ms[i], 512, 512, 1);
    p.mtiles = (Ms[i] + T::BM - 1) / T::BM;
    p.ntiles = (512 + T::BN - 1) / T::BN;
    p.tiles = p.mtiles * p.ntiles;
    grid += p.tiles;
  }
  double* d;
  (void)hipMalloc(&d, 64 * sizeof(double));
  hipStream_t s1, s2;
  (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  clock_sampler<<<1, 64, 0, s2>>>(d, 0);   // idle
  (void)hipStreamSynchronize(s2);
  for (int it = 0; it < 400; ++it) launch_one<EPI_BIAS, PRO_PLAIN, T, PM>(a, grid, s1);
  for (int i = 1; i < 16; ++i) clock_sampler<<<1, 64, 0, s2>>>(d, i);
  (void)hipDeviceSynchronize();
  double h[16];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("%-7s clock idle %.3f GHz; under back-to-back mlp1 launches:", PM ? "split3" : "fp32", h[0]);
  for (int i = 1; i < 16; ++i) printf(" %.2f", h[i]);
  printf("\n");
  (void)hipFree(d);
}

template <class T>
void probe(const char* name, float* A, float* W, float* Y, float* bias) {
  const int M1s[3] = {3072, 4096, 7168};   // + 1024 tokens: config-2 mlp1 is M1 = 4096
  for (int pmi = 0; pmi < 2; ++pmi) {
    printf("%-26s %-7s", name, pmi ? "split3" : "fp32");
    for (int mi = 0; mi < 3; ++mi) {
      const int m1 = M1s[mi];
      const float us = pmi == 0 ? run<T, PM_F32>(A, W, Y, bias, 1024, m1, 512, 512, 50)
                                : run<T, PM_SPLIT3>(A, W, Y, bias, 1024, m1, 512, 512, 50);
      printf("  M %5d: %7.2f us %6.1f TF/s", 1024 + m1, us, 2.0 * (1024 + m1) * 512 * 512 / us * 1e-6);
    }
    printf("\n");
  }
}

int main() {
  float *A, *W, *Y, *bias;
  const int MMAX = 4 * 4096 + 1024;
  hipMalloc(&A, (size_t)MMAX * 512 * 4);
  hipMalloc(&W, 768 * 512 * 4);
  hipMalloc(&Y, (size_t)MMAX * 768 * 4);
  hipMalloc(&bias, 768 * 4);
  std::vector<float> h((size_t)MMAX * 512);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
  hipMemcpy(A, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(W, h.data(), 768 * 512 * 4, hipMemcpyHostToDevice);
  hipMemset(bias, 0, 768 * 4);
#ifdef ONEPOSE_GEMM_PROBE_NOLOAD
  printf("in-loop global loads OFF\n");
#else
  printf("in-loop global loads on\n");
#endif
  if (getenv("PROBE_CLOCK")) {
    clock_under_load<Tile<64, 64, 1, 4, 32>, PM_F32>(A, W, Y, bias);
    clock_under_load<Tile<64, 64, 1, 4, 32>, PM_SPLIT3>(A, W, Y, bias);
    return 0;
  }
  {   // the production tile at 1 / 2 / 2.5 (config 2) / 3 / 4 tiles per CU
    using T = Tile<64, 64, 1, 4, 32>;
    const int M1s[5] = {1024, 3072, 4096, 5120, 7168};
    for (int pmi = 0; pmi < 2; ++pmi)
      for (int mi = 0; mi < 5; ++mi) {
        const int m1 = M1s[mi], tiles = (1024 / 64 + m1 / 64) * 8;
        const float us = pmi == 0 ? run<T, PM_F32>(A, W, Y, bias, 1024, m1, 512, 512, 50)
                                  : run<T, PM_SPLIT3>(A, W, Y, bias, 1024, m1, 512, 512, 50);
        printf("64x64 %-7s tiles %5d  %8.2f us  %6.1f TF/s (fp32-equivalent)\n",
               pmi ? "split3" : "fp32", tiles, us, 2.0 * (1024 + m1) * 512 * 512 / us * 1e-6);
      }
  }
  probe<Tile<64, 64, 1, 4, 32>>("64x64 4w (production)", A, W, Y, bias);
  probe<Tile<64, 64, 2, 4, 64>>("64x64 4w K2 FN2 bks64", A, W, Y, bias);
  probe<Tile<64, 64, 1, 2, 32>>("64x64 2w FN2", A, W, Y, bias);
  probe<Tile<64, 128, 1, 4, 32>>("64x128 4w FN2", A, W, Y, bias);
  probe<Tile<64, 64, 2, 8, 64>>("64x64 8w K2 bks64", A, W, Y, bias);
  return 0;
}
