// Dev tool (not shipped): time gemm_body tile shapes on the config-2 mlp1 / mlp2 / qkv GEMM
// shapes with the plain BIAS epilogue (2D side 1024 + 3D side 4096 tokens in one launch).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gemm_tile_sweep.hip -o tools/gemm_tile_sweep
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

template <class T, bool BF>
float run(float* A, float* W, float* Y, float* bias, int N, int K, int iters) {
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.nprob = 2;
  const int Ms[2] = {1024, 4096};
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
  for (int w = 0; w < 3; ++w) launch_one<EPI_BIAS, PRO_PLAIN, T, BF>(a, grid, nullptr);
  hipEventRecord(e0);
  for (int it = 0; it < iters; ++it) launch_one<EPI_BIAS, PRO_PLAIN, T, BF>(a, grid, nullptr);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / iters;   // us per launch
}

template <class T, bool BF = false>
void row(const char* name, float* A, float* W, float* Y, float* bias) {
  const int shapes[3][2] = {{512, 512}, {256, 512}, {768, 256}};   // mlp1, mlp2, qkv (N, K)
  printf("%-34s", name);
  for (auto& sh : shapes) {
    if (sh[1] % (2 * T::BKS)) {
      printf("      -      ");
      continue;
    }
    const float us = run<T, BF>(A, W, Y, bias, sh[0], sh[1], 50);
    printf(" %7.2f us %5.1fTF", us, 2.0 * 5120 * sh[0] * sh[1] / us * 1e-6);
  }
  printf("\n");
}

int main() {
  float *A, *W, *Y, *bias;
  hipMalloc(&A, 5120 * 512 * 4);
  hipMalloc(&W, 768 * 512 * 4);
  hipMalloc(&Y, 5120 * 768 * 4);
  hipMalloc(&bias, 768 * 4);
  std::vector<float> h(5120 * 512);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
  hipMemcpy(A, h.data(), 5120 * 512 * 4, hipMemcpyHostToDevice);
  hipMemcpy(W, h.data(), 768 * 512 * 4, hipMemcpyHostToDevice);
  hipMemset(bias, 0, 768 * 4);
  printf("%-34s %-20s %-20s %-20s\n", "tile (BM,BN,KS,NW,BKS)", "mlp1 512x512", "mlp2 256x512",
         "qkv 768x256");
  row<Tile<64, 64, 1, 4, 32>>("64x64 k1 4w bks32 (current)", A, W, Y, bias);
  row<Tile<64, 64, 1, 4, 32>, true>("64x64 k1 4w bks32 bf16", A, W, Y, bias);
  row<Tile<64, 64, 1, 4, 64>>("64x64 k1 4w bks64", A, W, Y, bias);
  row<Tile<64, 64, 2, 8, 64>>("64x64 k2 8w bks64", A, W, Y, bias);
  row<Tile<64, 128, 1, 4, 32>>("64x128 k1 4w bks32 (FN2)", A, W, Y, bias);
  row<Tile<128, 64, 1, 4, 32>>("128x64 k1 4w bks32 (WN1,FN2)", A, W, Y, bias);
  row<Tile<128, 64, 1, 8, 32>>("128x64 k1 8w bks32", A, W, Y, bias);
  row<Tile<128, 128, 1, 8, 32>>("128x128 k1 8w bks32 (FN2)", A, W, Y, bias);
  row<Tile<32, 64, 1, 2, 32>>("32x64 k1 2w bks32", A, W, Y, bias);
  row<Tile<32, 128, 1, 4, 32>>("32x128 k1 4w bks32", A, W, Y, bias);
  row<Tile<64, 32, 1, 2, 32>>("64x32 k1 2w bks32", A, W, Y, bias);
  row<Tile<32, 64, 2, 4, 64>>("32x64 k2 4w bks64", A, W, Y, bias);
  row<Tile<64, 32, 2, 4, 64>>("64x32 k2 4w bks64", A, W, Y, bias);
  row<Tile<32, 64, 1, 2, 32>>("32x64 k1 2w bks32", A, W, Y, bias);
  row<Tile<64, 64, 2, 8, 64>>("64x64 k2 8w bks64", A, W, Y, bias);
  row<Tile<32, 128, 2, 8, 64>>("32x128 k2 8w bks64", A, W, Y, bias);
  return 0;
}
