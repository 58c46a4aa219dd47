// Dev tool (not shipped): time the library's gemm_launch for every epilogue/prologue used by
// a config-2 layer (2D side 1024 tokens + 3D side 4096 tokens in one launch), and the same
// shapes with the plain BIAS epilogue, so epilogue overhead is visible.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gemm_epi_bench.hip -o tools/gemm_epi_bench
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
int main() {
  float *A, *W, *Y, *R, *mean, *rstd, *bias, *stats, *kvp, *ksp, *ksum;
  hipMalloc(&A, 5120 * 512 * 4); hipMalloc(&W, 768 * 512 * 4); hipMalloc(&Y, 5120 * 768 * 4);
  hipMalloc(&R, 5120 * 768 * 4); hipMalloc(&mean, 2 * 512 * 4); hipMalloc(&rstd, 2 * 512 * 4);
  hipMalloc(&bias, 768 * 4); hipMalloc(&stats, 2 * 160 * 1024 * 4);
  hipMalloc(&kvp, 160 * 16384 * 4); hipMalloc(&ksp, 160 * 256 * 4); hipMalloc(&ksum, 2 * 256 * 4);
  std::vector<float> h(5120 * 768, 0.01f);
  hipMemcpy(A, h.data(), 5120 * 512 * 4, hipMemcpyHostToDevice);
  hipMemcpy(W, h.data(), 768 * 512 * 4, hipMemcpyHostToDevice);
  hipMemcpy(mean, h.data(), 1024 * 4, hipMemcpyHostToDevice);
  hipMemcpy(rstd, h.data(), 1024 * 4, hipMemcpyHostToDevice);
  hipMemcpy(ksum, h.data(), 512 * 4, hipMemcpyHostToDevice);
  struct Case { const char* name; int epi, pro, tile, N, K; };
  Case cases[] = {{"qkv  QKV/32x128", EPI_QKV, PRO_PLAIN, TILE_32x128, 768, 256},
                  {"q    BIAS/64x64", EPI_BIAS, PRO_PLAIN, TILE_64x64, 256, 256},
                  {"mlp1 STATS+HEADZ/64x64", EPI_STATS, PRO_HEADZ, TILE_64x64, 512, 512},
                  {"mlp1 BIAS/64x64", EPI_BIAS, PRO_PLAIN, TILE_64x64, 512, 512},
                  {"mlp2 RESID+NORM/64x64", EPI_RESID, PRO_NORM_RELU, TILE_64x64, 256, 512},
                  {"mlp2 BIAS/64x64", EPI_BIAS, PRO_PLAIN, TILE_64x64, 256, 512}};
  for (auto& c : cases) {
    GemmArgs a;
    a.nprob = 2;
    const int Ms[2] = {1024, 4096};
    for (int i = 0; i < 2; ++i) {
      GemmProb& g = a.p[i];
      memset(&g, 0, sizeof(g));
      g.A0 = A + (i ? 1024 * c.K : 0); g.lda0 = c.K; g.ksplit = c.K; g.W = W; g.ldw = c.K;
      g.bias = bias; g.Y = Y + (i ? 1024 * c.N : 0); g.ldy = c.N; g.R = R + (i ? 1024 * c.N : 0);
      g.ldr = c.N; g.pro_mean = mean + i * 512; g.pro_rstd = rstd + i * 512; g.stats = stats + i * 160 * 1024;
      g.kvpart = kvp + (i ? 32 * 16384 : 0); g.kspart = ksp + (i ? 32 * 256 : 0);
      g.ksum = ksum + i * 256;
      g.M = Ms[i]; g.N = c.N; g.K = c.K; g.batch = 1; g.scale = 1; g.vdiv = 1; g.ns = 1;
      if (c.pro == PRO_HEADZ) {   // [x | phi(q)] = the two halves of one A row
        g.ksplit = 256; g.A1 = g.A0 + 256; g.lda1 = c.K; g.a1_bs = 0;
      }
    }
    for (int i = 0; i < 5; ++i) gemm_launch(c.epi, c.pro, c.tile, a, 0, 0);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int i = 0; i < 50; ++i) gemm_launch(c.epi, c.pro, c.tile, a, 0, 0);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-26s %8.2f us  %6.1f TF/s\n", c.name, ms * 1e3 / 50, 2.0 * 5120 * c.N * c.K / (ms * 1e3 / 50) * 1e-6);
  }
  // single launches separated by a sync: the per-launch time the pipeline actually sees
  for (auto& c : cases) {
    (void)c;
  }
}
