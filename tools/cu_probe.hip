// Dev tool (not shipped): per-workgroup timeline of the library's mlp1 GEMM (64x64 tiles,
// config-2 shape): CU id (XCC_ID, HW_ID[15:8]), start and end on the device clock.
// Prints the workgroups-per-CU histogram, start-time spread and workgroup durations.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -w tools/cu_probe.hip -o tools/cu_probe
#include "../onepose_amd/csrc/gemm.hip"
#include <algorithm>
#include <cstdarg>
#include <cstring>
#include <map>
#include <vector>
namespace onepose {
void set_error(const char* fmt, ...) { va_list ap; va_start(ap, fmt); vprintf(fmt, ap); va_end(ap); printf("\n"); }
void clear_error() {}
void prof_pre(int, hipStream_t) {}
void prof_post(int, hipStream_t) {}
StampAcc* prof_stamp_slot(int) { return nullptr; }
}
using namespace onepose;

struct Rec { unsigned long long t0, t1; unsigned cu; unsigned pad; unsigned long long c0, c1; };

template <int EPI, int PRO, class T>
__global__ __launch_bounds__(256) void timed_gemm(GemmArgs args, Rec* rec) {
  const unsigned long long t0 = (unsigned long long)wall_clock64();
  const unsigned long long c0 = (unsigned long long)clock64();
  gemm_body<EPI, PRO, T>(args);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    const unsigned long long c1 = (unsigned long long)clock64();
    rec[blockIdx.x] = {t0, (unsigned long long)wall_clock64(), ((xcc & 15) << 8) | ((hw >> 8) & 0xff), 0,
                       c0, c1};
  }
}

template <int EPI, int PRO, class T>
void run(const char* name, int N, int K, int tile) {
  float *A, *W, *Y, *bias, *stats, *R, *mean, *rstd;
  hipMalloc(&A, 5120 * 512 * 4); hipMalloc(&W, 512 * 512 * 4); hipMalloc(&Y, 5120 * 512 * 4);
  hipMalloc(&R, 5120 * 512 * 4); hipMalloc(&mean, 1024 * 4); hipMalloc(&rstd, 1024 * 4);
  hipMalloc(&bias, 512 * 4); hipMalloc(&stats, 2 * 160 * 1024 * 4);
  hipMemset(A, 0, 5120 * 512 * 4); hipMemset(W, 0, 512 * 512 * 4);
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.nprob = 2;
  const int Ms[2] = {1024, 4096};
  const int bm = gemm_tile_rows(tile);
  int grid = 0;
  for (int i = 0; i < 2; ++i) {
    GemmProb& g = a.p[i];
    g = gemm_prob(A + (i ? 1024 * K : 0), K, W, K, bias, Y + (i ? 1024 * N : 0), N, Ms[i], N, K, 1);
    g.R = R; g.ldr = N; g.pro_mean = mean; g.pro_rstd = rstd; g.stats = stats + i * 160 * 1024;
    g.mtiles = (Ms[i] + bm - 1) / bm; g.ntiles = N / T::BN; g.tiles = g.mtiles * g.ntiles;
    grid += g.tiles;
  }
  Rec* rec;
  hipMalloc(&rec, grid * sizeof(Rec));
  for (int it = 0; it < 6; ++it)
    hipLaunchKernelGGL((timed_gemm<EPI, PRO, T>), dim3(grid), dim3(256), 0, 0, a, rec);
  hipDeviceSynchronize();
  std::vector<Rec> h(grid);
  hipMemcpy(h.data(), rec, grid * sizeof(Rec), hipMemcpyDeviceToHost);
  int khz = 0;
  hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
  const double us = 1e3 / khz;
  unsigned long long t_min = ~0ull, t_max = 0;
  for (auto& r : h) { t_min = std::min(t_min, r.t0); t_max = std::max(t_max, r.t1); }
  std::map<unsigned, std::vector<Rec>> per_cu;
  for (auto& r : h) per_cu[r.cu].push_back(r);
  std::map<int, int> hist;
  for (auto& kv : per_cu) hist[(int)kv.second.size()]++;
  std::vector<double> dur, st;
  for (auto& r : h) { dur.push_back((r.t1 - r.t0) * us); st.push_back((r.t0 - t_min) * us); }
  double fsum = 0;
  for (auto& r : h) fsum += (double)(r.c1 - r.c0) / ((r.t1 - r.t0) * us);   // cycles per us
  printf("   shader clock %.0f MHz (s_memtime / s_memrealtime over the workgroups)\n", fsum / h.size());
  std::sort(dur.begin(), dur.end());
  std::sort(st.begin(), st.end());
  printf("%s grid %d: span %.2f us, %zu CUs, WGs/CU:", name, grid, (t_max - t_min) * us, per_cu.size());
  for (auto& kv : hist) printf(" %dx%d", kv.second, kv.first);
  printf("\n   WG dur us p0 %.2f p50 %.2f p90 %.2f max %.2f | start us p50 %.2f p90 %.2f max %.2f\n",
         dur[0], dur[dur.size() / 2], dur[dur.size() * 9 / 10], dur.back(), st[st.size() / 2],
         st[st.size() * 9 / 10], st.back());
  // busiest CU: its WGs' spans
  unsigned long long worst = 0; unsigned wcu = 0;
  for (auto& kv : per_cu) {
    unsigned long long e = 0;
    for (auto& r : kv.second) e = std::max(e, r.t1);
    if (e > worst) { worst = e; wcu = kv.first; }
  }
  printf("   last CU %03x:", wcu);
  for (auto& r : per_cu[wcu]) printf(" [%.1f-%.1f]", (r.t0 - t_min) * us, (r.t1 - t_min) * us);
  printf("\n");
}

int main() {
  run<EPI_BIAS, PRO_PLAIN, T64x64>("mlp1 BIAS 64x64", 512, 512, TILE_64x64);
  run<EPI_STATS, PRO_PLAIN, T64x64>("mlp1 STATS 64x64", 512, 512, TILE_64x64);
  run<EPI_RESID, PRO_NORM_RELU, T64x64>("mlp2 RESID 64x64", 256, 512, TILE_64x64);
  run<EPI_BIAS, PRO_PLAIN, T64x64>("q BIAS 64x64", 256, 256, TILE_64x64);
  return 0;
}
