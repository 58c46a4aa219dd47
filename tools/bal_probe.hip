// Dev tool (not shipped): gemm_bal.hip's balanced MLP conv 1 against the 64 x 64 kernel on the
// same random inputs (one launch, 1-2 problems, B samples), every output compared bit for bit:
// Y, the per-M-tile (mean, M2) partials, the group partials, mean, rstd.  Reports the first
// mismatches by (problem, sample, row, column).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -w -DONEPOSE_BAL -Ionepose_amd/csrc tools/bal_probe.hip \
//     onepose_amd/csrc/gemm.hip tools/experiments/gemm_bal.hip -o tools/bal_probe
#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <vector>
#include "gemm.h"

namespace onepose {
void set_error(const char* fmt, ...) { va_list ap; va_start(ap, fmt); vprintf(fmt, ap); va_end(ap); printf("\n"); }
void clear_error() {}
void prof_pre(int, hipStream_t) {}
void prof_post(int, hipStream_t) {}
StampAcc* prof_stamp_slot(int) { return nullptr; }
extern bool g_bal_disable;
}
using namespace onepose;

static unsigned g_s = 1;
static float frand() { g_s = g_s * 1664525u + 1013904223u; return (float)((g_s >> 8) / 16777216.0 - 0.5); }
template <class T> T* dup(const std::vector<T>& h) { T* d; hipMalloc(&d, h.size() * sizeof(T)); hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice); return d; }
template <class T> std::vector<T> get(const T* d, size_t n) { std::vector<T> h(n); hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost); return h; }

static bool g_time = false;

struct Prob {
  int M, B; bool acc0;
  float *x, *q, *mf, *ksum, *Y, *stats, *mean, *rstd, *acc; double* grp; unsigned* cnt;
  int cps, ngr;
};

int run(int nprob, const int* Ms, int B, const bool* acc0, bool bal, std::vector<std::vector<float>>* out) {
  g_s = 7;
  std::vector<float> w1a(512 * 256), bias(512);
  for (auto& v : w1a) v = frand() * 0.1f;
  for (auto& v : bias) v = frand();
  float* dw = dup(w1a); float* db = dup(bias);
  GemmArgs a; memset(&a, 0, sizeof(a)); a.nprob = nprob;
  std::vector<Prob> P(nprob);
  for (int i = 0; i < nprob; ++i) {
    Prob& p = P[i]; p.M = Ms[i]; p.B = B; p.acc0 = acc0[i];
    const int M = p.M, mt = (M + 63) / 64;
    std::vector<float> x((size_t)B * M * 256), q((size_t)B * M * 256), mf((size_t)B * 512 * 256), ks((size_t)B * 256);
    for (auto& v : x) v = frand(); for (auto& v : q) v = frand() + 0.6f; for (auto& v : mf) v = frand() * 0.1f; for (auto& v : ks) v = frand() + 0.6f;
    std::vector<float> acc((size_t)B * mt * 8 * 4 * 1024);
    for (auto& v : acc) v = frand();
    p.x = dup(x); p.q = dup(q); p.mf = dup(mf); p.ksum = dup(ks); p.acc = dup(acc);
    hipMalloc(&p.Y, (size_t)B * M * 512 * 4); hipMemset(p.Y, 0, (size_t)B * M * 512 * 4);
    hipMalloc(&p.stats, (size_t)B * mt * 1024 * 4); hipMemset(p.stats, 0, (size_t)B * mt * 1024 * 4);
    p.ngr = stats_groups(M, 64); p.cps = 16 * (1 + p.ngr);
    hipMalloc(&p.grp, (size_t)B * p.ngr * 1024 * 8); hipMemset(p.grp, 0, (size_t)B * p.ngr * 1024 * 8);
    hipMalloc(&p.cnt, (size_t)B * p.cps * 4); hipMemset(p.cnt, 0, (size_t)B * p.cps * 4);
    hipMalloc(&p.mean, (size_t)B * 512 * 4); hipMalloc(&p.rstd, (size_t)B * 512 * 4);
    GemmProb& g = a.p[i];
    g = gemm_prob(p.x, 256, dw, 256, db, p.Y, 512, M, 512, 512, B);
    g.A1 = p.q; g.lda1 = 256; g.a1_bs = (int64_t)M * 256; g.ksplit = 256;
    g.W1 = p.mf; g.ldw1 = 256; g.w1_bs = 512 * 256;
    g.stats = p.stats; g.st_cnt = p.cnt; g.st_cnt_bs = p.cps; g.st_grp = p.grp;
    g.st_mean = p.mean; g.st_rstd = p.rstd; g.ksum = p.ksum; g.ksum_bs = 256; g.ns = 1000.f;
    if (p.acc0) { g.acc0 = p.acc; g.acc0_bs = (int64_t)mt * 8 * 4 * 1024; }
  }
  g_bal_disable = !bal;
  const int rc = gemm_launch(EPI_STATS, PRO_HEADZ, TILE_64x64, a, 0, 0, PM_F32);
  hipDeviceSynchronize();
  if (rc) { printf("launch rc %d\n", rc); return rc; }
  if (g_time) {   // launch time alone: counters re-zeroed between launches (as the forward does)
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e9f, sum = 0.f;
    const int reps = 30;
    for (int r = 0; r < reps + 3; ++r) {
      for (auto& p : P) hipMemsetAsync(p.cnt, 0, (size_t)B * p.cps * 4, 0);
      hipEventRecord(e0, 0);
      gemm_launch(EPI_STATS, PRO_HEADZ, TILE_64x64, a, 0, 0, PM_F32);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (r >= 3) { best = fminf(best, ms); sum += ms; }
    }
    printf("  %s: %.2f us mean, %.2f us best\n", bal ? "balanced" : "64x64", sum / reps * 1e3, best * 1e3);
  }
  for (int i = 0; i < nprob; ++i) {
    Prob& p = P[i]; const int mt = (p.M + 63) / 64;
    out->push_back(get(p.Y, (size_t)B * p.M * 512));
    out->push_back(get(p.stats, (size_t)B * mt * 1024));
    out->push_back(get(p.mean, (size_t)B * 512));
    out->push_back(get(p.rstd, (size_t)B * 512));
  }
  return 0;
}

int main(int argc, char** argv) {
  struct Case { int nprob, M0, M1, B; bool a0, a1; };
  const Case cases[] = {{2, 96, 300, 1, false, false}, {1, 1000, 0, 3, false, false},
                        {2, 200, 777, 2, false, false}, {2, 1024, 4096, 1, false, false},
                        {2, 1024, 4096, 1, false, true}, {1, 40, 0, 1, false, false},
                        {1, 100, 0, 1, false, false}, {1, 64, 0, 1, false, false},
                        {2, 96, 300, 1, false, true}};
  const char* names[] = {"Y", "stats", "mean", "rstd"};
  int bad_total = 0;
  for (const Case& c : cases) {
    const int Ms[2] = {c.M0, c.M1};
    g_time = c.B == 1 && c.M0 == 1024;
    const bool a0[2] = {c.a0, c.a1};
    std::vector<std::vector<float>> o0, o1;
    if (run(c.nprob, Ms, c.B, a0, false, &o0) || run(c.nprob, Ms, c.B, a0, true, &o1)) return 1;
    printf("case nprob %d M %d/%d B %d acc0 %d/%d:", c.nprob, c.M0, c.M1, c.B, c.a0, c.a1);
    for (size_t k = 0; k < o0.size(); ++k) {
      int bad = 0, first = -1;
      for (size_t e = 0; e < o0[k].size(); ++e)
        if (memcmp(&o0[k][e], &o1[k][e], 4) != 0) { if (first < 0) first = (int)e; ++bad; }
      if (bad) {
        const int prob = (int)k / 4, M = Ms[prob];
        printf(" [p%d %s: %d differ, first %d", prob, names[k % 4], bad, first);
        if (k % 4 == 0) printf(" (b %d row %d col %d: %g vs %g)", first / (M * 512), (first / 512) % M, first % 512, o0[k][first], o1[k][first]);
        if (k % 4 == 1) printf(" (mtile-row %d col %d half %d)", first / 1024, first % 512, (first / 512) % 2);
        printf("]");
        bad_total += bad;
      }
    }
    printf(" %s\n", bad_total ? "" : "identical");
  }
  printf("bal_probe: %s\n", bad_total ? "MISMATCH" : "all identical");
  return 0;
}
