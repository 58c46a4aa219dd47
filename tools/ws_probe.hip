// Dev tool (not shipped): bf16 MLP conv 1 (EPI_STATS + PRO_HEADZ, W and A from bf16 planes, the
// DMA-2 loop) on the 256 x 128 eight-wave tile against the 64 x 128 tile it stands in for, on the
// same random inputs (one launch, 1-2 problems, B samples): Y, the per-64-row (mean, M2)
// partials, mean and rstd compared bit for bit; then both timed alone (30 launches, counters
// re-zeroed between launches as the forward does).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -w -Ionepose_amd/csrc tools/ws_probe.hip \
//     onepose_amd/csrc/gemm.hip -o tools/ws_probe
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
}
using namespace onepose;

static unsigned g_s = 1;
static float frand() { g_s = g_s * 1664525u + 1013904223u; return (float)((g_s >> 8) / 16777216.0 - 0.5); }
static uint16_t bf(float x) {   // round to nearest even
  unsigned u; memcpy(&u, &x, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static float unbf(uint16_t h) { unsigned u = (unsigned)h << 16; float x; memcpy(&x, &u, 4); return x; }
template <class T> T* dup(const std::vector<T>& h) { T* d; hipMalloc(&d, h.size() * sizeof(T)); hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice); return d; }
template <class T> std::vector<T> get(const T* d, size_t n) { std::vector<T> h(n); hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost); return h; }

struct Prob {
  int M;
  float *Y, *stats, *mean, *rstd;
  double* grp;
  unsigned* cnt;
  int cps;
};

// one operand in both forms: bf16 planes, and the fp32 values they hold
static void operand(size_t n, float scale, float off, float** f32, uint16_t** b16) {
  std::vector<float> f(n);
  std::vector<uint16_t> h(n);
  for (size_t i = 0; i < n; ++i) { h[i] = bf(frand() * scale + off); f[i] = unbf(h[i]); }
  *f32 = dup(f);
  *b16 = dup(h);
}

int run(int nprob, const int* Ms, int B, const bool* acc0, int tile, int reps, std::vector<std::vector<float>>* out) {
  g_s = 7;
  float *dw, *db, *dummy;
  uint16_t* dwp;
  operand(512 * 256, 0.1f, 0.f, &dw, &dwp);
  {
    std::vector<float> bias(512);
    for (auto& v : bias) v = frand();
    db = dup(bias);
  }
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.nprob = nprob;
  std::vector<Prob> P(nprob);
  for (int i = 0; i < nprob; ++i) {
    Prob& p = P[i];
    p.M = Ms[i];
    const int M = p.M, mt = (M + 63) / 64;
    float *x, *q, *mf, *ksum, *acc;
    uint16_t *xp, *qp, *mfp;
    operand((size_t)B * M * 256, 1.f, 0.f, &x, &xp);
    operand((size_t)B * M * 256, 1.f, 0.6f, &q, &qp);
    operand((size_t)B * 512 * 256, 0.1f, 0.f, &mf, &mfp);
    {
      std::vector<float> ks((size_t)B * 256), ac((size_t)B * mt * 4 * 4 * 2 * 1024);
      for (auto& v : ks) v = frand() + 0.6f;
      for (auto& v : ac) v = frand();
      ksum = dup(ks);
      acc = dup(ac);
    }
    hipMalloc(&p.Y, (size_t)B * M * 512 * 4);
    hipMemset(p.Y, 0, (size_t)B * M * 512 * 4);
    hipMalloc(&p.stats, (size_t)B * mt * 1024 * 4);
    hipMemset(p.stats, 0, (size_t)B * mt * 1024 * 4);
    const int ngr = stats_groups(M, 64);
    p.cps = 4 * (1 + ngr);
    hipMalloc(&p.grp, (size_t)B * ngr * 1024 * 8);
    hipMemset(p.grp, 0, (size_t)B * ngr * 1024 * 8);
    hipMalloc(&p.cnt, (size_t)B * p.cps * 4);
    hipMemset(p.cnt, 0, (size_t)B * p.cps * 4);
    hipMalloc(&p.mean, (size_t)B * 512 * 4);
    hipMalloc(&p.rstd, (size_t)B * 512 * 4);
    GemmProb& g = a.p[i];
    g = gemm_prob(x, 256, dw, 256, db, p.Y, 512, M, 512, 512, B);
    g.A1 = q; g.lda1 = 256; g.a1_bs = (int64_t)M * 256; g.ksplit = 256;
    g.W1 = mf; g.ldw1 = 256; g.w1_bs = 512 * 256;
    g.Wp = dwp; g.wp_bs = 0; g.wpl = 512 * 256;
    g.Wp1 = mfp; g.wp1_bs = 512 * 256; g.wpl1 = 512 * 256;
    g.Ap = xp; g.ap_bs = (int64_t)M * 256; g.apl = (int64_t)M * 256; g.ldap = 256;
    g.Ap1 = qp; g.ap1_bs = (int64_t)M * 256; g.apl1 = (int64_t)M * 256; g.ldap1 = 256;
    g.stats = p.stats; g.st_cnt = p.cnt; g.st_cnt_bs = p.cps; g.st_grp = p.grp;
    g.st_mean = p.mean; g.st_rstd = p.rstd; g.ksum = ksum; g.ksum_bs = 256; g.ns = 1000.f;
    if (acc0[i]) { g.acc0 = acc; g.acc0_bs = (int64_t)mt * 4 * 4 * 2 * 1024; }
  }
  (void)dummy;
  const int rc = gemm_launch(EPI_STATS, PRO_HEADZ, tile, a, 0, 0, PM_BF16);
  hipDeviceSynchronize();
  if (rc) { printf("launch rc %d\n", rc); return rc; }
  if (reps > 0) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e9f, sum = 0.f;
    for (int r = 0; r < reps + 3; ++r) {
      for (auto& p : P) hipMemsetAsync(p.cnt, 0, (size_t)B * p.cps * 4, 0);
      hipEventRecord(e0, 0);
      gemm_launch(EPI_STATS, PRO_HEADZ, tile, a, 0, 0, PM_BF16);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (r >= 3) { best = fminf(best, ms); sum += ms; }
    }
    printf("  %s: %.2f us mean, %.2f us best\n", tile == TILE_256x128W8 ? "256x128w8" : "64x128",
           sum / reps * 1e3, best * 1e3);
  }
  for (int i = 0; i < nprob; ++i) {
    Prob& p = P[i];
    const int mt = (p.M + 63) / 64;
    out->push_back(get(p.Y, (size_t)B * p.M * 512));
    out->push_back(get(p.stats, (size_t)B * mt * 1024));
    out->push_back(get(p.mean, (size_t)B * 512));
    out->push_back(get(p.rstd, (size_t)B * 512));
  }
  return 0;
}

int main() {
  struct Case { int nprob, M0, M1, B; bool a0, a1; int reps; };
  const Case cases[] = {{2, 96, 300, 1, false, false, 0},    {1, 1000, 0, 3, false, false, 0},
                        {2, 200, 777, 2, false, false, 0},   {1, 40, 0, 1, false, false, 0},
                        {1, 64, 0, 1, false, false, 0},      {1, 576, 0, 1, false, false, 0},
                        {2, 96, 300, 1, false, true, 0},     {2, 1000, 2500, 2, false, true, 0},
                        {2, 1024, 4096, 1, false, false, 30}, {2, 1024, 4096, 1, false, true, 30},
                        {2, 2048, 8192, 1, false, false, 30}, {2, 2048, 8192, 1, false, true, 30}};
  const char* names[] = {"Y", "stats", "mean", "rstd"};
  int bad_total = 0;
  for (const Case& c : cases) {
    const int Ms[2] = {c.M0, c.M1};
    const bool a0[2] = {c.a0, c.a1};
    std::vector<std::vector<float>> o0, o1;
    if (c.reps) printf("case nprob %d M %d/%d B %d acc0 %d/%d (timed):\n", c.nprob, c.M0, c.M1, c.B, c.a0, c.a1);
    if (run(c.nprob, Ms, c.B, a0, TILE_64x128, c.reps, &o0) ||
        run(c.nprob, Ms, c.B, a0, TILE_256x128W8, c.reps, &o1))
      return 1;
    printf("case nprob %d M %d/%d B %d acc0 %d/%d:", c.nprob, c.M0, c.M1, c.B, c.a0, c.a1);
    int bad_case = 0;
    for (size_t k = 0; k < o0.size(); ++k) {
      int bad = 0, first = -1;
      for (size_t e = 0; e < o0[k].size(); ++e)
        if (memcmp(&o0[k][e], &o1[k][e], 4) != 0) { if (first < 0) first = (int)e; ++bad; }
      if (bad) {
        const int prob = (int)k / 4, M = Ms[prob];
        printf(" [p%d %s: %d differ, first %d", prob, names[k % 4], bad, first);
        if (k % 4 == 0) printf(" (b %d row %d col %d: %g vs %g)", first / (M * 512), (first / 512) % M, first % 512, o0[k][first], o1[k][first]);
        if (k % 4 == 1) printf(" (mtile %d col %d half %d)", first / 1024, first % 512, (first / 512) % 2);
        printf("]");
        bad_case += bad;
      }
    }
    bad_total += bad_case;
    printf(" %s\n", bad_case ? "" : "identical");
  }
  printf("ws_probe: %s\n", bad_total ? "MISMATCH" : "all identical");
  return bad_total ? 2 : 0;
}
