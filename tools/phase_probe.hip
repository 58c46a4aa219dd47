// Where does a production GEMM launch spend its time?  Wraps gemm.hip's gemm_body in a kernel
// that stamps every workgroup (s_memrealtime / s_memtime at entry and after its last barrier,
// plus its CU from HW_ID / XCC_ID), and reports per launch: event time, device span, the
// in-kernel clock, workgroup duration spread, dispatch skew and per-CU load.
//
//   bash tools/probe_src.sh   (generates _gen/gemm.hip with the stamps, then builds)
__device__ unsigned long long* g_phase;
#define ONEPOSE_GEMM_PHASE(i) \
  if (threadIdx.x == 0) g_phase[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memtime();
#include "_gen/gemm.hip"   // tools/probe_src.sh
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <map>
#include <cstdarg>
#include <vector>

namespace onepose {
void set_error(const char* fmt, ...) { va_list ap; va_start(ap, fmt); vprintf(fmt, ap); va_end(ap); printf("\n"); }
void clear_error() {}
void prof_pre(int, hipStream_t) {}
void prof_post(int, hipStream_t) {}
StampAcc* prof_stamp_slot(int) { return nullptr; }
}
using namespace onepose;

struct WgRec {
  unsigned long long rt0, rt1, mt0, mt1;
  unsigned hwid, xcc, pad0, pad1;
};

// g_stagger (round 6, `stagger` mode): workgroups with hardware id >= g_stagger[0] wait
// g_stagger[1] shader cycles before their prologue, those >= g_stagger[2] g_stagger[3] cycles
// (dispatch order: the third workgroup of each CU comes from the last 256 ids) -- do co-resident
// workgroups whose prologues / epilogues coincide lose the MFMA pipe for them?
__device__ unsigned long long g_stagger[4];
template <int EPI, int PRO, class T, int PM, bool WPL, int DMA>
__global__ __launch_bounds__(T::NT) __attribute__((amdgpu_waves_per_eu(T::WPE)))
void phase_kernel(GemmArgs args, WgRec* rec) {
  __shared__ StampLds sl;
  StampTick tk{0ull, 0ull};
  {
    const unsigned long long d = blockIdx.x >= g_stagger[2] ? g_stagger[3]
                                 : blockIdx.x >= g_stagger[0] ? g_stagger[1] : 0ull;
    if (d) {
      const unsigned long long t0 = __builtin_amdgcn_s_memtime();
      while (__builtin_amdgcn_s_memtime() - t0 < d) __builtin_amdgcn_s_sleep(8);
    }
  }
  const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long mt0 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) g_phase[blockIdx.x * 8] = mt0;
  gemm_body<EPI, PRO, T, PM, WPL, DMA>(args, tk, &sl);
  __syncthreads();
  if (threadIdx.x == 0) g_phase[blockIdx.x * 8 + 3] = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    WgRec r;
    r.mt1 = __builtin_amdgcn_s_memtime();
    r.rt1 = __builtin_amdgcn_s_memrealtime();
    r.rt0 = rt0;
    r.mt0 = mt0;
    r.hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    r.xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);    // HW_REG_XCC_ID
    r.pad0 = r.pad1 = 0;
    rec[blockIdx.x] = r;
  }
}

// The verdict-r04 persistent form: a grid of `gridDim.x` resident workgroups, each taking the
// logical tiles blockIdx.x, blockIdx.x + gridDim.x, ... in turn (the production gemm_body per
// tile; its InstanceNorm tickets are per tile, so any tile order gives the same bits).
template <int EPI, int PRO, class T, int PM, bool WPL, int DMA>
__global__ __launch_bounds__(T::NT) __attribute__((amdgpu_waves_per_eu(T::WPE)))
void persist_kernel(GemmArgs args, int tiles) {
  __shared__ StampLds sl;
  StampTick tk{0ull, 0ull};
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    gemm_body<EPI, PRO, T, PM, WPL, DMA>(args, tk, &sl, t);
    __syncthreads();
  }
}

static std::vector<float> g_lastY;   // Y of the last run (first M x N)

struct Bufs {
  float *A, *W, *b, *Y, *stats, *mean, *rstd, *ksum;
  double* grp;   // InstanceNorm group partials (gemm.h st_grp)
  uint16_t* Wp;   // 3 bf16 planes of W ([N][K] each, MMAX-sized stride)
  uint16_t* Ab;   // bf16 copy of A ([MMAX][K], round to nearest even)
  uint16_t* Ap;   // 3 activation planes of A ([MMAX][K] each: the exact split; plane 0 = Ab)
  int64_t wpl, apl;
  unsigned* cnt;
  WgRec* rec;
};

template <int EPI, int PRO, class T, int PM = PM_F32, int DMA = 0>
void run(const char* name, Bufs& B, int M, int N, int K, bool fin, int iters) {
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.nprob = 1;
  GemmProb& p = a.p[0];
  p = gemm_prob(B.A, K, B.W, K, B.b, B.Y, N, M, N, K, 1);
  if (PM != PM_F32) {
    p.Wp = B.Wp;
    p.wpl = B.wpl;
  }
  if (DMA == 2) {   // A planes by global_load_lds (the product's QKV / MLP conv 1 in bf16 modes)
    p.Ap = B.Ap;
    p.apl = B.apl;
    p.ldap = K;
  }
  p.stats = B.stats;
  p.st_cnt = fin ? B.cnt : nullptr;
  p.st_cnt_bs = 1024;   // one sample: the whole counter buffer
  p.st_grp = B.grp;
  p.st_mean = B.mean;
  p.st_rstd = B.rstd;
  if (PRO == PRO_HEADZ) {   // K = [x (256) | phi(q) (256)] from the same A rows
    p.ksplit = K - 256;
    p.A1 = B.A + (K - 256);
    p.lda1 = K;
    p.ksum = B.ksum;
    p.ns = 4096.f;
    if (DMA == 2) {
      p.Ap1 = B.Ap + (K - 256);
      p.apl1 = B.apl;
      p.ldap1 = K;
    }
  }
  if (EPI == EPI_QKV) {
    p.kvpart = B.stats;    // [mtiles][4][64][64]: 80 x 64 KB = 5 MB < 16 MB
    p.kspart = B.stats + (6 << 20);
    p.vdiv = 4096.f;
  }
  if (EPI == EPI_SCORE) {   // S = D2 D3^T / scale: D3 rows from A's buffer (W holds 768 rows)
    p.W = B.A + (size_t)8192 * 512;
    p.ldw = K;
    p.rowstat = B.stats;
    p.colstat = B.stats + (4 << 20);
    p.scale = 16.f;
  }
  if (PRO == PRO_NORM_RELU) {
    p.pro_mean = B.mean;
    p.pro_rstd = B.rstd;
    p.R = B.Y;
    p.ldr = N;
  }
  p.mtiles = (M + T::BM - 1) / T::BM;
  p.ntiles = (N + T::BN - 1) / T::BN;
  p.tiles = p.mtiles * p.ntiles;
  const int grid = p.tiles;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  std::vector<WgRec> h(grid);
  std::vector<unsigned long long> ph((size_t)grid * 8);
  double pro = 0, loop = 0, epi = 0, e_stage = 0, e_merge = 0, e_ticket = 0, e_fin = 0;
  double ev_sum = 0, span_sum = 0, clk_sum = 0, dur_med = 0, dur_max = 0, dur_min = 0, skew50 = 0,
         skew_max = 0, tail = 0, cu_max = 0, cu_mean = 0, busy = 0;
  int cus = 0, maxper = 0;
  for (int it = -3; it < iters; ++it) {
    if (fin) hipMemsetAsync(B.cnt, 0, 4096);
    hipEventRecord(e0);
    hipLaunchKernelGGL((phase_kernel<EPI, PRO, T, PM, PM != PM_F32, DMA>), dim3(grid), dim3(T::NT), 0,
                       0, a, B.rec);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    if (it < 0) continue;
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(h.data(), B.rec, grid * sizeof(WgRec), hipMemcpyDeviceToHost);
    {
      unsigned long long* dp;
      hipMemcpyFromSymbol(&dp, HIP_SYMBOL(g_phase), sizeof(dp));
      hipMemcpy(ph.data(), dp, ph.size() * 8, hipMemcpyDeviceToHost);
      double a = 0, b = 0, c2 = 0, s4 = 0, s5 = 0, s6 = 0, s7 = 0;
      int n5 = 0;
      for (int i = 0; i < grid; ++i) {
        const unsigned long long* q = &ph[8 * i];
        a += (double)(q[1] - q[0]);
        b += (double)(q[2] - q[1]);
        c2 += (double)(q[3] - q[2]);
        if (q[4] > q[2] && q[4] <= q[3]) s4 += (double)(q[4] - q[2]);
        if (q[5] > q[4] && q[6] > q[5] && q[6] <= q[3]) {
          s5 += (double)(q[5] - q[4]);
          s6 += (double)(q[6] - q[5]);
          s7 += (double)(q[3] - q[6]);
          ++n5;
        }
      }
      pro += a / grid;
      loop += b / grid;
      epi += c2 / grid;
      e_stage += s4 / grid;
      if (n5) {
        e_merge += s5 / n5;
        e_ticket += s6 / n5;
        e_fin += s7 / n5;
      }
    }
    unsigned long long s0 = ~0ull, s1 = 0;
    double dm = 0, dr = 0;
    std::vector<double> dur, st, en;
    std::map<unsigned, std::vector<int>> percu;
    for (int i = 0; i < grid; ++i) {
      s0 = std::min(s0, h[i].rt0);
      s1 = std::max(s1, h[i].rt1);
      dm += (double)(h[i].mt1 - h[i].mt0);
      dr += (double)(h[i].rt1 - h[i].rt0);
      const unsigned cu = ((h[i].xcc & 0xf) << 16) | (((h[i].hwid >> 13) & 7) << 8) |
                          (((h[i].hwid >> 12) & 1) << 4) | ((h[i].hwid >> 8) & 0xf);
      percu[cu].push_back(i);
    }
    for (int i = 0; i < grid; ++i) {
      dur.push_back((h[i].rt1 - h[i].rt0) * 0.01);   // us (100 MHz)
      st.push_back((h[i].rt0 - s0) * 0.01);
      en.push_back((h[i].rt1 - s0) * 0.01);
    }
    std::vector<double> d2 = dur, s2 = st, e2 = en;
    std::sort(d2.begin(), d2.end());
    std::sort(s2.begin(), s2.end());
    std::sort(e2.begin(), e2.end());
    ev_sum += ms * 1e3;
    span_sum += (s1 - s0) * 0.01;
    clk_sum += dm / dr * 0.1;   // GHz
    dur_min += d2.front();
    dur_med += d2[grid / 2];
    dur_max += d2.back();
    skew50 += s2[grid / 2];
    skew_max += s2.back();
    tail += e2.back() - e2[grid / 2];
    double cmax = 0, csum = 0;
    int mp = 0;
    for (auto& kv : percu) {
      double lastend = 0, sumd = 0;
      for (int i : kv.second) {
        lastend = std::max(lastend, en[i]);
        sumd += dur[i];
      }
      cmax = std::max(cmax, lastend);
      csum += sumd;
      mp = std::max(mp, (int)kv.second.size());
    }
    cu_max += cmax;
    cu_mean += csum / percu.size();
    busy += csum / (percu.size() * ((s1 - s0) * 0.01));
    cus = (int)percu.size();
    maxper = mp;
  }
  const double n = iters;
  printf("   phases (cycles, mean per WG): prologue %.0f  loop %.0f (%.0f per stage)  epilogue %.0f"
         " [stage+sync %.0f | stats merge+drain %.0f | ticket+rows %.0f | rest %.0f]\n",
         pro / n, loop / n, loop / n / (K / T::BKS), epi / n, e_stage / n, e_merge / n,
         e_ticket / n, e_fin / n);
  printf("%-26s M %6d N %4d K %4d grid %5d | event %6.2f us span %6.2f | clock %.2f GHz | wg dur "
         "min/med/max %5.2f/%5.2f/%5.2f | start skew med/max %5.2f/%5.2f | tail(50%%->last) %5.2f | "
         "CUs %d, max wg/CU %d, sum wg-us/CU %6.2f, wg-occupancy %.2f\n",
         name, M, N, K, grid, ev_sum / n, span_sum / n, clk_sum / n, dur_min / n, dur_med / n,
         dur_max / n, skew50 / n, skew_max / n, tail / n, cus, maxper, cu_mean / n, busy / n);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  g_lastY.resize((size_t)M * N);
  hipMemcpy(g_lastY.data(), B.Y, g_lastY.size() * 4, hipMemcpyDeviceToHost);
}
// event time of the persistent form over `grid` workgroups; its Y against the one-shot run's
template <int EPI, int PRO, class T, int PM = PM_F32, int DMA = 0>
void persist_run(Bufs& B, int M, int N, int K, int grid, int iters) {
  std::vector<float> ref = g_lastY;
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.nprob = 1;
  GemmProb& p = a.p[0];
  p = gemm_prob(B.A, K, B.W, K, B.b, B.Y, N, M, N, K, 1);
  p.stats = B.stats;
  p.st_cnt = B.cnt;
  p.st_cnt_bs = 1024;
  p.st_grp = B.grp;
  p.st_mean = B.mean;
  p.st_rstd = B.rstd;
  p.ksplit = K - 256;
  p.A1 = B.A + (K - 256);
  p.lda1 = K;
  p.ksum = B.ksum;
  p.ns = 4096.f;
  p.mtiles = (M + T::BM - 1) / T::BM;
  p.ntiles = (N + T::BN - 1) / T::BN;
  p.tiles = p.mtiles * p.ntiles;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  double sum = 0;
  for (int it = -3; it < iters; ++it) {
    hipMemsetAsync(B.cnt, 0, 4096);
    hipEventRecord(e0);
    hipLaunchKernelGGL((persist_kernel<EPI, PRO, T, PM, PM != PM_F32, DMA>), dim3(grid), dim3(T::NT), 0,
                       0, a, p.tiles);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (it >= 0) sum += ms * 1e3;
  }
  std::vector<float> y((size_t)M * N);
  hipMemcpy(y.data(), B.Y, y.size() * 4, hipMemcpyDeviceToHost);
  size_t bad = 0;
  for (size_t i = 0; i < y.size() && i < ref.size(); ++i) bad += memcmp(&y[i], &ref[i], 4) != 0;
  printf("persistent grid %4d: tiles %d | event %6.2f us | Y vs one-shot: %zu of %zu differ\n", grid,
         p.tiles, sum / iters, bad, y.size());
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

static double maxdiff(const std::vector<float>& a, const std::vector<float>& b) {
  double d = 0;
  for (size_t i = 0; i < a.size() && i < b.size(); ++i) d = std::max(d, (double)std::fabs(a[i] - b[i]));
  return d;
}

int main(int argc, char** argv) {
  const int MMAX = 16384, K = 512, N = 768;   // W rows: up to 768 (QKV)
  srand(1);
  std::vector<float> hA((size_t)MMAX * K), hW((size_t)N * K), hb(N), hk(256, 30.f), hm(N, 0.1f),
      hr(N, 1.5f);
  for (auto& x : hA) x = (float)rand() / RAND_MAX * 2.f - 1.f;
  for (auto& x : hW) x = ((float)rand() / RAND_MAX * 2.f - 1.f) * 0.05f;
  for (auto& x : hb) x = (float)rand() / RAND_MAX - 0.5f;
  Bufs B;
  hipMalloc(&B.A, hA.size() * 4);
  hipMalloc(&B.W, hW.size() * 4);
  hipMalloc(&B.b, N * 4);
  hipMalloc(&B.Y, (size_t)MMAX * N * 4);
  hipMalloc(&B.stats, 32 << 20);
  hipMalloc(&B.mean, 4096);
  hipMalloc(&B.rstd, 4096);
  hipMalloc(&B.ksum, 4096);
  hipMalloc(&B.cnt, 4096);
  hipMalloc(&B.grp, 1 << 20);
  hipMalloc(&B.rec, 65536 * sizeof(WgRec));
  {
    unsigned long long* dp;
    hipMalloc(&dp, 65536 * 8 * 8);
    hipMemset(dp, 0, 65536 * 8 * 8);
    hipMemcpyToSymbol(HIP_SYMBOL(g_phase), &dp, sizeof(dp));
  }
  hipMemcpy(B.A, hA.data(), hA.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(B.W, hW.data(), hW.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(B.b, hb.data(), N * 4, hipMemcpyHostToDevice);
  hipMemcpy(B.ksum, hk.data(), 1024, hipMemcpyHostToDevice);
  hipMemcpy(B.mean, hm.data(), N * 4, hipMemcpyHostToDevice);
  hipMemcpy(B.rstd, hr.data(), N * 4, hipMemcpyHostToDevice);
  hipMemset(B.Y, 0, (size_t)MMAX * N * 4);
  {
    std::vector<uint16_t> pl((size_t)3 * N * K);
    auto bits = [](float x) { uint32_t u; memcpy(&u, &x, 4); return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16); };
    auto val = [](uint16_t h) { uint32_t u = (uint32_t)h << 16; float x; memcpy(&x, &u, 4); return x; };
    for (size_t i = 0; i < (size_t)N * K; ++i) {
      const float x = hW[i];
      const uint16_t h = bits(x);
      const float r = x - val(h);
      const uint16_t m = bits(r);
      pl[i] = h;
      pl[(size_t)N * K + i] = m;
      pl[(size_t)2 * N * K + i] = bits(r - val(m));
    }
    std::vector<uint16_t> ab(hA.size()), ap(3 * hA.size());
    for (size_t i = 0; i < hA.size(); ++i) {
      const float x = hA[i];
      const uint16_t h = bits(x);
      const float r = x - val(h);
      const uint16_t m = bits(r);
      ab[i] = ap[i] = h;
      ap[hA.size() + i] = m;
      ap[2 * hA.size() + i] = bits(r - val(m));
    }
    hipMalloc(&B.Ap, ap.size() * 2);
    hipMemcpy(B.Ap, ap.data(), ap.size() * 2, hipMemcpyHostToDevice);
    B.apl = (int64_t)hA.size();
    hipMalloc(&B.Ab, ab.size() * 2);
    hipMemcpy(B.Ab, ab.data(), ab.size() * 2, hipMemcpyHostToDevice);
    hipMalloc(&B.Wp, pl.size() * 2);
    hipMemcpy(B.Wp, pl.data(), pl.size() * 2, hipMemcpyHostToDevice);
    B.wpl = (int64_t)N * K;
  }
  const int it = 20;
  using T64x128 = Tile<64, 128, 1, 4, 32>;
  using T64x128B = Tile<64, 128, 1, 4, 64>;
  for (int r = 0; r < 2; ++r) run<EPI_STATS, PRO_HEADZ, T64x64>("warm", B, 5120, 512, 512, true, 200);
  if (argc > 1 && !strcmp(argv[1], "placement")) {   // round 6: which CU each hardware block lands on
    for (int m : {5120, 6144}) {
      run<EPI_STATS, PRO_HEADZ, T64x64>("placement", B, m, 512, 512, true, 1);
      const int grid = (m / 64) * 8;
      std::vector<WgRec> h(grid);
      hipMemcpy(h.data(), B.rec, grid * sizeof(WgRec), hipMemcpyDeviceToHost);
      std::map<unsigned, std::vector<int>> percu;
      for (int i = 0; i < grid; ++i) {
        const unsigned cu = ((h[i].xcc & 0xf) << 16) | (((h[i].hwid >> 13) & 7) << 8) |
                            (((h[i].hwid >> 12) & 1) << 4) | ((h[i].hwid >> 8) & 0xf);
        percu[cu].push_back(i);
      }
      // per CU: the within-XCD dispatch indices (block / 8) of its blocks, and the XCD check
      int xcd_ok = 0, slot_ok = 0, n3 = 0;
      std::map<int, int> hist;
      for (auto& kv : percu) {
        const auto& v = kv.second;
        bool same_xcd = true;
        for (int b : v) same_xcd &= (unsigned)(b & 7) == ((kv.first >> 16) & 7);
        xcd_ok += same_xcd;
        hist[(int)v.size()]++;
        // "slot by slot": the CU's k-th block has within-XCD index in [32k, 32k + 32)
        bool sl = true;
        std::vector<int> idx;
        for (int b : v) idx.push_back(b / 8);
        std::sort(idx.begin(), idx.end());
        for (size_t k = 0; k < idx.size(); ++k) sl &= idx[k] >= 32 * (int)k && idx[k] < 32 * (int)k + 32;
        slot_ok += sl;
        if (v.size() == 3) ++n3;
      }
      printf("M %d grid %d: CUs %zu, blocks per CU histogram:", m, grid, percu.size());
      for (auto& kv : hist) printf(" %d->%d", kv.first, kv.second);
      printf(" | CUs whose blocks share the block's XCD (b %% 8): %d | CUs filled slot by slot (k-th block index in [32k, 32k+32)): %d\n",
             xcd_ok, slot_ok);
      int shown = 0;
      for (auto& kv : percu) {
        if (shown++ >= 12) break;
        printf("  cu %06x:", kv.first);
        for (int b : kv.second) printf(" %d(x%d,i%d)", b, b & 7, b / 8);
        printf("\n");
      }
    }
    return 0;
  }
  if (argc > 1 && !strcmp(argv[1], "stagger")) {   // round 6: staggered workgroup starts
    // (the event time covers the delays; "span" starts at the first workgroup's post-delay stamp,
    // so read the event column)
    auto stag = [&](unsigned long long a, unsigned long long da, unsigned long long b,
                    unsigned long long db) {
      unsigned long long v[4] = {a, da, b, db};
      hipMemcpyToSymbol(HIP_SYMBOL(g_stagger), v, sizeof(v));
    };
    for (int m : {5120, 6144}) {
      printf("--- fp32 mlp1 STATS+HEADZ+fin, M %d: third workgroup per CU delayed ---\n", m);
      for (int r = 0; r < 2; ++r) {
        for (unsigned long long d : {0ull, 6000ull, 12000ull, 24000ull, 36000ull}) {
          stag(512, d, 1u << 30, 0);
          char nm[64];
          snprintf(nm, sizeof nm, "ids>=512 +%llu cyc", d);
          run<EPI_STATS, PRO_HEADZ, T64x64>(nm, B, m, 512, 512, true, it);
        }
        for (unsigned long long d : {6000ull, 12000ull, 20000ull}) {
          stag(256, d, 512, 2 * d);
          char nm[64];
          snprintf(nm, sizeof nm, "2nd +%llu, 3rd +%llu", d, 2 * d);
          run<EPI_STATS, PRO_HEADZ, T64x64>(nm, B, m, 512, 512, true, it);
        }
        stag(1u << 30, 0, 1u << 30, 0);
      }
    }
    return 0;
  }
  if (argc > 1 && !strcmp(argv[1], "mlp2")) {   // round 4: fp32 MLP conv 2 tiles (RESID + NORM)
    using T64x64K2W8 = Tile<64, 64, 2, 8, 64>;
    using T128x32K2W8 = Tile<128, 32, 2, 8, 64>;
    using T64x32K2W = Tile<64, 32, 2, 4, 64>;
    for (int m : {5120, 10240}) {
      printf("--- mlp2 RESID+NORM fp32, M %d N 256 K 512 ---\n", m);
      for (int r = 0; r < 2; ++r) {
        run<EPI_RESID, PRO_NORM_RELU, T64x32K2W>("fp32 64x32K2 (production)", B, m, 256, 512, false, it);
        run<EPI_RESID, PRO_NORM_RELU, T64x64K2W8>("fp32 64x64K2 w8", B, m, 256, 512, false, it);
        run<EPI_RESID, PRO_NORM_RELU, T128x32K2W8>("fp32 128x32K2 w8", B, m, 256, 512, false, it);
        run<EPI_RESID, PRO_NORM_RELU, T64x64>("fp32 64x64", B, m, 256, 512, false, it);
      }
    }
    return 0;
  }
  if (argc > 1 && !strcmp(argv[1], "big")) {   // round 4: wider split / bf16 tiles, 8 waves
    using T128x128W8 = Tile<128, 128, 1, 8, 32>;
    for (int m : {5120, 10240}) {
      printf("--- mlp1 STATS+HEADZ+fin, M %d ---\n", m);
      run<EPI_STATS, PRO_HEADZ, T64x64, PM_SPLIT3, 2>("split 64x64 dma2", B, m, 512, 512, true, it);
      run<EPI_STATS, PRO_HEADZ, T128x128W8, PM_SPLIT3, 2>("split 128x128 w8 dma2", B, m, 512, 512, true, it);
      run<EPI_STATS, PRO_HEADZ, T64x128, PM_BF16, 2>("bf16 64x128 dma2", B, m, 512, 512, true, it);
      run<EPI_STATS, PRO_HEADZ, T128x128W8, PM_BF16, 2>("bf16 128x128 w8 dma2", B, m, 512, 512, true, it);
      printf("--- qkv, M %d N 768 K 256 ---\n", m);
      run<EPI_QKV, PRO_PLAIN, T64x128, PM_SPLIT3, 2>("split 64x128 dma2", B, m, 768, 256, false, it);
      run<EPI_QKV, PRO_PLAIN, T128x128, PM_SPLIT3, 2>("split 128x128 dma2", B, m, 768, 256, false, it);
      run<EPI_QKV, PRO_PLAIN, T64x128, PM_BF16, 2>("bf16 64x128 dma2", B, m, 768, 256, false, it);
      run<EPI_QKV, PRO_PLAIN, T128x128, PM_BF16, 2>("bf16 128x128 dma2", B, m, 768, 256, false, it);
    }
    return 0;
  }
  if (argc > 1 && !strcmp(argv[1], "persist")) {   // round 5: the persistent form of fp32 MLP conv 1
    for (int m : {5120, 10240}) {
      printf("--- fp32 mlp1 STATS+HEADZ+fin, M %d: one-shot grid vs persistent grids ---\n", m);
      for (int r = 0; r < 2; ++r) {
        run<EPI_STATS, PRO_HEADZ, T64x64>("fp32 64x64 one-shot", B, m, 512, 512, true, it);
        for (int g : {256, 512, 768}) persist_run<EPI_STATS, PRO_HEADZ, T64x64>(B, m, 512, 512, g, it);
      }
    }
    return 0;
  }
  if (argc > 1 && !strcmp(argv[1], "ws")) {   // round 5: bf16 MLP conv 1 on 256 x 128, 8 waves
    using T256x128W8 = Tile<256, 128, 1, 8, 32, 2, 64>;
    for (int m : {5120, 10240}) {
      printf("--- bf16 mlp1 STATS+HEADZ+fin, M %d (A planes by DMA) ---\n", m);
      for (int r = 0; r < 2; ++r) {
        run<EPI_STATS, PRO_HEADZ, T64x128, PM_BF16, 2>("bf16 64x128 dma2", B, m, 512, 512, true, it);
        run<EPI_STATS, PRO_HEADZ, T256x128W8, PM_BF16, 2>("bf16 256x128 w8 dma2", B, m, 512, 512, true, it);
        run<EPI_STATS, PRO_HEADZ, T256x128W8, PM_BF16, 2>("bf16 256x128 w8 (no fin)", B, m, 512, 512, false, it);
      }
    }
    return 0;
  }
  if (argc > 1 && !strcmp(argv[1], "dma")) {   // round 4: the DMA-2 loop (A and W planes)
    for (int m : {5120, 10240}) {
      printf("--- mlp1 STATS+HEADZ+fin, M %d (A planes by DMA) ---\n", m);
      run<EPI_STATS, PRO_HEADZ, T64x64>("fp32 64x64 (production)", B, m, 512, 512, true, it);
      run<EPI_STATS, PRO_HEADZ, T64x64, PM_SPLIT3, 2>("split 64x64 dma2", B, m, 512, 512, true, it);
      run<EPI_STATS, PRO_HEADZ, T64x128, PM_SPLIT3, 2>("split 64x128 dma2", B, m, 512, 512, true, it);
      run<EPI_STATS, PRO_HEADZ, T64x128, PM_BF16, 2>("bf16 64x128 dma2", B, m, 512, 512, true, it);
      run<EPI_STATS, PRO_HEADZ, T64x128, PM_BF16, 1>("bf16 64x128 dma1", B, m, 512, 512, true, it);
      printf("--- qkv, M %d N 768 K 256 ---\n", m);
      run<EPI_QKV, PRO_PLAIN, T32x128>("fp32 32x128", B, m, 768, 256, false, it);
      run<EPI_QKV, PRO_PLAIN, T32x128, PM_SPLIT3, 2>("split 32x128 dma2", B, m, 768, 256, false, it);
      run<EPI_QKV, PRO_PLAIN, T64x128, PM_SPLIT3, 2>("split 64x128 dma2", B, m, 768, 256, false, it);
      run<EPI_QKV, PRO_PLAIN, T64x128, PM_BF16, 2>("bf16 64x128 dma2", B, m, 768, 256, false, it);
    }
    return 0;
  }
  printf("--- score GEMM (config 2: 1024 x 4096, K 256) ---\n");
  using T128x64W8 = Tile<128, 64, 1, 8, 32>;
  for (int r = 0; r < 2; ++r) {
    run<EPI_SCORE, PRO_PLAIN, T128x64W8>("fp32 score 128x64 W8", B, 1024, 4096, 256, false, it);
    run<EPI_SCORE, PRO_PLAIN, T64x64>("fp32 score 64x64", B, 1024, 4096, 256, false, it);
  }
  printf("--- fp32 mlp1 stage time vs workgroups per CU (256 / 512 / 640 / 768 tiles) ---\n");
  run<EPI_STATS, PRO_HEADZ, T64x64>("fp32 mlp1 1/CU", B, 2048, 512, 512, true, it);
  run<EPI_STATS, PRO_HEADZ, T64x64>("fp32 mlp1 2/CU", B, 4096, 512, 512, true, it);
  run<EPI_STATS, PRO_HEADZ, T64x64>("fp32 mlp1 2.5/CU", B, 5120, 512, 512, true, it);
  run<EPI_STATS, PRO_HEADZ, T64x64>("fp32 mlp1 3/CU", B, 6144, 512, 512, true, it);
  run<EPI_BIAS, PRO_PLAIN, T64x64>("fp32 plain 1/CU", B, 2048, 512, 512, false, it);
  run<EPI_BIAS, PRO_PLAIN, T64x64>("fp32 plain 3/CU", B, 6144, 512, 512, false, it);
  printf("--- mlp1 epilogue breakdown (M 5120) ---\n");
  run<EPI_STATS, PRO_HEADZ, T64x64>("fp32 mlp1", B, 5120, 512, 512, true, it);
  run<EPI_STATS, PRO_HEADZ, T64x128, PM_BF16, 1>("bf16 mlp1", B, 5120, 512, 512, true, it);
  run<EPI_STATS, PRO_HEADZ, T64x64>("fp32 mlp1 (no finalize)", B, 5120, 512, 512, false, it);
  run<EPI_STATS, PRO_HEADZ, T64x128, PM_BF16, 1>("bf16 mlp1 (no fin)", B, 5120, 512, 512, false, it);
  printf("--- M 10240 ---\n");
  run<EPI_STATS, PRO_HEADZ, T64x64>("fp32 mlp1", B, 10240, 512, 512, true, it);
  run<EPI_STATS, PRO_HEADZ, T64x128, PM_BF16, 1>("bf16 mlp1", B, 10240, 512, 512, true, it);
  return 0;
}
