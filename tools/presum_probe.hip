// Round 6 probe: what a bit-exact pre-sum of the KV chunk partials costs
// when one workgroup per (side, head) does it -- the form the fold's fixed chunk order allows
// inside QKV's last-arriving tile.  The fold (kv_fold256_kernel) sums chunk partials in this
// order: wave w takes chunks w, w + 4, w + 8, ... in order, then the four wave sums are added in
// wave order.  Here one 512-thread workgroup per (side, head) reads all of that head's partials
// (64 chunks x 16 KB on config 2's 3D side, 16 on the 2D side) and produces the same sums,
// every thread owning 8 of the head's 4096 KV entries.  Reported: event time of one launch of
// the 8 workgroups (4 heads x 2 sides), and of the whole-grid form for comparison (the same
// sums spread over 64 workgroups per head).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/presum_probe tools/presum_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int kHeads = 4, kEnt = 4096;

// grid: (side, head) x split; `split` workgroups share a head's 4096 entries
template <int SPLIT>
__global__ __launch_bounds__(512) void presum(const float* __restrict__ p3, int ch3,
                                              const float* __restrict__ p2, int ch2,
                                              float* __restrict__ out) {
  const int wg = blockIdx.x / SPLIT, part = blockIdx.x % SPLIT;
  const int side = wg / kHeads, h = wg % kHeads;
  const float* p = side ? p2 : p3;
  const int ch = side ? ch2 : ch3;
  constexpr int PER = kEnt / SPLIT / 512;   // entries per thread
  static_assert(PER >= 1, "split");
  const int e0 = part * (kEnt / SPLIT) + threadIdx.x * PER;
  float tot[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) tot[i] = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    float s[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) s[i] = 0.f;
    // every chunk of the residue class loaded before the in-order adds (16 loads in flight per
    // entry, as kv_fold256's KVF_DEPTH)
    constexpr int D = 16;
    for (int c0 = w; c0 < ch; c0 += 4 * D) {
      float v[D][PER];
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int c = c0 + 4 * d;
        const float* q = p + ((size_t)min(c, ch - 1) * kHeads + h) * kEnt + e0;
#pragma unroll
        for (int i = 0; i < PER; ++i) v[d][i] = c < ch ? q[i] : 0.f;
      }
#pragma unroll
      for (int d = 0; d < D; ++d)
#pragma unroll
        for (int i = 0; i < PER; ++i)
          if (c0 + 4 * d < ch) s[i] += v[d][i];
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) tot[i] = w == 0 ? s[i] : tot[i] + s[i];
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) out[(size_t)wg * kEnt + e0 + i] = tot[i];
}

template <int SPLIT>
static float time_it(const float* p3, int ch3, const float* p2, int ch2, float* out, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const dim3 grid(2 * kHeads * SPLIT);
  presum<SPLIT><<<grid, 512>>>(p3, ch3, p2, ch2, out);   // warm
  hipDeviceSynchronize();
  float best = 1e9f, sum = 0.f;
  for (int r = 0; r < reps; ++r) {
    hipEventRecord(a);
    presum<SPLIT><<<grid, 512>>>(p3, ch3, p2, ch2, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
    sum += ms;
  }
  hipEventDestroy(a);
  hipEventDestroy(b);
  printf("split %3d: %4d workgroups, event time best %.2f us, mean %.2f us\n", SPLIT,
         2 * kHeads * SPLIT, best * 1e3f, sum / reps * 1e3f);
  return best;
}

int main() {
  const int ch3 = 64, ch2 = 16;   // config 2: 4096 / 64 and 1024 / 64 chunk partials
  std::vector<float> h3((size_t)ch3 * kHeads * kEnt), h2((size_t)ch2 * kHeads * kEnt);
  for (size_t i = 0; i < h3.size(); ++i) h3[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
  for (size_t i = 0; i < h2.size(); ++i) h2[i] = (float)((i * 40503u) % 1000) * 1e-3f;
  float *p3, *p2, *out;
  CK(hipMalloc(&p3, h3.size() * 4));
  CK(hipMalloc(&p2, h2.size() * 4));
  CK(hipMalloc(&out, (size_t)2 * kHeads * kEnt * 4));
  CK(hipMemcpy(p3, h3.data(), h3.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(p2, h2.data(), h2.size() * 4, hipMemcpyHostToDevice));
  printf("bit-exact chunk pre-sum, config 2 (3D: %d chunks, 2D: %d, 4 heads x 4096 entries; "
         "%.1f MB read)\n", ch3, ch2, (h3.size() + h2.size()) * 4 / 1e6);
  time_it<1>(p3, ch3, p2, ch2, out, 50);    // one workgroup per (side, head): QKV's last tile
  time_it<2>(p3, ch3, p2, ch2, out, 50);
  time_it<8>(p3, ch3, p2, ch2, out, 50);    // whole-grid forms, for comparison
  CK(hipGetLastError());
  // check: the same sums on the host, in the fold's order
  std::vector<float> got((size_t)2 * kHeads * kEnt);
  CK(hipMemcpy(got.data(), out, got.size() * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int side = 0; side < 2; ++side)
    for (int h = 0; h < kHeads; ++h)
      for (int e = 0; e < kEnt; ++e) {
        const std::vector<float>& P = side ? h2 : h3;
        const int ch = side ? ch2 : ch3;
        float tot = 0.f;
        for (int w = 0; w < 4; ++w) {
          float s = 0.f;
          for (int c = w; c < ch; c += 4) s += P[((size_t)c * kHeads + h) * kEnt + e];
          tot = w == 0 ? s : tot + s;
        }
        if (tot != got[((size_t)side * kHeads + h) * kEnt + e]) ++bad;
      }
  printf("host check: %d of %d sums differ\n", bad, 2 * kHeads * kEnt);
  hipFree(p3);
  hipFree(p2);
  hipFree(out);
  return bad ? 1 : 0;
}
