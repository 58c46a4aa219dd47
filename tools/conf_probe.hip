// Dev tool (not shipped): what the dual-softmax conf kernel's time is made of, at config 2
// (1024 x 4096, B = 1).  Variants of a copy of conf_kernel (matcher.hip), HIP events over 200
// launches each:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/conf_probe.hip -o tools/conf_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

enum { NO_ROW_ATOMIC = 1, NO_COL_ATOMIC = 2, NO_WRITE = 4, NO_EXP = 8, NO_LOAD = 16, ROW_BATCH = 32, NT_LOAD = 64, NT_STORE = 128 };

__device__ __forceinline__ unsigned long long pack_best(float v, int idx) {
  return ((unsigned long long)__float_as_uint(v) << 32) | (unsigned)(0xFFFFFFFFu - (unsigned)idx);
}
__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int m) {
  const unsigned lo = __shfl_xor((unsigned)v, m, 64);
  const unsigned hi = __shfl_xor((unsigned)(v >> 32), m, 64);
  return ((unsigned long long)hi << 32) | lo;
}

template <int F, int RW>   // RW rows per wave
__global__ __launch_bounds__(256) void conf_v(float* S, int n1, int n3, const float* rowmax,
                                              const float* rowsum, const float* colmax,
                                              const float* colsum, unsigned long long* rowbest,
                                              unsigned long long* colbest) {
  __shared__ unsigned long long cb[4][256];
  const int ct = (n3 + 255) / 256;
  const int tilec = blockIdx.x % ct, tiler = blockIdx.x / ct;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int col[4];
  float cmx[4], cinv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    col[j] = tilec * 256 + lane * 4 + j;
    cmx[j] = colmax[col[j]];
    cinv[j] = 1.0f / colsum[col[j]];
  }
  float v[RW][4];
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const int n = min(tiler * 4 * RW + wave * RW + i, n1 - 1);
    if (F & NO_LOAD) {
      v[i][0] = v[i][1] = v[i][2] = v[i][3] = (float)(n & 7) * 0.01f;
    } else {
      typedef float fv4 __attribute__((ext_vector_type(4)));
      const fv4* ap = reinterpret_cast<const fv4*>(S + (int64_t)n * n3 + col[0]);
      const fv4 q = (F & NT_LOAD) ? __builtin_nontemporal_load(ap) : *ap;
      v[i][0] = q.x; v[i][1] = q.y; v[i][2] = q.z; v[i][3] = q.w;
    }
  }
  unsigned cbu[4] = {0u, 0u, 0u, 0u};
  int cbi[4] = {0, 0, 0, 0};
  unsigned long long rkey = 0ull;
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const int n = tiler * 4 * RW + wave * RW + i;
    if (n >= n1) break;
    const float rmx = rowmax[n];
    const float rinv = 1.0f / rowsum[n];
    unsigned ru = 0u;
    int ri = 0;
    float c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (F & NO_EXP) c[j] = ((v[i][j] - cmx[j]) * cinv[j]) * ((v[i][j] - rmx) * rinv);
      else c[j] = (expf(v[i][j] - cmx[j]) * cinv[j]) * (expf(v[i][j] - rmx) * rinv);
      const unsigned u = __float_as_uint(c[j]) + 1u;
      if (u > ru) { ru = u; ri = col[j]; }
      if (u > cbu[j]) { cbu[j] = u; cbi[j] = n; }
    }
    if (!(F & NO_WRITE)) {
      typedef float fv4 __attribute__((ext_vector_type(4)));
      fv4* sp = reinterpret_cast<fv4*>(S + (int64_t)n * n3 + col[0]);
      const fv4 o = {c[0], c[1], c[2], c[3]};
      if (F & NT_STORE) __builtin_nontemporal_store(o, sp);
      else *sp = o;
    }
    unsigned long long key = ru ? pack_best(__uint_as_float(ru - 1u), ri) : 0ull;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const unsigned long long other = shfl_xor_u64(key, o);
      key = other > key ? other : key;
    }
    if (F & ROW_BATCH) {
      if (lane == i) rkey = key;
    } else if (!(F & NO_ROW_ATOMIC) && lane == 0 && key != 0ull) {
      atomicMax(rowbest + n, key);
    }
  }
  if ((F & ROW_BATCH) && lane < RW && rkey != 0ull)   // one instruction, RW lanes / rows
    atomicMax(rowbest + tiler * 4 * RW + wave * RW + lane, rkey);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    cb[wave][lane * 4 + j] = cbu[j] ? pack_best(__uint_as_float(cbu[j] - 1u), cbi[j]) : 0ull;
  __syncthreads();
  const int cc = threadIdx.x, cg = tilec * 256 + cc;
  unsigned long long k = cb[0][cc];
  for (int w = 1; w < 4; ++w) k = cb[w][cc] > k ? cb[w][cc] : k;
  if (!(F & NO_COL_ATOMIC) && k != 0ull) atomicMax(colbest + cg, k);
}

template <int F, int RW>
void run(const char* name, float* S, int n1, int n3, float* rm, float* rs, float* cm, float* cs,
         unsigned long long* rb, unsigned long long* cbp) {
  const int grid = (n1 / (4 * RW)) * (n3 / 256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 20; ++w)
    hipLaunchKernelGGL((conf_v<F, RW>), dim3(grid), dim3(256), 0, 0, S, n1, n3, rm, rs, cm, cs, rb, cbp);
  hipEventRecord(e0);
  const int it = 200;
  for (int w = 0; w < it; ++w)
    hipLaunchKernelGGL((conf_v<F, RW>), dim3(grid), dim3(256), 0, 0, S, n1, n3, rm, rs, cm, cs, rb, cbp);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("%-28s rows/wave %2d  grid %5d  %7.2f us/launch\n", name, RW, grid, ms * 1e3 / it);
}

int main() {
  const int n1 = 1024, n3 = 4096;
  std::vector<float> h((size_t)n1 * n3);
  std::mt19937 rng(1);
  std::normal_distribution<float> N(0.f, 3.f);
  for (auto& x : h) x = N(rng);
  std::vector<float> rm(n1, 10.f), rs(n1, 100.f), cm(n3, 10.f), cs(n3, 100.f);
  float *S, *drm, *drs, *dcm, *dcs;
  unsigned long long *rb, *cb;
  hipMalloc(&S, h.size() * 4);
  hipMalloc(&drm, n1 * 4); hipMalloc(&drs, n1 * 4); hipMalloc(&dcm, n3 * 4); hipMalloc(&dcs, n3 * 4);
  hipMalloc(&rb, n1 * 8); hipMalloc(&cb, n3 * 8);
  hipMemcpy(drm, rm.data(), n1 * 4, hipMemcpyHostToDevice);
  hipMemcpy(drs, rs.data(), n1 * 4, hipMemcpyHostToDevice);
  hipMemcpy(dcm, cm.data(), n3 * 4, hipMemcpyHostToDevice);
  hipMemcpy(dcs, cs.data(), n3 * 4, hipMemcpyHostToDevice);
  // NO_WRITE first: S keeps its values for every read-only variant
  for (int rep = 0; rep < 2; ++rep) {
    hipMemcpy(S, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    run<NO_WRITE, 8>("no write", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
    run<NO_WRITE | NO_ROW_ATOMIC | NO_COL_ATOMIC, 8>("no write, no atomics", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
    run<NO_WRITE | NO_ROW_ATOMIC, 8>("no write, no row atomics", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
    run<NO_WRITE | NO_COL_ATOMIC, 8>("no write, no col atomics", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
    run<NO_WRITE | NO_EXP, 8>("no write, no exp", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
    run<NO_WRITE | NO_LOAD | NO_ROW_ATOMIC | NO_COL_ATOMIC, 8>("compute only", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
    run<0, 8>("as built (in place)", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
    run<0, 4>("as built, 16-row tiles", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
    run<0, 16>("as built, 64-row tiles", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
    run<NO_ROW_ATOMIC | NO_COL_ATOMIC, 8>("in place, no atomics", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
    run<NT_LOAD, 8>("nt loads", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
    run<NT_STORE, 8>("nt stores", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
    run<NT_LOAD | NT_STORE, 8>("nt loads + stores", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
    run<NO_ROW_ATOMIC | NT_LOAD | NT_STORE, 8>("nt, no row atomics", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
    run<ROW_BATCH, 8>("row atomics batched", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
    run<ROW_BATCH, 4>("row atomics batched", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
    run<ROW_BATCH, 16>("row atomics batched", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
    run<ROW_BATCH, 2>("row atomics batched", S, n1, n3, drm, drs, dcm, dcs, rb, cb);
  }
  return 0;
}
