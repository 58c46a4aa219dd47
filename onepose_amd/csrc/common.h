// Shared helpers for libonepose_hip: error reporting across the C-ABI, launch checks,
// wave-level reductions.  gfx950 only (wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <string>

#include "../../include/onepose_hip.h"

namespace onepose {

void set_error(const char* fmt, ...);
void clear_error();

constexpr int kWave = 64;
constexpr int kDim = 256;       // descriptor_dim (train_GATsSPG.yaml:44)
constexpr int kHeads = 4;       // AttentionPropagation(feature_dim, 4)
constexpr int kHeadDim = 64;

#define OP_REQUIRE(cond, ...)                         \
  do {                                                \
    if (!(cond)) {                                    \
      ::onepose::set_error(__VA_ARGS__);              \
      return ONEPOSE_ERR_INVALID;                     \
    }                                                 \
  } while (0)

#define OP_HIP(call)                                                              \
  do {                                                                            \
    hipError_t e_ = (call);                                                       \
    if (e_ != hipSuccess) {                                                       \
      ::onepose::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), \
                           __FILE__, __LINE__);                                   \
      return ONEPOSE_ERR_HIP;                                                     \
    }                                                                             \
  } while (0)

// After a kernel launch: surface launch-configuration errors immediately.
#define OP_LAUNCHED()  OP_HIP(hipGetLastError())

// ---- launch profiling (measurement hook, see onepose_profile_begin in the header) ----
enum KernelKind {
  K_TRANSPOSE = 0, K_GAT, K_QKV_GEMM, K_KV_REDUCE, K_MFOLD, K_MLP1, K_STATS, K_MLP2,
  K_FINAL, K_L2NORM, K_SCORE, K_SMX_REDUCE, K_CONF, K_MUTUAL, K_SELECT, K_PNP, K_PNP_REFIT,
  K_POSE_ERR, K_SAMPLE, K_SP_CONV, K_SP_NMS, K_SP_SELECT, K_SP_DESC, K_NUM_KINDS
};
void prof_pre(int kind, hipStream_t s);
void prof_post(int kind, hipStream_t s);
// Device-stamp accumulator of one kernel kind (onepose_profile_begin_device).
struct StampAcc {
  unsigned long long start;      // min over the running launch's workgroups (~0 when armed)
  unsigned long long total;      // sum of finished launches' durations, clock ticks
  unsigned long long launches;   // finished launches
  unsigned int arrived;          // workgroups of the running launch that have finished
  unsigned int pad;
};
// Accumulator for the next launch of `kind`, or null when stamping is off for it.
StampAcc* prof_stamp_slot(int kind);

__device__ __forceinline__ void stamp_begin(StampAcc* s) {
  if (s != nullptr && threadIdx.x == 0) atomicMin(&s->start, (unsigned long long)wall_clock64());
}
// Every thread of the workgroup calls this at the kernel's end (s is launch-uniform).  The
// workgroup that arrives last reads the clock after its arrival, so no earlier workgroup
// ended later; it books the launch and re-arms the slot.  No fence: an agent-scope release
// would write back the XCD's L2 (microseconds) and the timing needs no data hand-off.
__device__ __forceinline__ void stamp_end(StampAcc* s) {
  if (s == nullptr) return;
  __syncthreads();
  if (threadIdx.x != 0) return;
  const unsigned int blocks = gridDim.x * gridDim.y * gridDim.z;
  if (atomicAdd(&s->arrived, 1u) == blocks - 1) {
    const unsigned long long e = (unsigned long long)wall_clock64();
    const unsigned long long b = atomicExch(&s->start, ~0ull);
    atomicAdd(&s->total, e - b);
    atomicAdd(&s->launches, 1ull);
    atomicExch(&s->arrived, 0u);
  }
}

// hipLaunchKernelGGL bracketed by the profiling hook, then a launch-error check
#define OP_LAUNCH(kind, stream, ...)            \
  do {                                          \
    ::onepose::prof_pre((kind), (stream));      \
    hipLaunchKernelGGL(__VA_ARGS__);            \
    ::onepose::prof_post((kind), (stream));     \
    OP_LAUNCHED();                              \
  } while (0)

static inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Bump allocator over a caller-provided workspace.
struct Carve {
  char* base;
  size_t off = 0;
  explicit Carve(void* p) : base(static_cast<char*>(p)) {}
  template <class T>
  T* take(size_t count) {
    off = align_up(off, 256);
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += count * sizeof(T);
    return p;
  }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// F.elu as ATen computes it (x > 0 ? x : exp(x) - 1), GATs.py:102 / GATs_SuperGlue.py:90-91
__device__ __forceinline__ float elu1(float x) { return x > 0.f ? x : (expf(x) - 1.0f); }

// Chan et al. pairwise merge of (count, mean, M2) statistics (InstanceNorm moments).
__device__ __forceinline__ void chan_merge(double& n, double& mean, double& m2, double nb,
                                           double mb, double m2b) {
  if (nb == 0.0) return;
  const double nn = n + nb;
  const double delta = mb - mean;
  mean += delta * (nb / nn);
  m2 += m2b + delta * delta * (n * nb / nn);
  n = nn;
}

// Bijection hardware block id -> logical id giving each XCD (hardware blocks b, b+8, ...)
// a contiguous range of logical ids.  Placement is a speed hint only, never correctness.
__device__ __forceinline__ int xcd_contiguous(int bid, int grid) {
  const int xcd = bid & 7, idx = bid >> 3;
  const int per = grid >> 3, rem = grid & 7;
  return xcd < rem ? xcd * (per + 1) + idx : rem * (per + 1) + (xcd - rem) * per + idx;
}

}  // namespace onepose
