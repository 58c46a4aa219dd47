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
  K_TRANSPOSE = 0, K_GAT, K_KV_GEMM, K_Q_GEMM, K_KV_REDUCE, K_MFOLD, K_MLP1, K_STATS, K_MLP2,
  K_FINAL, K_L2NORM, K_SCORE, K_SMX_REDUCE, K_CONF, K_MUTUAL, K_SELECT, K_PNP, K_PNP_REFIT,
  K_POSE_ERR, K_SAMPLE, K_NUM_KINDS
};
void prof_pre(int kind, hipStream_t s);
void prof_post(int kind, hipStream_t s);

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

}  // namespace onepose
