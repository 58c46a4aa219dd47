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
// activation-plane buffers ([B][kPlanesMax][n][256] uint16) hold up to the split's 3 planes
constexpr int kPlanesMax = 3;

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
// Device-stamp accumulator of one launch site (graph node or eager launch) of a kernel kind
// (onepose_profile_begin_device).  Workgroups are spread over kStampShards counters and
// records by linear block id, so no word sees more than 1/16 of a launch's atomics (one
// word absorbs only ~88 atomics per us).  Per workgroup: thread 0 reads the clock at the start
// and takes a ticket from its shard (a returning atomic, issued where no wait includes it: the
// GEMMs take it after the K loop, which cut their stamp cost from ~1.1% to ~0.4% of the bench
// frame rate); at the end each wave counts itself in an LDS word, and the workgroup's last wave
// books launch e = ticket / (the shard's workgroups per launch) with two non-returning
// atomics: rec[e][shard] = (max of ~start, max end); the host takes min start / max end over
// the shards.  No barrier and no exposed round trip at the end: the earlier scheme (barrier +
// a returning atomic per workgroup on one word) cost the bench 3.5% (1456 vs 1509 frames/s).
constexpr int kStampShards = 16;
constexpr int kStampRecs = 256;   // launches per site recorded after arming (later ones dropped)
struct StampRec {
  unsigned long long nstart, end;   // ~min start, max end (0 = unused)
};
struct StampAcc {
  unsigned long long issued[kStampShards];   // workgroups started per shard since arming
  unsigned int overflow;                      // launches past kStampRecs (dropped)
  unsigned int pad[3];
  StampRec rec[kStampRecs][kStampShards];
};
struct StampTick {
  unsigned long long t0, tick;
};
struct StampLds {   // per workgroup, in LDS
  unsigned long long t0, tick;
  unsigned int arrived, pad;
};
// Accumulator for the next launch of `kind`, or null when stamping is off for it.
StampAcc* prof_stamp_slot(int kind);

__device__ __forceinline__ unsigned int stamp_block_id() {
  return blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
}
// stamp_start at the kernel's start, stamp_ticket anywhere before the first early return
// (stamp_begin = both).  Called by every thread (s is launch-uniform).  The kernel must pass a
// workgroup barrier before any wave reaches stamp_end (thread 0 zeroes the arrival word).
__device__ __forceinline__ StampTick stamp_start(StampAcc* s, StampLds* l) {
  StampTick k{0ull, 0ull};
  if (s != nullptr && threadIdx.x == 0) {
    l->arrived = 0u;
    k.t0 = (unsigned long long)wall_clock64();
  }
  return k;
}
__device__ __forceinline__ void stamp_ticket(StampAcc* s, StampTick& k) {
  if (s != nullptr && threadIdx.x == 0)
    k.tick = atomicAdd(&s->issued[stamp_block_id() % kStampShards], 1ull);
}
__device__ __forceinline__ StampTick stamp_begin(StampAcc* s, StampLds* l) {
  StampTick k = stamp_start(s, l);
  stamp_ticket(s, k);
  return k;
}
// Called at the end by every wave of the workgroup.
__device__ __forceinline__ void stamp_end(StampAcc* s, const StampTick& k, StampLds* l) {
  if (s == nullptr || (threadIdx.x & 63) != 0) return;
  if (threadIdx.x == 0) {   // wave 0 hands its ticket over before it counts itself
    l->t0 = k.t0;
    l->tick = k.tick;
  }
  const unsigned int nw = (blockDim.x * blockDim.y * blockDim.z + 63) / 64;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (atomicAdd(&l->arrived, 1u) != nw - 1) return;   // not the workgroup's last wave
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  const unsigned long long end = (unsigned long long)wall_clock64();
  const unsigned int blocks = gridDim.x * gridDim.y * gridDim.z, j = stamp_block_id() % kStampShards;
  const unsigned int per = blocks / kStampShards + (j < blocks % kStampShards ? 1u : 0u);
  const unsigned long long e = l->tick / per;
  if (e >= (unsigned long long)kStampRecs) {
    atomicAdd(&s->overflow, 1u);
    return;
  }
  atomicMax(&s->rec[e][j].nstart, ~l->t0);
  atomicMax(&s->rec[e][j].end, end);
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

// query_pose_error / Evaluator for one frame: t_err = |t_p - t_gt| * 100, R_err =
// deg(acos((tr(R_p R_gt^T) - 1) / 2)) with the trace clamped to <= 3 only (as the reference
// does; NaN -> 3 too), cm/deg flags at 1 / 3 / 5.  P, G: 3x4 row-major.
__device__ __forceinline__ void pose_error_one(const double* P, const double* G, double* rerr,
                                               double* terr, uint8_t* cmd3) {
  const double dx = P[3] - G[3], dy = P[7] - G[7], dz = P[11] - G[11];
  const double t = sqrt(dx * dx + dy * dy + dz * dz) * 100.0;
  double tr = 0.0;
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < 3; ++k) tr += P[i * 4 + k] * G[i * 4 + k];
  if (!(tr <= 3.0)) tr = 3.0;
  const double ang = acos((tr - 1.0) / 2.0) * (180.0 / M_PI);
  *rerr = ang;
  *terr = t;
  cmd3[0] = (t < 1.0 && ang < 1.0) ? 1 : 0;
  cmd3[1] = (t < 3.0 && ang < 3.0) ? 1 : 0;
  cmd3[2] = (t < 5.0 && ang < 5.0) ? 1 : 0;
}

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

// Activation planes: the bf16 modes' A operands, written by the producer of an activation
// beside its fp32 copy, so the next GEMM moves them to LDS by global_load_lds instead of
// rounding / splitting them in VALU every stage.  Plane q of x is the q-th piece of the exact
// split x = hi + mid + lo (hi = bf16(x) rounded to nearest even, mid = bf16(x - hi),
// lo = x - hi - mid; gemm.hip's store_quad_bf16 computes the same bits), `npl` planes (1: hi
// only, PM_BF16; 3: PM_SPLIT3) `pl` elements apart.  Four consecutive elements per call.
typedef __bf16 bf16x4_pl __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_planes4(uint16_t* p, int64_t pl, int npl, float4 v) {
  const float x[4] = {v.x, v.y, v.z, v.w};
  bf16x4_pl q0, q1, q2;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const __bf16 h = (__bf16)x[c];
    const float r = x[c] - (float)h;
    const __bf16 m = (__bf16)r;
    q0[c] = h;
    q1[c] = m;
    q2[c] = (__bf16)(r - (float)m);
  }
  *reinterpret_cast<bf16x4_pl*>(p) = q0;
  if (npl > 1) {
    *reinterpret_cast<bf16x4_pl*>(p + pl) = q1;
    *reinterpret_cast<bf16x4_pl*>(p + 2 * pl) = q2;
  }
}

// Bijection hardware block id -> logical id giving each XCD (hardware blocks b, b+8, ...)
// a contiguous range of logical ids.  Placement is a speed hint only, never correctness.
__device__ __forceinline__ int xcd_contiguous(int bid, int grid) {
  const int xcd = bid & 7, idx = bid >> 3;
  const int per = grid >> 3, rem = grid & 7;
  return xcd < rem ? xcd * (per + 1) + idx : rem * (per + 1) + (xcd - rem) * per + idx;
}

}  // namespace onepose
