// Dev tool (not shipped): can an fp32-accurate 3-way bf16 split GEMM beat the fp32-MFMA loop on
// the config-2 mlp1 shape (M = 5120, N = 512, K = 512)?  The production PM_SPLIT3 mode splits
// both operands in VALU and stores three bf16 LDS images of each: VALU- and LDS-write bound.
// Here the W operand comes pre-split from HBM (three bf16 planes, [N][K] each) straight into LDS
// by global_load_lds (no VGPR round trip, no VALU), A is loaded fp32, split in VALU and stored
// as three planes (one ds_write_b128 per plane and 8 elements); 64-byte LDS rows with the 16-B
// chunk XOR-swizzled by (row >> 2) & 3 (conflict-free ds_read_b128).  MODE 1: single-plane
// bf16 (A rounded, W plane 0), the bf16-attention analogue.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -w tools/split_probe.hip -o tools/split_probe
#include "../onepose_amd/csrc/gemm.hip"
#include <cmath>
#include <cstdarg>
#include <cstdlib>
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

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void split8(const float4& x0, const float4& x1, bf16x8_t& h, bf16x8_t& m,
                                       bf16x8_t& l) {
  const float x[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 hb = (__bf16)x[j];
    const float r = x[j] - (float)hb;
    const __bf16 mb = (__bf16)r;
    h[j] = hb;
    m[j] = mb;
    l[j] = (__bf16)(r - (float)mb);
  }
}

template <int BM, int BN, int MODE>
__global__ __launch_bounds__(256) void split_gemm(const float* __restrict__ A, int lda,
                                                  const __bf16* __restrict__ Wp, int64_t wplane,
                                                  int ldw, const float* __restrict__ bias,
                                                  float* __restrict__ Y, int ldy, int M, int N,
                                                  int K) {
  constexpr int NP = MODE == 0 ? 3 : 1;
  constexpr int FM = BM / 64, FN = BN / 64;
  constexpr int APL = BM * 64, WPL = BN * 64;     // bytes per plane image (64-B rows)
  constexpr int STAGE = NP * (APL + WPL);
  constexpr int CH = BM * 4 / 256;                // 16-B A chunks per thread per stage
  constexpr int WI = NP * BN / 16;                // 1-KB DMA pieces of W per stage
  static_assert(WI % 4 == 0, "W pieces split over 4 waves");
  __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];
  const int ntiles = (N + BN - 1) / BN;
  const int bid = xcd_contiguous(blockIdx.x, gridDim.x);
  const int mt = bid / ntiles, nt = bid - mt * ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int r = lane & 31, hh = lane >> 5;
  f16v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  float4 ra[CH][2];
  auto load_a = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int e = t + 256 * c, row = e >> 2, ch = e & 3;
      const float* p = A + (int64_t)min(m0 + row, M - 1) * lda + k0 + ch * 8;
      ra[c][0] = *reinterpret_cast<const float4*>(p);
      ra[c][1] = *reinterpret_cast<const float4*>(p + 4);
    }
  };
  auto store_a = [&](char* buf) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int e = t + 256 * c, row = e >> 2, ch = e & 3;
      const int off = row * 64 + ((ch ^ ((row >> 2) & 3)) << 4);
      if constexpr (MODE == 0) {
        bf16x8_t h, m, l;
        split8(ra[c][0], ra[c][1], h, m, l);
        *reinterpret_cast<bf16x8_t*>(buf + off) = h;
        *reinterpret_cast<bf16x8_t*>(buf + APL + off) = m;
        *reinterpret_cast<bf16x8_t*>(buf + 2 * APL + off) = l;
      } else {
        bf16x8_t h;
        const float x[8] = {ra[c][0].x, ra[c][0].y, ra[c][0].z, ra[c][0].w,
                            ra[c][1].x, ra[c][1].y, ra[c][1].z, ra[c][1].w};
#pragma unroll
        for (int j = 0; j < 8; ++j) h[j] = (__bf16)x[j];
        *reinterpret_cast<bf16x8_t*>(buf + off) = h;
      }
    }
  };
  auto dma_w = [&](int k0, char* buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < WI / 4; ++i) {
      const int j = wave + 4 * i;
      const int p = j / (BN / 16), rb = (j % (BN / 16)) * 16;
      const int row = rb + (lane >> 2), ch = (lane & 3) ^ ((row >> 2) & 3);
      const __bf16* src = Wp + p * wplane + (int64_t)min(n0 + row, N - 1) * ldw + k0 + ch * 8;
      char* dst = buf + NP * APL + p * WPL + rb * 64;
      __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
    }
  };
  auto compute = [&](const char* buf) __attribute__((always_inline)) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t fa[NP][FM], fw[NP][FN];
#pragma unroll
      for (int p = 0; p < NP; ++p) {
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int row = wm * (BM / 2) + i * 32 + r;
          const int off = row * 64 + (((2 * kk + hh) ^ ((row >> 2) & 3)) << 4);
          fa[p][i] = *reinterpret_cast<const bf16x8_t*>(buf + p * APL + off);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int row = wn * (BN / 2) + j * 32 + r;
          const int off = row * 64 + (((2 * kk + hh) ^ ((row >> 2) & 3)) << 4);
          fw[p][j] = *reinterpret_cast<const bf16x8_t*>(buf + NP * APL + p * WPL + off);
        }
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if constexpr (MODE == 0) {   // smallest terms first (as PM_SPLIT3)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2][i], fw[0][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fw[1][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fw[2][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fw[0][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fw[1][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fw[0][j], acc[i][j], 0, 0, 0);
          } else {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fw[0][j], acc[i][j], 0, 0, 0);
          }
        }
    }
  };
  const int nk = K / 32;
  char* b0 = lds;
  char* b1 = lds + STAGE;
  load_a(0);
  dma_w(0, b0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  store_a(b0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = (kt & 1) ? b1 : b0;
    char* nxt = (kt & 1) ? b0 : b1;
    const bool more = kt + 1 < nk;
    if (more) {
      load_a((kt + 1) * 32);
      dma_w((kt + 1) * 32, nxt);
    }
    compute(cur);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (more) store_a(nxt);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int gn = n0 + wn * (BN / 2) + j * 32 + r;
      if (gn >= N) continue;
      const float bv = bias[gn];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int gm = m0 + wm * (BM / 2) + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
        if (gm < M) Y[(int64_t)gm * ldy + gn] = acc[i][j][e] + bv;
      }
    }
}


// v2: W through a 3-stage LDS-DMA ring (issued two stages ahead), A through two register sets
// loaded by inline-asm global_load_dwordx4 (two stages ahead; hipcc does not count asm loads,
// so every wait is an explicit counted vmcnt), raw s_barrier (no vmcnt(0) drain).
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4v gload4(const float* p) {
  f4v v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// the wait also "defines" the registers of the set it retires, so no consumer of them can be
// scheduled above it (an asm load's result is otherwise available to the compiler at once)
template <int N, int CH>
__device__ __forceinline__ void wait_vm_set(f4v (&s)[CH][2]) {
  if constexpr (CH == 1) {
    asm volatile("s_waitcnt vmcnt(%2)" : "+v"(s[0][0]), "+v"(s[0][1]) : "n"(N) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(%4)"
                 : "+v"(s[0][0]), "+v"(s[0][1]), "+v"(s[1][0]), "+v"(s[1][1])
                 : "n"(N)
                 : "memory");
  }
}

template <int BM, int BN, int MODE>
__global__ __launch_bounds__(256) void split_gemm2(const float* __restrict__ A, int lda,
                                                   const __bf16* __restrict__ Wp, int64_t wplane,
                                                   int ldw, const float* __restrict__ bias,
                                                   float* __restrict__ Y, int ldy, int M, int N,
                                                   int K) {
  constexpr int NP = MODE == 0 ? 3 : 1;
  constexpr int FM = BM / 64, FN = BN / 64;
  constexpr int APL = BM * 64, WPL = BN * 64;
  constexpr int ASTAGE = NP * APL, WSTAGE = NP * WPL;
  constexpr int CH = BM * 4 / 256;
  constexpr int WI = NP * BN / 16;
  static_assert(WI % 4 == 0, "W pieces split over 4 waves");
  constexpr int VM_PER_STEP = 2 * CH + WI / 4;   // vector-memory ops one step issues per wave
  __shared__ __attribute__((aligned(16))) char lds[2 * ASTAGE + 3 * WSTAGE];
  char* abuf = lds;
  char* wring = lds + 2 * ASTAGE;
  const int ntiles = (N + BN - 1) / BN;
  const int bid = xcd_contiguous(blockIdx.x, gridDim.x);
  const int mt = bid / ntiles, nt = bid - mt * ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int r = lane & 31, hh = lane >> 5;
  f16v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  f4v ra[2][CH][2];
  auto load_a = [&](int k0, f4v (&dst)[CH][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int e = t + 256 * c, row = e >> 2, ch = e & 3;
      const float* p = A + (int64_t)min(m0 + row, M - 1) * lda + k0 + ch * 8;
      dst[c][0] = gload4(p);
      dst[c][1] = gload4(p + 4);
    }
  };
  auto store_a = [&](char* buf, const f4v (&src)[CH][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int e = t + 256 * c, row = e >> 2, ch = e & 3;
      const int off = row * 64 + ((ch ^ ((row >> 2) & 3)) << 4);
      if constexpr (MODE == 0) {
        bf16x8_t h, m, l;
        split8(make_float4(src[c][0][0], src[c][0][1], src[c][0][2], src[c][0][3]),
               make_float4(src[c][1][0], src[c][1][1], src[c][1][2], src[c][1][3]), h, m, l);
        *reinterpret_cast<bf16x8_t*>(buf + off) = h;
        *reinterpret_cast<bf16x8_t*>(buf + APL + off) = m;
        *reinterpret_cast<bf16x8_t*>(buf + 2 * APL + off) = l;
      } else {
        bf16x8_t h;
        const float x[8] = {src[c][0][0], src[c][0][1], src[c][0][2], src[c][0][3],
                            src[c][1][0], src[c][1][1], src[c][1][2], src[c][1][3]};
#pragma unroll
        for (int j = 0; j < 8; ++j) h[j] = (__bf16)x[j];
        *reinterpret_cast<bf16x8_t*>(buf + off) = h;
      }
    }
  };
  auto dma_w = [&](int k0, char* buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < WI / 4; ++i) {
      const int j = wave + 4 * i;
      const int p = j / (BN / 16), rb = (j % (BN / 16)) * 16;
      const int row = rb + (lane >> 2), ch = (lane & 3) ^ ((row >> 2) & 3);
      const __bf16* src = Wp + p * wplane + (int64_t)min(n0 + row, N - 1) * ldw + k0 + ch * 8;
      __builtin_amdgcn_global_load_lds(src, buf + p * WPL + rb * 64, 16, 0, 0);
    }
  };
  auto compute = [&](const char* ab, const char* wb) __attribute__((always_inline)) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t fa[NP][FM], fw[NP][FN];
#pragma unroll
      for (int p = 0; p < NP; ++p) {
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int row = wm * (BM / 2) + i * 32 + r;
          const int off = row * 64 + (((2 * kk + hh) ^ ((row >> 2) & 3)) << 4);
          fa[p][i] = *reinterpret_cast<const bf16x8_t*>(ab + p * APL + off);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int row = wn * (BN / 2) + j * 32 + r;
          const int off = row * 64 + (((2 * kk + hh) ^ ((row >> 2) & 3)) << 4);
          fw[p][j] = *reinterpret_cast<const bf16x8_t*>(wb + p * WPL + off);
        }
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if constexpr (MODE == 0) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2][i], fw[0][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fw[1][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fw[2][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fw[0][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fw[1][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fw[0][j], acc[i][j], 0, 0, 0);
          } else {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fw[0][j], acc[i][j], 0, 0, 0);
          }
        }
    }
  };
  const int nk = K / 32;   // >= 2
  // prologue: stages 0 and 1 in flight; stage 0 split into A buffer 0
  load_a(0, ra[0]);
  dma_w(0, wring);
  load_a(32, ra[1]);
  dma_w(32, wring + WSTAGE);
  wait_vm_set<VM_PER_STEP>(ra[0]);   // stage 0 landed (stage 1 may still be in flight)
  store_a(abuf, ra[0]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nk; ++kt) {
    const bool pre = kt + 2 < nk;   // wave-uniform
    if (pre) {
      if (kt & 1) load_a((kt + 2) * 32, ra[1]);
      else load_a((kt + 2) * 32, ra[0]);
      dma_w((kt + 2) * 32, wring + ((kt + 2) % 3) * WSTAGE);
    }
    compute(abuf + (kt & 1) * ASTAGE, wring + (kt % 3) * WSTAGE);
    if (kt + 1 < nk) {   // stage kt + 1 landed: its A registers are set (kt + 1) & 1
      if (kt & 1) {
        if (pre) wait_vm_set<VM_PER_STEP>(ra[0]); else wait_vm_set<0>(ra[0]);
        store_a(abuf, ra[0]);
      } else {
        if (pre) wait_vm_set<VM_PER_STEP>(ra[1]); else wait_vm_set<0>(ra[1]);
        store_a(abuf + ASTAGE, ra[1]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int gn = n0 + wn * (BN / 2) + j * 32 + r;
      if (gn >= N) continue;
      const float bv = bias[gn];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int gm = m0 + wm * (BM / 2) + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
        if (gm < M) Y[(int64_t)gm * ldy + gn] = acc[i][j][e] + bv;
      }
    }
}

template <int BM, int BN, int MODE>
float time_split2(const float* A, const __bf16* Wp, int64_t wplane, const float* bias, float* Y,
                  int M, int N, int K, int iters) {
  const int grid = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w)
    hipLaunchKernelGGL((split_gemm2<BM, BN, MODE>), dim3(grid), dim3(256), 0, 0, A, K, Wp, wplane, K,
                       bias, Y, N, M, N, K);
  hipEventRecord(e0);
  for (int it = 0; it < iters; ++it)
    hipLaunchKernelGGL((split_gemm2<BM, BN, MODE>), dim3(grid), dim3(256), 0, 0, A, K, Wp, wplane, K,
                       bias, Y, N, M, N, K);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / iters;
}

// host split of W into three bf16 planes (round to nearest even, exact residuals)
static uint16_t bf16_bits(float x) {
  uint32_t u;
  memcpy(&u, &x, 4);
  const uint32_t lsb = (u >> 16) & 1u;
  u += 0x7fffu + lsb;
  return (uint16_t)(u >> 16);
}
static float bf16_float(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

template <int BM, int BN, int MODE>
float time_split(const float* A, const __bf16* Wp, int64_t wplane, const float* bias, float* Y,
                 int M, int N, int K, int iters) {
  const int grid = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w)
    hipLaunchKernelGGL((split_gemm<BM, BN, MODE>), dim3(grid), dim3(256), 0, 0, A, K, Wp, wplane, K,
                       bias, Y, N, M, N, K);
  hipEventRecord(e0);
  for (int it = 0; it < iters; ++it)
    hipLaunchKernelGGL((split_gemm<BM, BN, MODE>), dim3(grid), dim3(256), 0, 0, A, K, Wp, wplane, K,
                       bias, Y, N, M, N, K);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / iters;
}

float time_f32(float* A, float* W, float* Y, float* bias, int M, int N, int K, int iters) {
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.nprob = 1;
  GemmProb& p = a.p[0];
  p = gemm_prob(A, K, W, K, bias, Y, N, M, N, K, 1);
  p.mtiles = (M + 63) / 64;
  p.ntiles = (N + 63) / 64;
  p.tiles = p.mtiles * p.ntiles;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) launch_one<EPI_BIAS, PRO_PLAIN, T64x64, PM_F32>(a, p.tiles, nullptr);
  hipEventRecord(e0);
  for (int it = 0; it < iters; ++it) launch_one<EPI_BIAS, PRO_PLAIN, T64x64, PM_F32>(a, p.tiles, nullptr);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / iters;
}

// the production gemm.hip kernels in the split mode with W planes (DMA loop), by epilogue
template <int EPI, int PRO, int PM, bool DMA>
float time_prod(float* A, const __bf16* Wp, int64_t wplane, float* bias, float* Y, int M, int N,
                int K, int iters, float* stats, unsigned* cnt, float* mean, float* rstd,
                float* ksum) {
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.nprob = 1;
  GemmProb& p = a.p[0];
  p = gemm_prob(A, K, nullptr, K, bias, Y, N, M, N, K, 1);
  p.Wp = reinterpret_cast<const uint16_t*>(Wp);
  p.wpl = wplane;
  p.stats = stats;
  p.st_cnt = cnt;
  p.st_mean = mean;
  p.st_rstd = rstd;
  if (PRO == PRO_HEADZ) {   // K = [x (256) | phi(q) (256)], the second range from the same A
    p.ksplit = 256;
    p.A1 = A + 256;
    p.lda1 = K;
    p.ksum = ksum;
    p.ns = 4096.f;
  }
  p.mtiles = (M + 63) / 64;
  p.ntiles = (N + 63) / 64;
  p.tiles = p.mtiles * p.ntiles;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) {
    if (cnt) hipMemset(cnt, 0, 4096);
    launch_one<EPI, PRO, T64x64, PM, true, DMA>(a, p.tiles, nullptr);
  }
  float tot = 0.f;
  for (int it = 0; it < iters; ++it) {
    if (cnt) hipMemsetAsync(cnt, 0, 4096);
    hipEventRecord(e0);
    launch_one<EPI, PRO, T64x64, PM, true, DMA>(a, p.tiles, nullptr);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    tot += ms;
  }
  return tot * 1e3f / iters;
}

int main(int argc, char** argv) {
  const int N = 512, K = 512;
  const int Ms[] = {5120, 10240, 16384 + 1024, 32 * 17408 / 8};
  srand(1);
  const int MMAX = 70000;
  std::vector<float> hA((size_t)MMAX * K), hW((size_t)N * K), hb(N);
  for (auto& x : hA) x = (float)rand() / RAND_MAX * 2.f - 1.f;
  for (auto& x : hW) x = ((float)rand() / RAND_MAX * 2.f - 1.f) * 0.05f;
  for (auto& x : hb) x = (float)rand() / RAND_MAX - 0.5f;
  std::vector<uint16_t> planes((size_t)3 * N * K);
  for (size_t i = 0; i < (size_t)N * K; ++i) {
    const float x = hW[i];
    const uint16_t h = bf16_bits(x);
    const float rr = x - bf16_float(h);
    const uint16_t m = bf16_bits(rr);
    const uint16_t l = bf16_bits(rr - bf16_float(m));
    planes[i] = h;
    planes[(size_t)N * K + i] = m;
    planes[(size_t)2 * N * K + i] = l;
  }
  float *A, *W, *b, *Y, *Y2;
  __bf16* Wp;
  hipMalloc(&A, hA.size() * 4);
  hipMalloc(&W, hW.size() * 4);
  hipMalloc(&b, N * 4);
  hipMalloc(&Y, (size_t)MMAX * N * 4);
  hipMalloc(&Y2, (size_t)MMAX * N * 4);
  hipMalloc(&Wp, planes.size() * 2);
  hipMemcpy(A, hA.data(), hA.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(W, hW.data(), hW.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(b, hb.data(), N * 4, hipMemcpyHostToDevice);
  hipMemcpy(Wp, planes.data(), planes.size() * 2, hipMemcpyHostToDevice);
  const int64_t wpl = (int64_t)N * K;
  // correctness at M = 5120: split vs fp32 MFMA vs fp64 on sampled entries
  {
    const int M = 5120;
    time_f32(A, W, Y, b, M, N, K, 1);
    time_split<64, 128, 0>(A, Wp, wpl, b, Y2, M, N, K, 1);
    std::vector<float> y1((size_t)M * N), y2((size_t)M * N);
    hipMemcpy(y1.data(), Y, y1.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(y2.data(), Y2, y2.size() * 4, hipMemcpyDeviceToHost);
    double e1 = 0, e2 = 0, d12 = 0;
    for (int s = 0; s < 4000; ++s) {
      const int i = (s * 7919) % M, j = (s * 104729) % N;
      double ref = hb[j];
      for (int k = 0; k < K; ++k) ref += (double)hA[(size_t)i * K + k] * hW[(size_t)j * K + k];
      e1 = fmax(e1, fabs(y1[(size_t)i * N + j] - ref));
      e2 = fmax(e2, fabs(y2[(size_t)i * N + j] - ref));
    }
    for (size_t i = 0; i < y1.size(); ++i) d12 = fmax(d12, fabs(y1[i] - y2[i]));
    printf("max |err| vs fp64: fp32-MFMA %.3g  split3(64x128) %.3g   max |fp32 - split3| %.3g\n", e1,
           e2, d12);
    time_split<128, 128, 0>(A, Wp, wpl, b, Y2, M, N, K, 1);
    hipMemcpy(y2.data(), Y2, y2.size() * 4, hipMemcpyDeviceToHost);
    d12 = 0;
    for (size_t i = 0; i < y1.size(); ++i) d12 = fmax(d12, fabs(y1[i] - y2[i]));
    printf("max |fp32 - split3(128x128)| %.3g\n", d12);
    time_split<64, 64, 0>(A, Wp, wpl, b, Y2, M, N, K, 1);
    hipMemcpy(y2.data(), Y2, y2.size() * 4, hipMemcpyDeviceToHost);
    d12 = 0;
    for (size_t i = 0; i < y1.size(); ++i) d12 = fmax(d12, fabs(y1[i] - y2[i]));
    printf("max |fp32 - split3(64x64)| %.3g\n", d12);
    time_split<64, 128, 1>(A, Wp, wpl, b, Y2, M, N, K, 1);
    hipMemcpy(y2.data(), Y2, y2.size() * 4, hipMemcpyDeviceToHost);
    d12 = 0;
    for (size_t i = 0; i < y1.size(); ++i) d12 = fmax(d12, fabs(y1[i] - y2[i]));
    printf("max |fp32 - bf16(64x128)| %.3g\n", d12);
    time_split2<64, 128, 0>(A, Wp, wpl, b, Y2, M, N, K, 1);
    hipMemcpy(y2.data(), Y2, y2.size() * 4, hipMemcpyDeviceToHost);
    d12 = 0;
    for (size_t i = 0; i < y1.size(); ++i) d12 = fmax(d12, fabs(y1[i] - y2[i]));
    printf("v2: max |fp32 - split3(64x128)| %.3g\n", d12);
    time_split2<64, 64, 0>(A, Wp, wpl, b, Y2, M, N, K, 1);
    hipMemcpy(y2.data(), Y2, y2.size() * 4, hipMemcpyDeviceToHost);
    d12 = 0;
    for (size_t i = 0; i < y1.size(); ++i) d12 = fmax(d12, fabs(y1[i] - y2[i]));
    printf("v2: max |fp32 - split3(64x64)| %.3g\n", d12);
  }
  {
    float *stats, *mean, *rstd, *ksum;
    unsigned* cnt;
    hipMalloc(&stats, 8 << 20);
    hipMalloc(&mean, 4096);
    hipMalloc(&rstd, 4096);
    hipMalloc(&ksum, 4096);
    hipMalloc(&cnt, 4096);
    std::vector<float> ks(1024, 30.f);
    hipMemcpy(ksum, ks.data(), 4096, hipMemcpyHostToDevice);
    const int M = 5120, it = 30;
    printf("production kernels, M 5120 N 512 K 512, per-launch events (serial):\n");
    printf("  fp32 BIAS              %7.2f us\n", time_f32(A, W, Y, b, M, N, K, it));
    printf("  split DMA BIAS         %7.2f us\n", time_prod<EPI_BIAS, PRO_PLAIN, PM_SPLIT3, true>(A, Wp, wpl, b, Y, M, N, K, it, stats, nullptr, mean, rstd, ksum));
    printf("  split DMA STATS        %7.2f us\n", time_prod<EPI_STATS, PRO_PLAIN, PM_SPLIT3, true>(A, Wp, wpl, b, Y, M, N, K, it, stats, nullptr, mean, rstd, ksum));
    printf("  split DMA STATS+fin    %7.2f us\n", time_prod<EPI_STATS, PRO_PLAIN, PM_SPLIT3, true>(A, Wp, wpl, b, Y, M, N, K, it, stats, cnt, mean, rstd, ksum));
    printf("  split DMA STATS+HEADZ  %7.2f us\n", time_prod<EPI_STATS, PRO_HEADZ, PM_SPLIT3, true>(A, Wp, wpl, b, Y, M, N, K, it, stats, cnt, mean, rstd, ksum));
    printf("  split reg STATS+HEADZ  %7.2f us\n", time_prod<EPI_STATS, PRO_HEADZ, PM_SPLIT3, false>(A, Wp, wpl, b, Y, M, N, K, it, stats, cnt, mean, rstd, ksum));
    printf("  bf16 DMA STATS+HEADZ   %7.2f us\n", time_prod<EPI_STATS, PRO_HEADZ, PM_BF16, true>(A, Wp, wpl, b, Y, M, N, K, it, stats, cnt, mean, rstd, ksum));
    printf("  bf16 reg STATS+HEADZ   %7.2f us\n", time_prod<EPI_STATS, PRO_HEADZ, PM_BF16, false>(A, Wp, wpl, b, Y, M, N, K, it, stats, cnt, mean, rstd, ksum));
  }
  for (int M : Ms) {
    const double gf = 2.0 * M * N * K * 1e-9;
    const int it = 50;
    const float f = time_f32(A, W, Y, b, M, N, K, it);
    const float s1 = time_split<64, 64, 0>(A, Wp, wpl, b, Y2, M, N, K, it);
    const float s2 = time_split<64, 128, 0>(A, Wp, wpl, b, Y2, M, N, K, it);
    const float s3 = time_split<128, 128, 0>(A, Wp, wpl, b, Y2, M, N, K, it);
    const float q1 = time_split<64, 128, 1>(A, Wp, wpl, b, Y2, M, N, K, it);
    const float q2 = time_split<128, 128, 1>(A, Wp, wpl, b, Y2, M, N, K, it);
    printf("M %6d: fp32-64x64 %7.2f us (%5.1f TF) | split3 64x64 %7.2f (%5.1f) 64x128 %7.2f (%5.1f) "
           "128x128 %7.2f (%5.1f) | bf16 64x128 %7.2f (%5.1f) 128x128 %7.2f (%5.1f)\n",
           M, f, gf / f * 1e3, s1, gf / s1 * 1e3, s2, gf / s2 * 1e3, s3, gf / s3 * 1e3, q1, gf / q1 * 1e3,
           q2, gf / q2 * 1e3);
    const float v1 = time_split2<64, 64, 0>(A, Wp, wpl, b, Y2, M, N, K, it);
    const float v2 = time_split2<64, 128, 0>(A, Wp, wpl, b, Y2, M, N, K, it);
    const float v3 = time_split2<128, 64, 0>(A, Wp, wpl, b, Y2, M, N, K, it);
    const float w1 = time_split2<64, 128, 1>(A, Wp, wpl, b, Y2, M, N, K, it);
    const float w2 = time_split2<128, 128, 1>(A, Wp, wpl, b, Y2, M, N, K, it);
    printf("   v2 split3 64x64 %7.2f (%5.1f) 64x128 %7.2f (%5.1f) 128x64 %7.2f (%5.1f) | bf16 64x128 %7.2f (%5.1f) 128x128 %7.2f (%5.1f)\n",
           v1, gf / v1 * 1e3, v2, gf / v2 * 1e3, v3, gf / v3 * 1e3, w1, gf / w1 * 1e3, w2, gf / w2 * 1e3);
  }
  return 0;
}
