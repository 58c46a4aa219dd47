// GATsSPG matcher forward on gfx950 (GATsSuperGlue.forward, GATs_SuperGlue.py:203-278).
//
// Data layout in HBM (per batch sample, fp32):
//   X2 [N1][256], X3 [N3][256]       token-major descriptors (ping-pong buffers)
//   QKV [N][768]                     phi(q) | phi(k) | v/Ns, channels head-major (h*64+d)
//   KVt [h][q][d], ksum [h*64+d]     linear-attention state of one source tensor
//   O, MSG [N][256], Y1 [N][512]     attention output, merged message, MLP hidden
//   S/conf [N1][N3]                  score matrix, overwritten in place by conf_matrix
// The reference's [B, C, N] inputs are transposed once on entry; the leaf descriptors
// ([B, 256, N3*L], per-object constants, 33.5 MB at N3=4096) are read in place by the
// GAT kernel and never copied.
//
// Layer schedule (AttentionalGNN.forward, GATs_SuperGlue.py:67-85): for each of the 12
// layers, GAT layers update X3 only; self/cross layers run both sides in the same
// launches (two problems per grid) because delta0 and delta1 both read the pre-update
// descriptors (:77-78, :82-83).
#include <cmath>
#include <cstdarg>
#include <cstring>
#include <vector>

#include "gemm.h"

namespace onepose {

// ------------------------------------------------------------------------------------
// errors
// ------------------------------------------------------------------------------------
static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}
void clear_error() { g_last_error.clear(); }

// ------------------------------------------------------------------------------------
// launch profiling
// ------------------------------------------------------------------------------------
namespace {
struct Prof {
  uint64_t mask = 0;
  std::vector<hipEvent_t> ev;
  std::vector<int> kinds;
  int n = 0;
};
Prof g_prof;
const char* kKindNames[K_NUM_KINDS] = {
    "transpose_in", "gat", "qkv_gemm", "kv_partial", "kv_reduce", "attn_apply", "merge_gemm",
    "mlp1_gemm", "stats_finalize", "mlp2_gemm", "final_gemm", "l2norm", "score_gemm",
    "softmax_reduce", "conf", "mutual", "select", "pnp_ransac", "pose_error", "sample_desc",
    "pnp_refit"};
}  // namespace

void prof_pre(int kind, hipStream_t s) {
  if (!((g_prof.mask >> kind) & 1ull) || 2 * g_prof.n + 1 >= (int)g_prof.ev.size()) return;
  hipEventRecord(g_prof.ev[2 * g_prof.n], s);
}
void prof_post(int kind, hipStream_t s) {
  if (!((g_prof.mask >> kind) & 1ull) || 2 * g_prof.n + 1 >= (int)g_prof.ev.size()) return;
  hipEventRecord(g_prof.ev[2 * g_prof.n + 1], s);
  g_prof.kinds[g_prof.n] = kind;
  ++g_prof.n;
}

// ------------------------------------------------------------------------------------
// weight packing (host)
// ------------------------------------------------------------------------------------
namespace {

constexpr int kLayers = 12;
constexpr int kApLayers = 8;
constexpr int kGatLayers = 4;

// packed panel, floats
constexpr int64_t kApWqkv = 768 * 256, kApBqkv = 768, kApWm = 256 * 256, kApBm = 256;
constexpr int64_t kApW1 = 512 * 512, kApB1 = 512, kApW2 = 256 * 512, kApB2 = 256;
constexpr int64_t kApFloats = kApWqkv + kApBqkv + kApWm + kApBm + kApW1 + kApB1 + kApW2 + kApB2;
constexpr int64_t kGatFloats = 512;
constexpr int64_t kFinalFloats = 256 * 256 + 256;
constexpr int64_t kPackedFloats = kApLayers * kApFloats + kGatLayers * kGatFloats + kFinalFloats;

struct ApW {
  const float *wqkv, *bqkv, *wm, *bm, *w1, *b1, *w2, *b2;
};
ApW ap_weights(const float* base, int ap) {
  const float* p = base + (int64_t)ap * kApFloats;
  ApW w;
  w.wqkv = p; p += kApWqkv;
  w.bqkv = p; p += kApBqkv;
  w.wm = p; p += kApWm;
  w.bm = p; p += kApBm;
  w.w1 = p; p += kApW1;
  w.b1 = p; p += kApB1;
  w.w2 = p; p += kApW2;
  w.b2 = p;
  return w;
}
const float* gat_weights(const float* base, int g) {
  return base + kApLayers * kApFloats + (int64_t)g * kGatFloats;
}
const float* final_weights(const float* base) {
  return base + kApLayers * kApFloats + kGatLayers * kGatFloats;
}

struct TensorSpec {
  std::string name;
  int64_t numel;
};

const std::vector<TensorSpec>& tensor_specs() {
  static std::vector<TensorSpec> specs = [] {
    std::vector<TensorSpec> s;
    for (int i = 0; i < kLayers; ++i) {
      std::string p = "gnn.layers." + std::to_string(i) + ".";
      if (i % 3 == 0) {
        s.push_back({p + "W", 256 * 256});
        s.push_back({p + "a", 512});
      } else {
        for (int j = 0; j < 3; ++j) {
          s.push_back({p + "attn.proj." + std::to_string(j) + ".weight", 256 * 256});
          s.push_back({p + "attn.proj." + std::to_string(j) + ".bias", 256});
        }
        s.push_back({p + "attn.merge.weight", 256 * 256});
        s.push_back({p + "attn.merge.bias", 256});
        s.push_back({p + "mlp.0.weight", 512 * 512});
        s.push_back({p + "mlp.0.bias", 512});
        s.push_back({p + "mlp.3.weight", 256 * 512});
        s.push_back({p + "mlp.3.bias", 256});
      }
    }
    s.push_back({"final_proj.weight", 256 * 256});
    s.push_back({"final_proj.bias", 256});
    return s;
  }();
  return specs;
}

}  // namespace

// ------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------

// [B][256][N] (batch stride `bs`, may be 0) -> [B][N][256]
__global__ __launch_bounds__(256) void transpose_in_kernel(const float* __restrict__ src,
                                                           int64_t bs, int n,
                                                           float* __restrict__ dst) {
  __shared__ float tile[64][65];
  const int n0 = blockIdx.x * 64, c0 = blockIdx.y * 64, b = blockIdx.z;
  const float* s = src + b * bs;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int nn = n0 + tx;
    tile[r][tx] = (nn < n) ? s[(int64_t)(c0 + r) * n + nn] : 0.f;
  }
  __syncthreads();
  float* d = dst + (int64_t)b * n * kDim;
  for (int r = ty; r < 64; r += 4) {
    const int nn = n0 + r;
    if (nn < n) d[(int64_t)nn * kDim + c0 + tx] = tile[tx][r];
  }
}

// Linear-attention source reduction, one 64-token chunk per workgroup, one head per wave:
//   KVpart[h][d][q] = sum_m phi(k)[m][h,d] * v[m][h,q]      (einsum 'bdhm,bqhm->bqdh', :96)
//   kspart[h*64+d]  = sum_m phi(k)[m][h,d]                 (key.sum(3), :97)
// The chunk's phi(k)|v rows (2 KB contiguous per token) are staged into LDS 32 tokens at a
// time with 16-byte loads; v_mfma_f32_32x32x2_f32 then runs with the token as the K
// dimension straight out of LDS (32 consecutive lanes read 32 consecutive channels).
struct KvProb {
  const float* qkv;   // [B][N][768]
  float* part;        // [B][chunks][4][64][64]
  float* kspart;      // [B][chunks][256]
  int n, chunks, blocks;
};
struct KvArgs {
  KvProb p[2];
};

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kKvStage = 32;   // tokens per LDS stage

__global__ __launch_bounds__(256) void kv_partial_kernel(KvArgs args) {
  __shared__ __attribute__((aligned(16))) float stage[kKvStage * 512];
  int bid = blockIdx.x;
  const bool second = bid >= args.p[0].blocks;
  const KvProb& P = second ? args.p[1] : args.p[0];
  if (second) bid -= args.p[0].blocks;
  const int b = bid / P.chunks, chunk = bid - b * P.chunks;
  const int t = threadIdx.x, lane = t & 63, h = t >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  const float* base = P.qkv + (int64_t)b * P.n * 768;
  const int m_begin = chunk * 64;

  floatx16 acc00, acc01, acc10, acc11;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc00[i] = acc01[i] = acc10[i] = acc11[i] = 0.f;
  float ks0 = 0.f, ks1 = 0.f;
  for (int s0 = 0; s0 < 64; s0 += kKvStage) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kKvStage * 128 / 256; ++i) {   // 32 rows x 128 float4
      const int e = t + 256 * i, r = e >> 7, c4 = e & 127;
      const int tok = m_begin + s0 + r;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (tok < P.n) v = *reinterpret_cast<const float4*>(base + (int64_t)tok * 768 + 256 + c4 * 4);
      *reinterpret_cast<float4*>(stage + r * 512 + c4 * 4) = v;
    }
    __syncthreads();
    const float* ka = stage + h * 64 + l32;
    const float* va = stage + 256 + h * 64 + l32;
#pragma unroll 4
    for (int k = 0; k < kKvStage; k += 2) {
      const int r = (k + half) * 512;
      const float a0 = ka[r], a1 = ka[r + 32], v0 = va[r], v1 = va[r + 32];
      ks0 += a0;
      ks1 += a1;
      acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, v0, acc00, 0, 0, 0);
      acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, v1, acc01, 0, 0, 0);
      acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, v0, acc10, 0, 0, 0);
      acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, v1, acc11, 0, 0, 0);
    }
  }
  float* out = P.part + ((int64_t)b * P.chunks + chunk) * 16384 + h * 4096;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int d = (i & 3) + 8 * (i >> 2) + 4 * half;
    out[d * 64 + l32] = acc00[i];
    out[d * 64 + 32 + l32] = acc01[i];
    out[(d + 32) * 64 + l32] = acc10[i];
    out[(d + 32) * 64 + 32 + l32] = acc11[i];
  }
  ks0 += __shfl_xor(ks0, 32, 64);
  ks1 += __shfl_xor(ks1, 32, 64);
  if (half == 0) {
    float* ko = P.kspart + ((int64_t)b * P.chunks + chunk) * 256 + h * 64;
    ko[l32] = ks0;
    ko[32 + l32] = ks1;
  }
}

// Sum the chunk partials -> KV[h][d][q], ksum[256], one float4 of outputs per thread with
// eight chunk loads in flight; the summation order is fixed (deterministic).
__global__ __launch_bounds__(256) void kv_reduce_kernel(KvArgs args, float* kv, float* ksum,
                                                        int batch) {
  constexpr int per = (16384 + 256) / 4;   // float4 outputs per (source, sample)
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= 2 * batch * per) return;
  const int src = idx / (batch * per);
  const int r = idx - src * batch * per;
  const int b = r / per, e4 = r - b * per;
  const KvProb& P = src ? args.p[1] : args.p[0];
  const float4* p;
  int64_t stride;
  float4* out;
  if (e4 < 4096) {
    p = reinterpret_cast<const float4*>(P.part + (int64_t)b * P.chunks * 16384) + e4;
    stride = 4096;
    out = reinterpret_cast<float4*>(kv + ((int64_t)src * batch + b) * 16384) + e4;
  } else {
    p = reinterpret_cast<const float4*>(P.kspart + (int64_t)b * P.chunks * 256) + (e4 - 4096);
    stride = 64;
    out = reinterpret_cast<float4*>(ksum + ((int64_t)src * batch + b) * 256) + (e4 - 4096);
  }
  float4 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  int c = 0;
  for (; c + 8 <= P.chunks; c += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float4 v = p[(int64_t)(c + j) * stride];
      acc[j].x += v.x; acc[j].y += v.y; acc[j].z += v.z; acc[j].w += v.w;
    }
  }
  float4 tail = make_float4(0.f, 0.f, 0.f, 0.f);
  for (; c < P.chunks; ++c) {
    const float4 v = p[(int64_t)c * stride];
    tail.x += v.x; tail.y += v.y; tail.z += v.z; tail.w += v.w;
  }
  float4 s = acc[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) { s.x += acc[j].x; s.y += acc[j].y; s.z += acc[j].z; s.w += acc[j].w; }
  s.x += tail.x; s.y += tail.y; s.z += tail.z; s.w += tail.w;
  *out = s;
}

// Linear-attention apply (GATs_SuperGlue.py:97-98):
//   Z[n,h]   = 1 / (sum_d phi(q)[n][h,d] * ksum[h,d] + 1e-6)
//   O[n][h*64+q] = (sum_d phi(q)[n][h,d] * KV[h][d][q]) * Z[n,h] * Ns
// One 64-token tile per workgroup, one head per wave.  phi(q) tile [64][256] and the four
// 64x64 KV blocks (transposed to [h][q][d]) are staged in LDS (pitches 260 / 68 floats:
// conflict-free ds_read_b128), then 2x2 32x32 MFMA accumulators per wave.
struct ApplyProb {
  const float* qkv;    // query side [B][Nq][768] (phi(q) in columns 0..255)
  const float* kv;     // source [B][4][64 d][64 q]
  const float* ksum;   // source [B][256]
  float* out;          // [B][Nq][256]
  int nq;
  float ns;            // source length (v_length)
  int mtiles, blocks;
};
struct ApplyArgs {
  ApplyProb p[2];
};
constexpr int kQPitch = 260, kKvPitch = 68;
constexpr size_t kApplyLds = (64 * kQPitch + 4 * 64 * kKvPitch + 4 * 64) * sizeof(float);

__global__ __launch_bounds__(256) void attn_apply_kernel(ApplyArgs args) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* qs = sm;                          // [64][260]
  float* kvs = qs + 64 * kQPitch;          // [4][64 q][68]
  float* zs = kvs + 4 * 64 * kKvPitch;     // [4][64]
  int bid = blockIdx.x;
  const bool second = bid >= args.p[0].blocks;
  const ApplyProb& P = second ? args.p[1] : args.p[0];
  if (second) bid -= args.p[0].blocks;
  const int b = bid / P.mtiles, mt = bid - b * P.mtiles;
  const int m0 = mt * 64;
  const int t = threadIdx.x, lane = t & 63, h = t >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  const float* q = P.qkv + (int64_t)b * P.nq * 768;
  const float* kvg = P.kv + (int64_t)b * 16384;
  const float* ks = P.ksum + (int64_t)b * 256;
#pragma unroll
  for (int i = 0; i < 16; ++i) {   // phi(q) tile: 64 rows x 64 float4
    const int e = t + 256 * i, r = e >> 6, c4 = e & 63;
    const int tok = m0 + r;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tok < P.nq) v = *reinterpret_cast<const float4*>(q + (int64_t)tok * 768 + c4 * 4);
    *reinterpret_cast<float4*>(qs + r * kQPitch + c4 * 4) = v;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {   // KV[h][d][q] -> kvs[h][q][d]
    const int e = t + 256 * i;     // float4 index over [4][64][16]
    const int hh = e >> 10, d = (e >> 4) & 63, q4 = e & 15;
    const float4 v = *reinterpret_cast<const float4*>(kvg + hh * 4096 + d * 64 + q4 * 4);
    float* o = kvs + hh * 64 * kKvPitch + (q4 * 4) * kKvPitch + d;
    o[0] = v.x;
    o[kKvPitch] = v.y;
    o[2 * kKvPitch] = v.z;
    o[3 * kKvPitch] = v.w;
  }
  __syncthreads();
  {  // Z for token `lane`, head h
    const float* row = qs + lane * kQPitch + h * 64;
    float s = 0.f;
#pragma unroll 4
    for (int d = 0; d < 64; d += 4) {
      const float4 a = *reinterpret_cast<const float4*>(row + d);
      const float4 k = *reinterpret_cast<const float4*>(ks + h * 64 + d);
      s += a.x * k.x;
      s += a.y * k.y;
      s += a.z * k.z;
      s += a.w * k.w;
    }
    zs[h * 64 + lane] = 1.0f / (s + 1e-6f);
  }
  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[0][0][i] = acc[0][1][i] = acc[1][0][i] = acc[1][1][i] = 0.f;
  const float* qa0 = qs + l32 * kQPitch + h * 64 + half * 4;
  const float* qa1 = qa0 + 32 * kQPitch;
  const float* kb0 = kvs + h * 64 * kKvPitch + l32 * kKvPitch + half * 4;
  const float* kb1 = kb0 + 32 * kKvPitch;
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const float4 a0 = *reinterpret_cast<const float4*>(qa0 + kk * 8);
    const float4 a1 = *reinterpret_cast<const float4*>(qa1 + kk * 8);
    const float4 b0 = *reinterpret_cast<const float4*>(kb0 + kk * 8);
    const float4 b1 = *reinterpret_cast<const float4*>(kb1 + kk * 8);
#define MF(ACC, A, B) ACC = __builtin_amdgcn_mfma_f32_32x32x2f32(A, B, ACC, 0, 0, 0)
    MF(acc[0][0], a0.x, b0.x); MF(acc[0][0], a0.y, b0.y); MF(acc[0][0], a0.z, b0.z); MF(acc[0][0], a0.w, b0.w);
    MF(acc[0][1], a0.x, b1.x); MF(acc[0][1], a0.y, b1.y); MF(acc[0][1], a0.z, b1.z); MF(acc[0][1], a0.w, b1.w);
    MF(acc[1][0], a1.x, b0.x); MF(acc[1][0], a1.y, b0.y); MF(acc[1][0], a1.z, b0.z); MF(acc[1][0], a1.w, b0.w);
    MF(acc[1][1], a1.x, b1.x); MF(acc[1][1], a1.y, b1.y); MF(acc[1][1], a1.z, b1.z); MF(acc[1][1], a1.w, b1.w);
#undef MF
  }
  __syncthreads();
  float* o = P.out + (int64_t)b * P.nq * 256 + h * 64;
#pragma unroll
  for (int tb = 0; tb < 2; ++tb) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = tb * 32 + (i & 3) + 8 * (i >> 2) + 4 * half;
      const int tok = m0 + row;
      if (tok < P.nq) {
        const float z = zs[h * 64 + row];
        o[(int64_t)tok * 256 + l32] = acc[tb][0][i] * z * P.ns;
        o[(int64_t)tok * 256 + 32 + l32] = acc[tb][1][i] * z * P.ns;
      }
    }
  }
}

// InstanceNorm1d statistics (GATs_SuperGlue.py:145; biased variance, eps 1e-5): combine the
// per-64-row-tile (mean, M2) partials (Chan et al., double).  One workgroup per (side,
// sample, 64-channel group); four tile-interleaved partial combines per channel, merged in
// a fixed order.
struct StatsProb {
  const float* part;  // [B][mtiles][2][512]
  float* mean;        // [B][512]
  float* rstd;
  int m, mtiles;
};
struct StatsArgs {
  StatsProb p[2];
};
__device__ __forceinline__ void chan_merge(double& n, double& mean, double& m2, double nb,
                                           double mb, double m2b) {
  if (nb == 0.0) return;
  const double nn = n + nb;
  const double delta = mb - mean;
  mean += delta * (nb / nn);
  m2 += m2b + delta * delta * (n * nb / nn);
  n = nn;
}
__global__ __launch_bounds__(256) void stats_finalize_kernel(StatsArgs args, int batch) {
  __shared__ double red[3][4][64];
  const int g = blockIdx.x & 7, b = (blockIdx.x >> 3) % batch, side = (blockIdx.x >> 3) / batch;
  const StatsProb& P = side ? args.p[1] : args.p[0];
  const int t = threadIdx.x, tg = t >> 6, c = g * 64 + (t & 63);
  const float* part = P.part + (int64_t)b * P.mtiles * 1024;
  double n = 0.0, mean = 0.0, m2 = 0.0;
  for (int ti = tg; ti < P.mtiles; ti += 4) {
    const double nb = (double)min(64, P.m - ti * 64);
    chan_merge(n, mean, m2, nb, part[ti * 1024 + c], part[ti * 1024 + 512 + c]);
  }
  red[0][tg][t & 63] = n;
  red[1][tg][t & 63] = mean;
  red[2][tg][t & 63] = m2;
  __syncthreads();
  if (tg == 0) {
    for (int k = 1; k < 4; ++k) chan_merge(n, mean, m2, red[0][k][t], red[1][k][t], red[2][k][t]);
    P.mean[b * 512 + c] = (float)mean;
    P.rstd[b * 512 + c] = (float)(1.0 / sqrt(m2 / n + 1e-5));
  }
}

// GraphAttentionLayer (GATs.py:62-123) with include_self=True, with_linear_transform=False,
// additional=False, concat=True, W a folded (h.(W a) == (h W) a):
//   s3 = h3.wa_hi, s2_j = leaf_j.wa_lo, e = LeakyReLU_0.2(s3 + [s3, s2_1..L])
//   alpha = softmax(e), out = ELU(alpha_0 h3 + sum_j alpha_j leaf_j)
// P = 64/L 3D points per workgroup; the workgroup's P*L leaf columns are staged in LDS once
// (16-byte loads) and read twice (logits, weighted sum) -- leaves cross HBM once per layer.
__global__ __launch_bounds__(256) void gat_kernel(const float* __restrict__ x3,
                                                  const float* __restrict__ leaves,
                                                  int64_t leaves_bs, const float* __restrict__ wa,
                                                  float* __restrict__ y3, int n3, int L,
                                                  int P) {
  extern __shared__ float smem[];
  const int cols = P * L;
  const int pitch = cols + 1;
  float* lt = smem;                      // [256][pitch]
  float* h3 = lt + 256 * pitch;          // [8][256]
  float* logit = h3 + P * 256;           // [P][1+L]
  const int b = blockIdx.y, p0 = blockIdx.x * P;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t ncol = (int64_t)n3 * L;
  const float* lv = leaves + b * leaves_bs + (int64_t)p0 * L;
  if ((ncol & 3) == 0 && (cols & 3) == 0 && (int64_t)(p0 + P) * L <= ncol) {
    const int c4s = cols >> 2;   // 16-byte loads; rows are 16-byte aligned
    for (int e = t; e < 256 * c4s; e += 256) {
      const int c = e / c4s, j4 = e - c * c4s;
      const float4 v = *reinterpret_cast<const float4*>(lv + (int64_t)c * ncol + j4 * 4);
      float* d = lt + c * pitch + j4 * 4;
      d[0] = v.x;
      d[1] = v.y;
      d[2] = v.z;
      d[3] = v.w;
    }
  } else {
    for (int e = t; e < 256 * cols; e += 256) {
      const int c = e / cols, j = e - c * cols;
      lt[c * pitch + j] = ((int64_t)p0 * L + j < ncol) ? lv[(int64_t)c * ncol + j] : 0.f;
    }
  }
  const float* xb = x3 + (int64_t)b * n3 * kDim;
  for (int e = t; e < P * 256; e += 256) {
    const int p = e >> 8, c = e & 255;
    h3[e] = (p0 + p < n3) ? xb[(int64_t)(p0 + p) * kDim + c] : 0.f;
  }
  __syncthreads();
  const float* wa_lo = wa;
  const float* wa_hi = wa + 256;
  // logits: dots 0..cols-1 are leaves, cols..cols+7 are the 3D points
  for (int k = wave; k < cols + P; k += 4) {
    float s = 0.f;
    if (k < cols) {
#pragma unroll
      for (int i = 0; i < 4; ++i) s += lt[(lane + 64 * i) * pitch + k] * wa_lo[lane + 64 * i];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) s += h3[(k - cols) * 256 + lane + 64 * i] * wa_hi[lane + 64 * i];
    }
    s = wave_sum(s);
    if (lane == 0) {
      if (k < cols) logit[(k / L) * (1 + L) + 1 + (k % L)] = s;
      else logit[(k - cols) * (1 + L)] = s;
    }
  }
  __syncthreads();
  if (t < P) {
    float* e = logit + t * (1 + L);
    const float s3 = e[0];
    float mx = -INFINITY;
    for (int j = 0; j <= L; ++j) {
      float v = s3 + (j == 0 ? s3 : e[j]);
      v = v > 0.f ? v : v * 0.2f;
      e[j] = v;
      mx = fmaxf(mx, v);
    }
    float sum = 0.f;
    for (int j = 0; j <= L; ++j) {
      const float v = expf(e[j] - mx);
      e[j] = v;
      sum += v;
    }
    for (int j = 0; j <= L; ++j) e[j] = e[j] / sum;
  }
  __syncthreads();
  float* yb = y3 + (int64_t)b * n3 * kDim;
  const int c = t;
  for (int p = 0; p < P; ++p) {
    if (p0 + p >= n3) break;
    const float* al = logit + p * (1 + L);
    float acc = al[0] * h3[p * 256 + c];
    for (int j = 0; j < L; ++j) acc += al[1 + j] * lt[c * pitch + p * L + j];
    yb[(int64_t)(p0 + p) * kDim + c] = elu1(acc);
  }
}

// F.normalize(x, p=2, dim=channels), one wave per token row (GATs_SuperGlue.py:245-246).
__global__ __launch_bounds__(256) void l2norm_kernel(float* x2, int rows2, float* x3, int rows3) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  float* p;
  if (row < rows2) p = x2 + (int64_t)row * kDim;
  else if (row < rows2 + rows3) p = x3 + (int64_t)(row - rows2) * kDim;
  else return;
  float4 v = *reinterpret_cast<float4*>(p + lane * 4);
  const float ss = wave_sum(v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w);
  const float n = fmaxf(sqrtf(ss), 1e-12f);
  v.x /= n;
  v.y /= n;
  v.z /= n;
  v.w /= n;
  *reinterpret_cast<float4*>(p + lane * 4) = v;
}

// Combine the score GEMM's per-tile softmax partials: rows over N3 tiles (softmax dim 2),
// columns over N1 tiles (softmax dim 1).  Also resets the packed argmax words.
__global__ __launch_bounds__(256) void softmax_reduce_kernel(
    const float* rowpart, int ntiles3, const float* colpart, int mtiles1, int batch, int n1,
    int n3, float* rowmax, float* rowsum, float* colmax, float* colsum,
    unsigned long long* rowbest, unsigned long long* colbest) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t nr = (int64_t)batch * n1, nc = (int64_t)batch * n3;
  if (idx < nr) {
    const float* p = rowpart + idx * ntiles3 * 2;
    float mx = -INFINITY;
    for (int i = 0; i < ntiles3; ++i) mx = fmaxf(mx, p[2 * i]);
    float s = 0.f;
    for (int i = 0; i < ntiles3; ++i) s += p[2 * i + 1] * expf(p[2 * i] - mx);
    rowmax[idx] = mx;
    rowsum[idx] = s;
    rowbest[idx] = 0ull;
  } else if (idx < nr + nc) {
    const int64_t j = idx - nr;
    const float* p = colpart + j * mtiles1 * 2;
    float mx = -INFINITY;
    for (int i = 0; i < mtiles1; ++i) mx = fmaxf(mx, p[2 * i]);
    float s = 0.f;
    for (int i = 0; i < mtiles1; ++i) s += p[2 * i + 1] * expf(p[2 * i] - mx);
    colmax[j] = mx;
    colsum[j] = s;
    colbest[j] = 0ull;
  }
}

// (value, index) packed so that one unsigned max picks the larger value and, on ties, the
// smaller index -- torch CPU max(dim) semantics (first occurrence).  conf >= 0.
__device__ __forceinline__ unsigned long long pack_best(float v, int idx) {
  return ((unsigned long long)__float_as_uint(v) << 32) | (unsigned)(0xFFFFFFFFu - (unsigned)idx);
}
__device__ __forceinline__ int best_index(unsigned long long p) {
  return (int)(0xFFFFFFFFu - (unsigned)(p & 0xFFFFFFFFull));
}
__device__ __forceinline__ float best_value(unsigned long long p) {
  return __uint_as_float((unsigned)(p >> 32));
}
__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int m) {
  const unsigned lo = __shfl_xor((unsigned)v, m, 64);
  const unsigned hi = __shfl_xor((unsigned)(v >> 32), m, 64);
  return ((unsigned long long)hi << 32) | lo;
}

// conf = softmax(S, dim=1) * softmax(S, dim=2) (GATs_SuperGlue.py:253) in place over S,
// plus row/column max+argmax (:256) folded in through 64-bit atomicMax.
__global__ __launch_bounds__(256) void conf_kernel(float* S, int n1, int n3,
                                                   const float* rowmax, const float* rowsum,
                                                   const float* colmax, const float* colsum,
                                                   unsigned long long* rowbest,
                                                   unsigned long long* colbest, int write_conf) {
  __shared__ unsigned long long cb[4][64];
  const int nt3 = (n3 + 63) / 64;
  const int tilen = blockIdx.x % nt3, tilem = blockIdx.x / nt3;
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m = tilen * 64 + lane;           // 3D column
  const bool col_ok = m < n3;
  float* Sb = S + (int64_t)b * n1 * n3;
  float cmx = 0.f, cinv = 0.f;
  if (col_ok) {
    cmx = colmax[(int64_t)b * n3 + m];
    cinv = 1.0f / colsum[(int64_t)b * n3 + m];
  }
  unsigned long long cbest = 0ull;
  for (int i = 0; i < 16; ++i) {
    const int n = tilem * 64 + wave + 4 * i;  // 2D row
    if (n >= n1) break;
    const float rmx = rowmax[(int64_t)b * n1 + n];
    const float rinv = 1.0f / rowsum[(int64_t)b * n1 + n];
    unsigned long long key = 0ull;
    if (col_ok) {
      float* ps = Sb + (int64_t)n * n3 + m;
      const float s = *ps;
      const float c = (expf(s - cmx) * cinv) * (expf(s - rmx) * rinv);
      if (write_conf) *ps = c;
      key = pack_best(c, m);
      const unsigned long long ck = pack_best(c, n);
      cbest = ck > cbest ? ck : cbest;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const unsigned long long other = shfl_xor_u64(key, o);
      key = other > key ? other : key;
    }
    if (lane == 0 && key != 0ull) atomicMax(rowbest + (int64_t)b * n1 + n, key);
  }
  cb[wave][lane] = cbest;
  __syncthreads();
  if (wave == 0 && col_ok) {
    unsigned long long k = cb[0][lane];
    for (int w = 1; w < 4; ++w) k = cb[w][lane] > k ? cb[w][lane] : k;
    if (k != 0ull) atomicMax(colbest + (int64_t)b * n3 + m, k);
  }
}

// Mutual nearest neighbour + threshold (GATs_SuperGlue.py:256-267).
__global__ __launch_bounds__(256) void mutual_kernel(const unsigned long long* rowbest,
                                                     const unsigned long long* colbest,
                                                     int batch, int n1, int n3, float thr,
                                                     int64_t* matches0, int64_t* matches1,
                                                     float* ms0, float* ms1) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t nr = (int64_t)batch * n1, nc = (int64_t)batch * n3;
  if (idx < nr) {
    const int b = (int)(idx / n1), n = (int)(idx - (int64_t)b * n1);
    const unsigned long long p = rowbest[idx];
    const int i0 = min(max(best_index(p), 0), n3 - 1);
    const float v = best_value(p);
    const int i1 = best_index(colbest[(int64_t)b * n3 + i0]);
    const bool mutual = i1 == n;
    const float s = mutual ? v : 0.f;
    ms0[idx] = s;
    matches0[idx] = (mutual && s > thr) ? (int64_t)i0 : -1;
  } else if (idx < nr + nc) {
    const int64_t j = idx - nr;
    const int b = (int)(j / n3), m = (int)(j - (int64_t)b * n3);
    const int i1 = min(max(best_index(colbest[j]), 0), n1 - 1);
    const unsigned long long p = rowbest[(int64_t)b * n1 + i1];
    const bool mutual = best_index(p) == m;
    const float v = best_value(p);
    const float s = mutual ? v : 0.f;
    ms1[j] = s;
    matches1[j] = (mutual && v > thr) ? (int64_t)i1 : -1;
  }
}

// ------------------------------------------------------------------------------------
// workspace plan
// ------------------------------------------------------------------------------------
namespace {

struct Plan {
  float *x2[2], *x3[2];
  float *qkv2, *qkv3;
  float *kvpart2, *kvpart3, *kspart2, *kspart3;
  float *kvt, *ksum;
  float *o2, *o3, *msg2, *msg3, *y12, *y13;
  float *stats2, *stats3, *mean, *rstd;
  float *f2, *f3, *s;
  float *rowpart, *colpart, *rowmax, *rowsum, *colmax, *colsum;
  unsigned long long *rowbest, *colbest;
  size_t bytes;
};

Plan make_plan(void* ws, int B, int n1, int n3, bool with_conf) {
  Carve c(ws);
  Plan p;
  const size_t t2 = (size_t)B * n1, t3 = (size_t)B * n3;
  for (int i = 0; i < 2; ++i) {
    p.x2[i] = c.take<float>(t2 * 256);
    p.x3[i] = c.take<float>(t3 * 256);
  }
  p.qkv2 = c.take<float>(t2 * 768);
  p.qkv3 = c.take<float>(t3 * 768);
  const int ch2 = ceil_div(n1, 64), ch3 = ceil_div(n3, 64);
  p.kvpart2 = c.take<float>((size_t)B * ch2 * 16384);
  p.kvpart3 = c.take<float>((size_t)B * ch3 * 16384);
  p.kspart2 = c.take<float>((size_t)B * ch2 * 256);
  p.kspart3 = c.take<float>((size_t)B * ch3 * 256);
  p.kvt = c.take<float>((size_t)2 * B * 16384);
  p.ksum = c.take<float>((size_t)2 * B * 256);
  p.o2 = c.take<float>(t2 * 256);
  p.o3 = c.take<float>(t3 * 256);
  p.msg2 = c.take<float>(t2 * 256);
  p.msg3 = c.take<float>(t3 * 256);
  p.y12 = c.take<float>(t2 * 512);
  p.y13 = c.take<float>(t3 * 512);
  p.stats2 = c.take<float>((size_t)B * ch2 * 1024);
  p.stats3 = c.take<float>((size_t)B * ch3 * 1024);
  p.mean = c.take<float>((size_t)2 * B * 512);
  p.rstd = c.take<float>((size_t)2 * B * 512);
  p.f2 = c.take<float>(t2 * 256);
  p.f3 = c.take<float>(t3 * 256);
  p.s = with_conf ? nullptr : c.take<float>((size_t)B * n1 * n3);
  p.rowpart = c.take<float>(t2 * ch3 * 2);
  p.colpart = c.take<float>(t3 * ch2 * 2);
  p.rowmax = c.take<float>(t2);
  p.rowsum = c.take<float>(t2);
  p.colmax = c.take<float>(t3);
  p.colsum = c.take<float>(t3);
  p.rowbest = c.take<unsigned long long>(t2);
  p.colbest = c.take<unsigned long long>(t3);
  p.bytes = align_up(c.off, 256);
  return p;
}

GemmProb gemm_prob(const float* A, int lda, const float* W, int ldw, const float* bias,
                   float* Y, int ldy, int M, int N, int K, int batch) {
  GemmProb g;
  memset(&g, 0, sizeof(g));
  g.A0 = A;
  g.lda0 = lda;
  g.a0_bs = (int64_t)M * lda;
  g.ksplit = K;
  g.W = W;
  g.ldw = ldw;
  g.bias = bias;
  g.Y = Y;
  g.ldy = ldy;
  g.y_bs = (int64_t)M * ldy;
  g.M = M;
  g.N = N;
  g.K = K;
  g.batch = batch;
  g.scale = 1.f;
  g.vdiv = 1.f;
  return g;
}

}  // namespace
}  // namespace onepose

// ------------------------------------------------------------------------------------
// C-ABI
// ------------------------------------------------------------------------------------
using namespace onepose;

extern "C" {

const char* onepose_last_error(void) { return g_last_error.c_str(); }
int onepose_abi_version(void) { return 1; }

int onepose_profile_begin(uint64_t kind_mask, int capacity) {
  clear_error();
  OP_REQUIRE(capacity >= 0, "profile: capacity %d", capacity);
  const size_t need = 2 * (size_t)capacity + 2;
  while (g_prof.ev.size() < need) {
    hipEvent_t e;
    OP_HIP(hipEventCreate(&e));
    g_prof.ev.push_back(e);
  }
  g_prof.kinds.assign(capacity + 1, -1);
  g_prof.n = 0;
  g_prof.mask = kind_mask;
  return ONEPOSE_OK;
}

int onepose_profile_end(int* kinds, float* ms, int capacity, int* count) {
  clear_error();
  g_prof.mask = 0;
  const int n = g_prof.n;
  if (count) *count = n;
  if (n > 0) OP_HIP(hipEventSynchronize(g_prof.ev[2 * n - 1]));
  for (int i = 0; i < n && i < capacity; ++i) {
    float t = 0.f;
    OP_HIP(hipEventElapsedTime(&t, g_prof.ev[2 * i], g_prof.ev[2 * i + 1]));
    if (ms) ms[i] = t;
    if (kinds) kinds[i] = g_prof.kinds[i];
  }
  g_prof.n = 0;
  return ONEPOSE_OK;
}

const char* onepose_profile_kind_name(int kind) {
  return (kind >= 0 && kind < K_NUM_KINDS) ? kKindNames[kind] : nullptr;
}

int onepose_matcher_num_tensors(void) { return (int)tensor_specs().size(); }

const char* onepose_matcher_tensor_name(int i) {
  const auto& s = tensor_specs();
  if (i < 0 || i >= (int)s.size()) return nullptr;
  return s[i].name.c_str();
}

int64_t onepose_matcher_tensor_numel(int i) {
  const auto& s = tensor_specs();
  if (i < 0 || i >= (int)s.size()) return -1;
  return s[i].numel;
}

size_t onepose_matcher_packed_bytes(void) { return (size_t)kPackedFloats * sizeof(float); }

int onepose_matcher_pack(const float* const* tensors, int n_tensors, void* packed_host) {
  clear_error();
  const auto& specs = tensor_specs();
  OP_REQUIRE(tensors != nullptr && packed_host != nullptr, "pack: null pointer");
  OP_REQUIRE(n_tensors == (int)specs.size(), "pack: expected %d tensors, got %d",
             (int)specs.size(), n_tensors);
  for (int i = 0; i < n_tensors; ++i) OP_REQUIRE(tensors[i] != nullptr, "pack: tensor %d null", i);
  float* out = static_cast<float*>(packed_host);
  int ti = 0, ap = 0, gat = 0;
  for (int layer = 0; layer < kLayers; ++layer) {
    if (layer % 3 == 0) {
      const float* W = tensors[ti++];   // [256 in][256 out]
      const float* a = tensors[ti++];   // [512]
      float* wa = out + kApLayers * kApFloats + (int64_t)gat * kGatFloats;
      for (int c = 0; c < 256; ++c) {
        double lo = 0.0, hi = 0.0;
        for (int j = 0; j < 256; ++j) {
          lo += (double)W[c * 256 + j] * (double)a[j];
          hi += (double)W[c * 256 + j] * (double)a[256 + j];
        }
        wa[c] = (float)lo;
        wa[256 + c] = (float)hi;
      }
      ++gat;
      continue;
    }
    float* p = out + (int64_t)ap * kApFloats;
    float* wqkv = p;
    float* bqkv = wqkv + kApWqkv;
    float* wm = bqkv + kApBqkv;
    float* bm = wm + kApWm;
    float* w1 = bm + kApBm;
    float* b1 = w1 + kApW1;
    float* w2 = b1 + kApB1;
    float* b2 = w2 + kApW2;
    // q/k/v: packed row h*64+d <- reference row d*4+h (view(B, 64, 4, N), :116)
    for (int j = 0; j < 3; ++j) {
      const float* w = tensors[ti++];
      const float* bias = tensors[ti++];
      for (int cp = 0; cp < 256; ++cp) {
        const int h = cp / 64, d = cp % 64, cr = d * 4 + h;
        memcpy(wqkv + (int64_t)(j * 256 + cp) * 256, w + (int64_t)cr * 256, 256 * sizeof(float));
        bqkv[j * 256 + cp] = bias[cr];
      }
    }
    {  // merge: packed column h*64+q <- reference column q*4+h
      const float* w = tensors[ti++];
      const float* bias = tensors[ti++];
      for (int o = 0; o < 256; ++o)
        for (int cp = 0; cp < 256; ++cp) {
          const int h = cp / 64, q = cp % 64;
          wm[o * 256 + cp] = w[o * 256 + q * 4 + h];
        }
      memcpy(bm, bias, 256 * sizeof(float));
    }
    memcpy(w1, tensors[ti++], kApW1 * sizeof(float));
    memcpy(b1, tensors[ti++], kApB1 * sizeof(float));
    memcpy(w2, tensors[ti++], kApW2 * sizeof(float));
    memcpy(b2, tensors[ti++], kApB2 * sizeof(float));
    ++ap;
  }
  float* fin = out + kApLayers * kApFloats + kGatLayers * kGatFloats;
  memcpy(fin, tensors[ti++], 256 * 256 * sizeof(float));
  memcpy(fin + 256 * 256, tensors[ti++], 256 * sizeof(float));
  return ONEPOSE_OK;
}

size_t onepose_match_workspace_bytes(int batch, int n1, int n3, int num_leaf, int with_conf) {
  (void)num_leaf;
  if (batch <= 0 || n1 <= 0 || n3 <= 0) return 0;
  return make_plan(nullptr, batch, n1, n3, with_conf != 0).bytes;
}

}  // extern "C"

namespace onepose {
namespace {
int init_kernel_attributes() {
  static int rc = -1;
  if (rc == -1) {
    rc = ONEPOSE_OK;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(attn_apply_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)kApplyLds) !=
            hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(gat_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
      rc = ONEPOSE_ERR_HIP;
  }
  return rc;
}
}  // namespace
}  // namespace onepose

extern "C" {

int onepose_match(const void* packed_weights, const float* desc2d, int64_t desc2d_bstride,
                  const float* desc3d, int64_t desc3d_bstride, const float* leaves,
                  int64_t leaves_bstride, int batch, int n1, int n3, int num_leaf,
                  float scale_factor, float match_threshold, int64_t* matches0,
                  int64_t* matches1, float* mscores0, float* mscores1, float* conf,
                  void* workspace, size_t workspace_bytes, void* stream_) {
  clear_error();
  OP_REQUIRE(packed_weights && desc2d && desc3d && leaves, "match: null input");
  OP_REQUIRE(matches0 && matches1 && mscores0 && mscores1, "match: null output");
  OP_REQUIRE(batch >= 1 && n1 >= 1 && n3 >= 1, "match: batch=%d n1=%d n3=%d", batch, n1, n3);
  OP_REQUIRE(num_leaf >= 1 && num_leaf <= 16, "match: num_leaf=%d not in [1,16]", num_leaf);
  OP_REQUIRE(scale_factor != 0.f, "match: scale_factor 0");
  const bool with_conf = conf != nullptr;
  const Plan need = make_plan(nullptr, batch, n1, n3, with_conf);
  OP_REQUIRE(workspace != nullptr, "match: null workspace");
  if (workspace_bytes < need.bytes) {
    set_error("match: workspace %zu < %zu bytes", workspace_bytes, need.bytes);
    return ONEPOSE_ERR_WORKSPACE;
  }
  hipStream_t st = static_cast<hipStream_t>(stream_);
  if (init_kernel_attributes() != ONEPOSE_OK) {
    set_error("match: hipFuncSetAttribute failed");
    return ONEPOSE_ERR_HIP;
  }
  Plan p = make_plan(workspace, batch, n1, n3, with_conf);
  const float* wbase = static_cast<const float*>(packed_weights);
  const int B = batch;
  float* S = with_conf ? conf : p.s;

  OP_LAUNCH(K_TRANSPOSE, st, transpose_in_kernel, dim3(ceil_div(n1, 64), 4, B), dim3(256), 0, st,
                     desc2d, desc2d_bstride, n1, p.x2[0]);
  OP_LAUNCH(K_TRANSPOSE, st, transpose_in_kernel, dim3(ceil_div(n3, 64), 4, B), dim3(256), 0, st,
                     desc3d, desc3d_bstride, n3, p.x3[0]);

  int c2 = 0, c3 = 0, ap = 0, gat = 0;
  const int ch2 = ceil_div(n1, 64), ch3 = ceil_div(n3, 64);
  const int gat_p = max(1, 64 / num_leaf);
  const size_t gat_lds =
      (size_t)(256 * (gat_p * num_leaf + 1) + gat_p * 256 + gat_p * (1 + num_leaf)) * 4;
  for (int layer = 0; layer < kLayers; ++layer) {
    const int kind = layer % 3;  // 0 GATs, 1 self, 2 cross
    if (kind == 0) {
      OP_LAUNCH(K_GAT, st, gat_kernel, dim3(ceil_div(n3, gat_p), B), dim3(256), gat_lds, st,
                         p.x3[c3], leaves, leaves_bstride, gat_weights(wbase, gat), p.x3[c3 ^ 1],
                         n3, num_leaf, gat_p);
      c3 ^= 1;
      ++gat;
      continue;
    }
    const ApW w = ap_weights(wbase, ap++);
    int rc;
    {  // q | k | v projections of both tensors
      GemmArgs a;
      a.nprob = 2;
      a.p[0] = gemm_prob(p.x2[c2], 256, w.wqkv, 256, w.bqkv, p.qkv2, 768, n1, 768, 256, B);
      a.p[0].phi_cols = 512;
      a.p[0].vdiv = (float)n1;
      a.p[1] = gemm_prob(p.x3[c3], 256, w.wqkv, 256, w.bqkv, p.qkv3, 768, n3, 768, 256, B);
      a.p[1].phi_cols = 512;
      a.p[1].vdiv = (float)n3;
      if ((rc = gemm_launch(EPI_QKV, PRO_PLAIN, a, st, K_QKV)) != ONEPOSE_OK) return rc;
    }
    KvArgs kva;
    kva.p[0] = {p.qkv2, p.kvpart2, p.kspart2, n1, ch2, B * ch2};
    kva.p[1] = {p.qkv3, p.kvpart3, p.kspart3, n3, ch3, B * ch3};
    OP_LAUNCH(K_KV_PARTIAL, st, kv_partial_kernel, dim3(B * (ch2 + ch3)), dim3(256), 0, st, kva);
    {
      const int total = 2 * B * (16384 + 256) / 4;
      OP_LAUNCH(K_KV_REDUCE, st, kv_reduce_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, st,
                kva, p.kvt, p.ksum, B);
    }
    {  // self: side s attends to itself; cross: 2D attends to 3D and vice versa
      const int src2 = (kind == 1) ? 0 : 1, src3 = (kind == 1) ? 1 : 0;
      const float ns2 = (float)(src2 == 0 ? n1 : n3), ns3 = (float)(src3 == 0 ? n1 : n3);
      ApplyArgs aa;
      aa.p[0] = {p.qkv2, p.kvt + (size_t)src2 * B * 16384, p.ksum + (size_t)src2 * B * 256,
                 p.o2, n1, ns2, ch2, B * ch2};
      aa.p[1] = {p.qkv3, p.kvt + (size_t)src3 * B * 16384, p.ksum + (size_t)src3 * B * 256,
                 p.o3, n3, ns3, ch3, B * ch3};
      OP_LAUNCH(K_APPLY, st, attn_apply_kernel, dim3(B * (ch2 + ch3)), dim3(256), kApplyLds, st, aa);
    }
    {  // merge
      GemmArgs a;
      a.nprob = 2;
      a.p[0] = gemm_prob(p.o2, 256, w.wm, 256, w.bm, p.msg2, 256, n1, 256, 256, B);
      a.p[1] = gemm_prob(p.o3, 256, w.wm, 256, w.bm, p.msg3, 256, n3, 256, 256, B);
      if ((rc = gemm_launch(EPI_BIAS, PRO_PLAIN, a, st, K_MERGE)) != ONEPOSE_OK) return rc;
    }
    {  // MLP conv 1 on cat[x, message] + InstanceNorm partials
      GemmArgs a;
      a.nprob = 2;
      a.p[0] = gemm_prob(p.x2[c2], 256, w.w1, 512, w.b1, p.y12, 512, n1, 512, 512, B);
      a.p[0].A1 = p.msg2;
      a.p[0].lda1 = 256;
      a.p[0].a1_bs = (int64_t)n1 * 256;
      a.p[0].ksplit = 256;
      a.p[0].stats = p.stats2;
      a.p[1] = gemm_prob(p.x3[c3], 256, w.w1, 512, w.b1, p.y13, 512, n3, 512, 512, B);
      a.p[1].A1 = p.msg3;
      a.p[1].lda1 = 256;
      a.p[1].a1_bs = (int64_t)n3 * 256;
      a.p[1].ksplit = 256;
      a.p[1].stats = p.stats3;
      if ((rc = gemm_launch(EPI_STATS, PRO_PLAIN, a, st, K_MLP1)) != ONEPOSE_OK) return rc;
    }
    {
      StatsArgs sa;
      sa.p[0] = {p.stats2, p.mean, p.rstd, n1, ch2};
      sa.p[1] = {p.stats3, p.mean + (size_t)B * 512, p.rstd + (size_t)B * 512, n3, ch3};
      OP_LAUNCH(K_STATS, st, stats_finalize_kernel, dim3(2 * B * 8), dim3(256), 0,
                         st, sa, B);
    }
    {  // MLP conv 2 on ReLU(InstanceNorm(.)) + residual: desc + delta
      GemmArgs a;
      a.nprob = 2;
      a.p[0] = gemm_prob(p.y12, 512, w.w2, 512, w.b2, p.x2[c2 ^ 1], 256, n1, 256, 512, B);
      a.p[0].R = p.x2[c2];
      a.p[0].ldr = 256;
      a.p[0].r_bs = (int64_t)n1 * 256;
      a.p[0].pro_mean = p.mean;
      a.p[0].pro_rstd = p.rstd;
      a.p[0].pro_bs = 512;
      a.p[1] = gemm_prob(p.y13, 512, w.w2, 512, w.b2, p.x3[c3 ^ 1], 256, n3, 256, 512, B);
      a.p[1].R = p.x3[c3];
      a.p[1].ldr = 256;
      a.p[1].r_bs = (int64_t)n3 * 256;
      a.p[1].pro_mean = p.mean + (size_t)B * 512;
      a.p[1].pro_rstd = p.rstd + (size_t)B * 512;
      a.p[1].pro_bs = 512;
      if ((rc = gemm_launch(EPI_RESID, PRO_NORM_RELU, a, st, K_MLP2)) != ONEPOSE_OK) return rc;
    }
    c2 ^= 1;
    c3 ^= 1;
  }

  int rc;
  {  // final_proj on both sides, then L2 normalise
    const float* fw = final_weights(wbase);
    GemmArgs a;
    a.nprob = 2;
    a.p[0] = gemm_prob(p.x2[c2], 256, fw, 256, fw + 65536, p.f2, 256, n1, 256, 256, B);
    a.p[1] = gemm_prob(p.x3[c3], 256, fw, 256, fw + 65536, p.f3, 256, n3, 256, 256, B);
    if ((rc = gemm_launch(EPI_BIAS, PRO_PLAIN, a, st, K_FINAL)) != ONEPOSE_OK) return rc;
    const int rows = B * (n1 + n3);
    OP_LAUNCH(K_L2NORM, st, l2norm_kernel, dim3(ceil_div(rows, 4)), dim3(256), 0, st, p.f2, B * n1,
                       p.f3, B * n3);
  }
  {  // S = D2^T D3 / scale_factor with softmax partials
    GemmArgs a;
    a.nprob = 1;
    a.p[0] = gemm_prob(p.f2, 256, p.f3, 256, nullptr, S, n3, n1, n3, 256, B);
    a.p[0].w_bs = (int64_t)n3 * 256;
    a.p[0].scale = scale_factor;
    a.p[0].rowstat = p.rowpart;
    a.p[0].colstat = p.colpart;
    if ((rc = gemm_launch(EPI_SCORE, PRO_PLAIN, a, st, K_SCORE)) != ONEPOSE_OK) return rc;
  }
  {
    const int64_t total = (int64_t)B * (n1 + n3);
    OP_LAUNCH(K_SMX_REDUCE, st, softmax_reduce_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256),
                       0, st, p.rowpart, ch3, p.colpart, ch2, B, n1, n3, p.rowmax, p.rowsum,
                       p.colmax, p.colsum, p.rowbest, p.colbest);
    OP_LAUNCH(K_CONF, st, conf_kernel, dim3(ch2 * ch3, B), dim3(256), 0, st, S, n1, n3, p.rowmax,
                       p.rowsum, p.colmax, p.colsum, p.rowbest, p.colbest, with_conf ? 1 : 0);
    OP_LAUNCH(K_MUTUAL, st, mutual_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                       p.rowbest, p.colbest, B, n1, n3, match_threshold, matches0, matches1,
                       mscores0, mscores1);
  }
  return ONEPOSE_OK;
}

}  // extern "C"
