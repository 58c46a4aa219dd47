// GATsSPG matcher forward on gfx950 (GATsSuperGlue.forward, GATs_SuperGlue.py:203-278).
//
// Data layout in HBM (per batch sample, fp32):
//   X2 [N1][256], X3 [N3][256]       token-major descriptors (ping-pong buffers)
//   KVpart [chunk][h][d][q]          per-64-token linear-attention partials (kv GEMM epilogue)
//   KV [h][d][q], ksum [h*64+d]      linear-attention state of one source tensor
//   QZ [N][256]                      phi(q) * Z * Ns, channels head-major (h*64+d)
//   Mf [512][256]                    per-frame folded weights  (W1b Wm) KV_h^T  per head
//   Y1 [N][512]                      MLP hidden
//   S/conf [N1][N3]                  score matrix, overwritten in place by conf_matrix
// The reference's [B, C, N] inputs are transposed once on entry; the leaf descriptors
// ([B, 256, N3*L], per-object constants, 33.5 MB at N3=4096) are read in place by the
// GAT kernel and never copied.
//
// Layer schedule (AttentionalGNN.forward, GATs_SuperGlue.py:67-85): for each of the 12
// layers, GAT layers update X3 only; self/cross layers run both sides in the same
// launches (two problems per grid) because delta0 and delta1 both read the pre-update
// descriptors (:77-78, :82-83).  One attention layer (AttentionPropagation, :123-132):
//   1. kv GEMM  [phi(k)_h | v_h/Ns] per 128-column tile, epilogue: KV_h / sum phi(k) partials
//   2. kv_reduce: KV[src], ksum[src]
//   3. m_fold: Mf = C_h KV_h^T with C = W1b Wm  (merge conv folded into MLP conv 1)
//   4. q GEMM, epilogue phi(q) * Z * Ns
//   5. MLP conv 1 = [W1a | Mf] [x ; QZ] + (b1 + W1b bm), epilogue InstanceNorm partials
//   6. InstanceNorm statistics (finalized by the last M-tile of each column block of step 5)
//   7. MLP conv 2 on ReLU(norm(.)) + residual
// Steps 3-5 are an exact re-association of message = merge(attention), MLP(cat[x, msg])
// (the linear attention output and the merge conv are linear in the message): the fp32
// result differs from the reference's evaluation order only in rounding.
#include <cmath>
#include <cstdarg>
#include <cstring>
#include <vector>

#include "gemm.h"

#include <algorithm>
#include <atomic>
#include <mutex>
#include <unordered_map>

namespace onepose {

// GEMM tile per layer GEMM (gemm.h; measured per shape on config 2).
constexpr int kTileKV = TILE_32x128, kTileMLP1 = TILE_64x64,
              kTileMLP2 = TILE_64x64, kTileMLP2F32 = TILE_64x32K2, kTileFinal = TILE_64x64;
// fp32 final projection + L2: whole rows on 8 waves (two per SIMD; 160 workgroups at config 2).
// Same-box A/B at config 2 (profiles/r04/final_proj/): 1718 / 1719 frames/s on 4 waves, 1727 /
// 1732 on 8 (final 0.021 -> 0.019 ms per frame, bit-identical), 1700 / 1703 unfused (BIAS 64 x
// 64 + l2norm_kernel)
constexpr int kTileFinalL2 = TILE_32x256W8;
constexpr int kTileScore = TILE_128x64W8, kScoreBM = 128;
// mlp2 in the split mode below 4 tiles per CU: 32 x 64 on 2 waves (config 2: 640 workgroups
// instead of 320; 0.231 -> 0.213 ms per frame); the bf16 mode keeps 64 x 64 (32 x 64 measured
// 0.110 -> 0.117 at config 2 and 0.154 -> 0.166 at config 5, profiles/r04/planes/)
constexpr int kTileMLP2Split = TILE_32x64W2;
constexpr int kFusedFoldMaxBatch = 4;   // kv_fold up to this batch, kv_reduce + m_fold above
constexpr int kMlp2WideTiles = 1024;    // fp32 mlp2: 64x64 tiles from this many (4 per CU)
constexpr int kQkvWideTiles = 256;      // fp32 qkv: 64x128 tiles from this many 64-row tiles
constexpr int kQkvWiderTiles = 4096;    //   of the 3D side; 128x128 from this many (qkv_tile_for)

// Object-cache header (ObjLayout::hdr, written by onepose_object_prepare): what the prepare
// built and its generation, so a forward can check on the device that the memory it was handed
// still holds that cache -- a cache freed without onepose_object_release and its address reused
// passes the host registry's check, not this one.
constexpr unsigned kCacheMagic = 0x4f504331u;   // "OPC1"
constexpr int kCacheHdrWords = 8;
struct CacheHdr {
  unsigned magic, n3, num_leaf, precision, flags, gen_lo, gen_hi, check;
};
static_assert(sizeof(CacheHdr) == kCacheHdrWords * 4, "header words");
inline CacheHdr cache_hdr(int n3, int num_leaf, int precision, int flags, unsigned long long gen) {
  CacheHdr h{kCacheMagic, (unsigned)n3, (unsigned)num_leaf, (unsigned)precision, (unsigned)flags,
             (unsigned)gen, (unsigned)(gen >> 32), 0u};
  h.check = ~(h.magic ^ h.n3 ^ (h.num_leaf << 8) ^ (h.precision << 16) ^ (h.flags << 24) ^
              h.gen_lo ^ (h.gen_hi * 2654435761u));
  return h;
}
// the library's sticky device error word (onepose_device_errors)
__device__ unsigned g_device_errors;
__global__ void cache_hdr_kernel(unsigned* hdr, CacheHdr h) {
  if (threadIdx.x < kCacheHdrWords) hdr[threadIdx.x] = (&h.magic)[threadIdx.x];
}

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
  bool device = false;   // device-stamp mode
  std::vector<hipEvent_t> ev;
  std::vector<int> kinds;
  int n = 0;
  StampAcc* acc[K_NUM_KINDS] = {};   // device, kStampPool sites, allocated per stamped kind
  int next[K_NUM_KINDS] = {};   // round-robin pool cursor per kind
};
// Each launch (or graph node captured while stamping) gets its own accumulator from the
// kind's pool, so launches of one kind that run concurrently (several match streams)
// never share one; a graph node keeps its accumulator across replays, which of the same
// graph are serialised.
// Launch sites per kind: a graph node keeps its site; eager launches cycle through the pool,
// and 120 is a multiple of the per-frame launch counts (8 mlp1, 12 SuperPoint convs), so a
// site always sees the same grid (the ticket -> launch arithmetic divides by its wave count).
constexpr int kStampPool = 120;
Prof g_prof;
const char* kKindNames[K_NUM_KINDS] = {
    "transpose_in", "gat", "qkv_gemm", "kv_reduce", "m_fold", "mlp1_gemm",
    "stats_finalize", "mlp2_gemm", "final_gemm", "l2norm", "score_gemm", "softmax_reduce",
    "conf", "mutual", "select", "pnp_ransac", "pnp_refit", "pose_error", "sample_desc",
    "sp_conv", "sp_nms", "sp_select", "sp_desc"};
}  // namespace

StampAcc* prof_stamp_slot(int kind) {
  if (!g_prof.device || !((g_prof.mask >> kind) & 1ull) || g_prof.acc[kind] == nullptr)
    return nullptr;
  const int i = g_prof.next[kind]++ % kStampPool;
  return g_prof.acc[kind] + i;
}

void prof_pre(int kind, hipStream_t s) {
  if (g_prof.device) return;
  if (!((g_prof.mask >> kind) & 1ull) || 2 * g_prof.n + 1 >= (int)g_prof.ev.size()) return;
  (void)hipEventRecord(g_prof.ev[2 * g_prof.n], s);
}
void prof_post(int kind, hipStream_t s) {
  if (g_prof.device) return;
  if (!((g_prof.mask >> kind) & 1ull) || 2 * g_prof.n + 1 >= (int)g_prof.ev.size()) return;
  (void)hipEventRecord(g_prof.ev[2 * g_prof.n + 1], s);
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

// packed panel, floats (per attention layer):
//   Wqkv [768][256]: rows 0..255 q head-major (packed row h*64+d <- reference row d*4+h),
//                    then per head h: 64 rows of k_h, 64 rows of v_h
//   bqkv [768]
//   W1a [512][256] = mlp.0.weight[:, :256]
//   C   [512][256] = mlp.0.weight[:, 256:] @ merge.weight, columns head-major (h*64+q)
//   b1f [512]      = mlp.0.bias + mlp.0.weight[:, 256:] @ merge.bias
//   W2 [256][512], b2 [256]
//   CT [4][64][512]: CT[h][q][o] = C[o][h*64+q]  (the fold's operand, o contiguous)
constexpr int64_t kApWqkv = 768 * 256, kApBqkv = 768;
constexpr int64_t kApW1a = 512 * 256, kApC = 512 * 256, kApB1 = 512, kApW2 = 256 * 512,
                  kApB2 = 256, kApCT = 512 * 256;
constexpr int64_t kApFloats = kApWqkv + kApBqkv + kApW1a + kApC + kApB1 + kApW2 + kApB2 + kApCT;
constexpr int64_t kGatFloats = 512;
constexpr int64_t kFinalFloats = 256 * 256 + 256;
constexpr int64_t kPackedFloats = kApLayers * kApFloats + kGatLayers * kGatFloats + kFinalFloats;
// ... then, per attention layer, the bf16 planes of its three weight matrices for the bf16
// modes (gemm.h GemmProb::Wp): Wqkv, W1a and W2 split exactly into hi / mid / lo
// (hi = bf16(x) rounded to nearest even: PM_BF16's operand), [3][rows][cols] uint16 each.
constexpr int64_t kPlWqkv = 768 * 256, kPlW1a = 512 * 256, kPlW2 = 256 * 512;
constexpr int64_t kApPlanes = 3 * (kPlWqkv + kPlW1a + kPlW2);   // uint16 per layer
constexpr int64_t kPackedBytes = kPackedFloats * 4 + kApLayers * kApPlanes * 2;

struct ApW {
  const float *wqkv, *bqkv, *w1a, *c, *b1, *w2, *b2, *ct;
  const uint16_t *wqkv_p, *w1a_p, *w2_p;   // bf16 planes
};
ApW ap_weights(const float* base, int ap) {
  const float* p = base + (int64_t)ap * kApFloats;
  ApW w;
  const uint16_t* pl = reinterpret_cast<const uint16_t*>(base + kPackedFloats) + (int64_t)ap * kApPlanes;
  w.wqkv_p = pl;
  w.w1a_p = pl + 3 * kPlWqkv;
  w.w2_p = w.w1a_p + 3 * kPlW1a;
  w.wqkv = p; p += kApWqkv;
  w.bqkv = p; p += kApBqkv;
  w.w1a = p; p += kApW1a;
  w.c = p; p += kApC;
  w.b1 = p; p += kApB1;
  w.w2 = p; p += kApW2;
  w.b2 = p; p += kApB2;
  w.ct = p;
  return w;
}

// bf16 bits of x rounded to nearest even (the device's (__bf16)x for finite x)
uint16_t bf16_rne(float x) {
  uint32_t u;
  memcpy(&u, &x, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
float bf16_val(uint16_t b) {
  const uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
// the exact split x = hi + mid + lo of gemm.hip's store_quad_bf16, into planes n elements apart
void split_planes(const float* x, int64_t n, uint16_t* out) {
  for (int64_t i = 0; i < n; ++i) {
    const uint16_t h = bf16_rne(x[i]);
    const float r = x[i] - bf16_val(h);
    const uint16_t m = bf16_rne(r);
    out[i] = h;
    out[n + i] = m;
    out[2 * n + i] = bf16_rne(r - bf16_val(m));
  }
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

// Reference layout [B][256][n] (channel-major, GATs_SuperGlue.py:211-217) -> token-major
// [B][n][256], both inputs in one launch.  64 tokens x 64 channels per workgroup through a
// padded LDS tile; 16-byte loads along tokens when n % 4 == 0, 16-byte stores along channels.
struct TransProb {
  const void* src;   // fp32, or fp16 with f16 (the reference's .float() upcast, exact)
  int64_t bs;
  int n, tiles;   // tokens, workgroups per sample (ceil(n/64) * 4)
  float* dst;
  uint16_t* dstp = nullptr;   // bf16 modes: dst's activation planes ([B][3][n][256]; npl of them)
  int f16 = 0;
};
struct TransArgs {
  TransProb p[2];
  unsigned* zero;   // the forward's in-launch arrival counters, zeroed here (first kernel)
  int nzero;
  int npl = 0;      // activation planes per dstp (0: none)
  unsigned long long* zero64 = nullptr;   // the packed column winners (fused conf), zeroed here
  int64_t nzero64 = 0;
  // object-cache forwards: the cache's header against the one its prepare recorded (a stale
  // cache -- freed and its memory reused -- sets *err and the sticky device error word, and the
  // forward's mutual_kernel then reports no match)
  const unsigned* hdr = nullptr;
  CacheHdr expect{};
  unsigned* err = nullptr;
};
__global__ __launch_bounds__(256) void transpose_in_kernel(TransArgs args, int batch) {
  __shared__ float tile[64][65];
  if (blockIdx.x == 0 && threadIdx.x == 0 && args.err != nullptr) {
    unsigned bad = 0u;
    if (args.hdr != nullptr) {
      const unsigned* e = &args.expect.magic;
#pragma unroll
      for (int i = 0; i < kCacheHdrWords; ++i) bad |= args.hdr[i] != e[i] ? 1u : 0u;
    }
    *args.err = bad;
    if (bad) atomicOr(&g_device_errors, ONEPOSE_DEVERR_STALE_CACHE);
  }
  int bid = blockIdx.x;
  const bool second = bid >= args.p[0].tiles * batch;
  const TransProb& P = second ? args.p[1] : args.p[0];
  if (second) bid -= args.p[0].tiles * batch;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < args.nzero; i += gridDim.x * 256)
    args.zero[i] = 0u;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < args.nzero64; i += gridDim.x * 256)
    args.zero64[i] = 0ull;
  const int b = bid / P.tiles, r = bid - b * P.tiles;
  const int n0 = (r >> 2) * 64, c0 = (r & 3) * 64, n = P.n;
  const float* s = static_cast<const float*>(P.src) + b * P.bs;
  const _Float16* sh = static_cast<const _Float16*>(P.src) + b * P.bs;
  const int t = threadIdx.x;
  if (P.f16) {   // descriptors in fp16: converted as loaded (GATs_SuperGlue.py:219-221 .float())
    if ((n & 3) == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = t + 256 * i, ch = e >> 4, tq = (e & 15) * 4;
        typedef _Float16 half4 __attribute__((ext_vector_type(4)));
        half4 v = {0, 0, 0, 0};
        if (n0 + tq < n) v = *reinterpret_cast<const half4*>(sh + (int64_t)(c0 + ch) * n + n0 + tq);
        tile[ch][tq] = (float)v[0];
        tile[ch][tq + 1] = (float)v[1];
        tile[ch][tq + 2] = (float)v[2];
        tile[ch][tq + 3] = (float)v[3];
      }
    } else {
      for (int i = 0; i < 16; ++i) {
        const int ch = (t >> 6) + 4 * i, tk = t & 63;
        tile[ch][tk] = (n0 + tk < n) ? (float)sh[(int64_t)(c0 + ch) * n + n0 + tk] : 0.f;
      }
    }
  } else if ((n & 3) == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // 64 channels x 16 float4 of tokens
      const int e = t + 256 * i, ch = e >> 4, tq = (e & 15) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (n0 + tq < n) v = *reinterpret_cast<const float4*>(s + (int64_t)(c0 + ch) * n + n0 + tq);
      tile[ch][tq] = v.x;
      tile[ch][tq + 1] = v.y;
      tile[ch][tq + 2] = v.z;
      tile[ch][tq + 3] = v.w;
    }
  } else {
    for (int i = 0; i < 16; ++i) {
      const int ch = (t >> 6) + 4 * i, tk = t & 63;
      tile[ch][tk] = (n0 + tk < n) ? s[(int64_t)(c0 + ch) * n + n0 + tk] : 0.f;
    }
  }
  __syncthreads();
  float* d = P.dst + (int64_t)b * n * kDim;
  uint16_t* dp = P.dstp != nullptr ? P.dstp + (int64_t)b * kPlanesMax * n * kDim : nullptr;
#pragma unroll
  for (int i = 0; i < 4; ++i) {   // 64 tokens x 16 float4 of channels
    const int e = t + 256 * i, tk = e >> 4, cq = (e & 15) * 4;
    if (n0 + tk < n) {
      const float4 v = make_float4(tile[cq][tk], tile[cq + 1][tk], tile[cq + 2][tk], tile[cq + 3][tk]);
      *reinterpret_cast<float4*>(d + (int64_t)(n0 + tk) * kDim + c0 + cq) = v;
      if (dp != nullptr)
        store_planes4(dp + (int64_t)(n0 + tk) * kDim + c0 + cq, (int64_t)n * kDim, args.npl, v);
    }
  }
}

// Linear-attention source state.  The qkv GEMM's epilogue (EPI_QKV) leaves, per 32-token
// chunk, KVpart[h][d][q] = sum_m phi(k)[m][h,d] v[m][h,q]/Ns  (einsum 'bdhm,bqhm->bqdh', :96)
// and kspart[h*64+d] = sum_m phi(k)[m][h,d]  (key.sum(3), :97); kv_reduce sums the chunks.
struct KvProb {
  const float* part;  // [B][chunks][4][64][64]
  const float* kspart;  // [B][chunks][256]
  int chunks;
};
struct KvArgs {
  KvProb p[2];
};

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// Sum the chunk partials -> KV[h][d][q], ksum[256].  Each workgroup owns 64 float4 outputs
// of one (source, sample); its four waves sum interleaved quarters of the chunks (eight
// loads in flight each) and the quarters are added in a fixed order (deterministic).
__global__ __launch_bounds__(256) void kv_reduce_kernel(KvArgs args, float* kv, float* ksum,
                                                        int batch) {
  constexpr int per = (16384 + 256) / 4;   // float4 outputs per (source, sample) = 4160
  constexpr int groups = per / 64;         // 65 workgroups per (source, sample)
  __shared__ float4 red[4][64];
  const int g = blockIdx.x % groups, bs = blockIdx.x / groups;
  const int b = bs % batch, src = bs / batch;
  const KvProb& P = src ? args.p[1] : args.p[0];
  const int lane = threadIdx.x & 63, q4 = threadIdx.x >> 6;
  const int e4 = g * 64 + lane;
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
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int c = q4;
  for (; c + 28 < P.chunks; c += 32) {
    float4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = p[(int64_t)(c + 4 * j) * stride];
#pragma unroll
    for (int j = 0; j < 8; ++j) { acc.x += v[j].x; acc.y += v[j].y; acc.z += v[j].z; acc.w += v[j].w; }
  }
  for (; c < P.chunks; c += 4) {
    const float4 v = p[(int64_t)c * stride];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  red[q4][lane] = acc;
  __syncthreads();
  if (q4 == 0) {
    float4 s = red[0][lane];
#pragma unroll
    for (int j = 1; j < 4; ++j) { s.x += red[j][lane].x; s.y += red[j][lane].y; s.z += red[j][lane].z; s.w += red[j][lane].w; }
    *out = s;
  }
}

// Folded message weights, per (side, sample, head h, 64-row block of o):
//   Mf[o][h*64+d] = sum_q C[o][h*64+q] * KV_src[h][d][q]
// so that  W1b merge(attention(x, src)) = Mf (phi(q) * Z * Ns)  (GATs_SuperGlue.py:96-98,
// :119-120, then mlp[0]).  64x64 output, K = 64, 2x2 waves of 32x32 MFMA tiles; operands
// are L2-resident (C: 512 KB per layer, KV: 64 KB per source).
struct FoldProb {
  const float* kv;    // [B][4][64][64] of the source
  float* mf;          // [B][512][256] fp32, or [B][3][512][256] bf16 planes (planes != 0)
};
struct FoldArgs {
  FoldProb p[2];
  const float* c;     // [512][256]
  int planes;         // bf16 modes: Mf as the exact hi / mid / lo planes (GemmProb::Wp1)
};
constexpr int64_t kMfElems = 512 * 256;
constexpr int64_t kMfFloats = 3 * kMfElems / 2;   // a sample's Mf region (room for the planes;
                                                  // the fp32 Mf uses its first kMfElems)

// x -> (hi, mid, lo): the exact split of gemm.hip's store_quad_bf16
__device__ __forceinline__ void split_bf16(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r = x - (float)h;
  m = (__bf16)r;
  l = (__bf16)(r - (float)m);
}
__global__ __launch_bounds__(256) void m_fold_kernel(FoldArgs args, int batch) {
  const int ot = blockIdx.x & 7, h = (blockIdx.x >> 3) & 3;
  const int bs = blockIdx.x >> 5, b = bs % batch, side = bs / batch;
  const FoldProb& P = side ? args.p[1] : args.p[0];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1, half = lane >> 5, l32 = lane & 31;
  const float* a = args.c + (int64_t)(ot * 64 + wm * 32 + l32) * 256 + h * 64 + half * 4;
  const float* w = P.kv + (int64_t)b * 16384 + h * 4096 + (wn * 32 + l32) * 64 + half * 4;
  floatx16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const float4 av = *reinterpret_cast<const float4*>(a + kk * 8);
    const float4 wv = *reinterpret_cast<const float4*>(w + kk * 8);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, wv.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, wv.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, wv.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, wv.w, acc, 0, 0, 0);
  }
  const int64_t e0 = (int64_t)(ot * 64 + wm * 32) * 256 + h * 64 + wn * 32 + l32;
  if (args.planes) {
    __bf16* out = reinterpret_cast<__bf16*>(P.mf) + (int64_t)b * 3 * kMfElems + e0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int64_t e = ((i & 3) + 8 * (i >> 2) + 4 * half) * 256;
      split_bf16(acc[i], out[e], out[kMfElems + e], out[2 * kMfElems + e]);
    }
    return;
  }
  float* out = P.mf + (int64_t)b * kMfFloats + e0;
#pragma unroll
  for (int i = 0; i < 16; ++i) out[((i & 3) + 8 * (i >> 2) + 4 * half) * 256] = acc[i];
}

// kv_reduce and m_fold in one launch (whole frames): a workgroup that has reduced KV_h rows
// d0..d0+3 of one source also owns Mf columns h*64 + d0..d0+3 of the side attending to it,
// since  Mf[o][h*64+d] = sum_q C[o][h*64+q] KV_h[d][q]  reads only those rows; the fold reads
// CT[h][q][o], the per-head transpose of C (coalesced over o).  Workgroup 64 of each (source,
// sample) is sum phi(k) (chunk sum only).
struct KvFoldArgs {
  KvProb p[2];     // chunk partials of source slot 0 / 1
  float* mf[2];    // Mf of the side that attends to slot 0 / 1 (FoldProb::mf's layouts)
  const float* ct; // [4][64][512]  C transposed per head (packed weights)
  int planes;      // bf16 modes: Mf as bf16 planes
};
typedef float f2v __attribute__((ext_vector_type(2)));

// kv_fold on 256-thread workgroups (88 VGPRs), small enough to share a CU with the other frame's
// GEMM workgroups (a 1024-thread form, 16 waves and 40 KB LDS, measured the same in the frame).
// The chunk sum is kv_reduce's (wave w sums chunks w, w+4, ... in order, the four wave sums
// added in wave order), so KV / ksum equal kv_reduce's bit for bit.  The fold: KVF_OSPLIT
// workgroups share a KV row block, each folding 512 / KVF_OSPLIT rows of Mf, so each reads that
// share of C_h (a 512-row workgroup reads all 128 KB of it, 16 MB per launch at config 2, and
// was the slower half of the kernel: 1625 -> 1627 frames/s, kv_fold 9.5 -> 8.7 us per launch
// with launch overhead, `tools/ab_multi.sh`); q quarters accumulated in q order, then added in
// quarter order.
constexpr int KVF_DEPTH = 16;   // chunk loads in flight per lane
constexpr int KVF_OSPLIT = 2;   // Mf row blocks per KV row block (256 Mf rows per workgroup)
__global__ __launch_bounds__(256) void kv_fold256_kernel(KvFoldArgs args, float* kv, float* ksum,
                                                         int batch) {
  constexpr int OS = KVF_OSPLIT;
  constexpr int groups = 64 * OS + 1;      // workgroups per (source, sample); the last: sum phi(k)
  __shared__ float4 red[4][64];            // wave sums; then KV rows d0..d0+3
  const int gb = blockIdx.x % groups, bs = blockIdx.x / groups;
  const int b = bs % batch, src = bs / batch;
  const KvProb& P = src ? args.p[1] : args.p[0];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const bool ks_wg = gb == 64 * OS;
  const int g = ks_wg ? 64 : gb % 64, os = ks_wg ? 0 : gb / 64;   // KV row block, Mf row block
  const int e4 = g * 64 + lane;
  const int h = (g >> 4) & 3, d0 = (g & 15) * 4;
  // uniform base + 32-bit lane offsets: one VGPR per load address
  const bool kvrow = g < 64;
  const float4* base = kvrow
      ? reinterpret_cast<const float4*>(P.part + (int64_t)b * P.chunks * 16384)
      : reinterpret_cast<const float4*>(P.kspart + (int64_t)b * P.chunks * 256);
  const int stride = kvrow ? 4096 : 64;
  const int idx = kvrow ? e4 : e4 - 4096;
  // Up to KVF_DEPTH chunk loads in flight per lane (config 2 at 16: one round for either
  // side; the predicated-off slots add nothing, and the adds keep kv_reduce's order: chunk w,
  // w + 4, ...)
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int c = w; c < P.chunks; c += 4 * KVF_DEPTH) {
    float4 v[KVF_DEPTH];
#pragma unroll
    for (int j = 0; j < KVF_DEPTH; ++j)
      v[j] = c + 4 * j < P.chunks ? base[idx + (c + 4 * j) * stride] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < KVF_DEPTH; ++j) { acc.x += v[j].x; acc.y += v[j].y; acc.z += v[j].z; acc.w += v[j].w; }
  }
  // the fold's first quarter of C (independent of KV) is in flight across the reduction below
  const int o = os * 256 + t;   // Mf row o
  const float* ct = args.ct + (h * 64) * 512 + o;
  float cv[16];
  if (g != 64) {
#pragma unroll
    for (int i = 0; i < 16; ++i) cv[i] = *reinterpret_cast<const std::remove_reference_t<decltype(cv[0])>*>(ct + i * 512);
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0) {
    float4 s = red[0][lane];
#pragma unroll
    for (int j = 1; j < 4; ++j) { s.x += red[j][lane].x; s.y += red[j][lane].y; s.z += red[j][lane].z; s.w += red[j][lane].w; }
    if (os == 0) {   // (every Mf row block sums the same KV rows)
      if (e4 < 4096)
        reinterpret_cast<float4*>(kv + ((int64_t)src * batch + b) * 16384)[e4] = s;
      else
        reinterpret_cast<float4*>(ksum + ((int64_t)src * batch + b) * 256)[e4 - 4096] = s;
    }
    red[0][lane] = s;   // KV rows d0..d0+3: red[0][16 j + q/4] = KV_h[d0 + j][q .. q+3]
  }
  if (g == 64) return;
  __syncthreads();
  const float* kvr = reinterpret_cast<const float*>(&red[0][0]);
  // one Mf row per thread, its four d as two packed pairs (d0, d0 + 1), (d0 + 2, d0 + 3); q
  // quarters accumulated in q order, then added in quarter order
  f2v y01, y23;
#pragma unroll
  for (int qq = 0; qq < 4; ++qq) {
    if (qq > 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) cv[i] = ct[(qq * 16 + i) * 512];
    }
    f2v a01 = (f2v)(0.f), a23 = (f2v)(0.f);
#pragma unroll
    for (int i = 0; i < 16; i += 4) {
      const float4 k0 = *reinterpret_cast<const float4*>(kvr + 0 * 64 + qq * 16 + i);
      const float4 k1 = *reinterpret_cast<const float4*>(kvr + 1 * 64 + qq * 16 + i);
      const float4 k2 = *reinterpret_cast<const float4*>(kvr + 2 * 64 + qq * 16 + i);
      const float4 k3 = *reinterpret_cast<const float4*>(kvr + 3 * 64 + qq * 16 + i);
      a01 = __builtin_elementwise_fma((f2v)(cv[i]), (f2v){k0.x, k1.x}, a01);
      a23 = __builtin_elementwise_fma((f2v)(cv[i]), (f2v){k2.x, k3.x}, a23);
      a01 = __builtin_elementwise_fma((f2v)(cv[i + 1]), (f2v){k0.y, k1.y}, a01);
      a23 = __builtin_elementwise_fma((f2v)(cv[i + 1]), (f2v){k2.y, k3.y}, a23);
      a01 = __builtin_elementwise_fma((f2v)(cv[i + 2]), (f2v){k0.z, k1.z}, a01);
      a23 = __builtin_elementwise_fma((f2v)(cv[i + 2]), (f2v){k2.z, k3.z}, a23);
      a01 = __builtin_elementwise_fma((f2v)(cv[i + 3]), (f2v){k0.w, k1.w}, a01);
      a23 = __builtin_elementwise_fma((f2v)(cv[i + 3]), (f2v){k2.w, k3.w}, a23);
    }
    y01 = qq == 0 ? a01 : y01 + a01;
    y23 = qq == 0 ? a23 : y23 + a23;
  }
  const int64_t e0 = (int64_t)o * 256 + h * 64 + d0;
  if (args.planes) {
    bf16x4 q0, q1, q2;
    const float y[4] = {y01.x, y01.y, y23.x, y23.y};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      __bf16 h, m, l;
      split_bf16(y[c], h, m, l);
      q0[c] = h;
      q1[c] = m;
      q2[c] = l;
    }
    __bf16* mp = reinterpret_cast<__bf16*>(src ? args.mf[1] : args.mf[0]) + (int64_t)b * 3 * kMfElems + e0;
    *reinterpret_cast<bf16x4*>(mp) = q0;
    *reinterpret_cast<bf16x4*>(mp + kMfElems) = q1;
    *reinterpret_cast<bf16x4*>(mp + 2 * kMfElems) = q2;
    return;
  }
  float* mf = (src ? args.mf[1] : args.mf[0]) + (int64_t)b * kMfFloats + e0;
  *reinterpret_cast<float4*>(mf) = make_float4(y01.x, y01.y, y23.x, y23.y);
}

// InstanceNorm1d statistics (GATs_SuperGlue.py:145; biased variance, eps 1e-5): per-64-row-tile
// (mean, M2) partials from MLP conv 1, Chan-merged (double) in tile order by the last tile of
// each column block inside that launch (gemm.hip, EPI_STATS with st_cnt).
struct StatsProb {
  const float* part;  // [B][mtiles][2][512]
  float* mean;        // [B][512]
  float* rstd;
  int m, mtiles, rows;   // tokens, partial tiles, rows per tile
};
struct StatsArgs {
  StatsProb p[2];
};
// ---- N3-sharded frames (onepose_match_sharded): per-rank partials and their merges ----
// Every exchange is an all-gather of a fixed-size block per rank (rank-major in `recv`), merged
// in rank order, so results do not depend on the collective's reduction order.

// dst[i] = sum_r recv[r * block + off + i]   (KV and sum phi(k) of the sharded 3D side)
__global__ __launch_bounds__(256) void shard_sum_kernel(const float* recv, int world,
                                                        int64_t block, int64_t off, int64_t count,
                                                        float* dst) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= count) return;
  float s = 0.f;
  for (int r = 0; r < world; ++r) s += recv[r * block + off + i];
  dst[i] = s;
}

// This rank's (n, mean, M2) per channel of the 3D side's MLP hidden layer: out[b][c][3] doubles
__global__ __launch_bounds__(256) void stats_partial_kernel(StatsProb P, int batch, double* out) {
  __shared__ double red[3][16][17];
  const int g = blockIdx.x & 31, b = blockIdx.x >> 5;
  const int t = threadIdx.x, tg = t >> 4, cl = t & 15, c = g * 16 + cl;
  const float* part = P.part + (int64_t)b * P.mtiles * 1024;
  double n = 0.0, mean = 0.0, m2 = 0.0;
  for (int ti = tg; ti < P.mtiles; ti += 16) {
    const double nb = (double)min(P.rows, P.m - ti * P.rows);
    chan_merge(n, mean, m2, nb, part[ti * 1024 + c], part[ti * 1024 + 512 + c]);
  }
  red[0][tg][cl] = n;
  red[1][tg][cl] = mean;
  red[2][tg][cl] = m2;
  __syncthreads();
  if (tg == 0) {
    for (int k = 1; k < 16; ++k) chan_merge(n, mean, m2, red[0][k][cl], red[1][k][cl], red[2][k][cl]);
    double* o = out + ((int64_t)b * 512 + c) * 3;
    o[0] = n;
    o[1] = mean;
    o[2] = m2;
  }
}

// Chan-merge the ranks' (n, mean, M2) in rank order -> InstanceNorm mean / rstd
__global__ __launch_bounds__(256) void stats_merge_kernel(const double* recv, int world,
                                                          int64_t block, int batch, float* mean,
                                                          float* rstd) {
  const int i = blockIdx.x * 256 + threadIdx.x;   // (b, c)
  if (i >= batch * 512) return;
  double n = 0.0, mu = 0.0, m2 = 0.0;
  for (int r = 0; r < world; ++r) {
    const double* q = recv + r * block + (int64_t)i * 3;
    chan_merge(n, mu, m2, q[0], q[1], q[2]);
  }
  mean[i] = (float)mu;
  rstd[i] = (float)(1.0 / sqrt(m2 / n + 1e-5));
}

// Row softmax statistics over every rank's columns: max of maxima, rescaled sum of sums
__global__ __launch_bounds__(256) void rowstat_merge_kernel(const float* recv, int world,
                                                            int64_t block, int64_t rows,
                                                            float* rowmax, float* rowsum) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows) return;
  float mx = -INFINITY;
  for (int r = 0; r < world; ++r) mx = fmaxf(mx, recv[r * block + i]);
  float s = 0.f;
  for (int r = 0; r < world; ++r) {
    const float m = recv[r * block + i];
    s += recv[r * block + rows + i] * expf(m - mx);
  }
  rowmax[i] = mx;
  rowsum[i] = s;
}

// Row winners (packed value | global column) across ranks: unsigned max
__global__ __launch_bounds__(256) void best_max_kernel(const unsigned long long* recv, int world,
                                                       int64_t block, int64_t count,
                                                       unsigned long long* dst) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= count) return;
  unsigned long long k = 0ull;
  for (int r = 0; r < world; ++r) k = recv[r * block + i] > k ? recv[r * block + i] : k;
  dst[i] = k;
}

// colbest [B][n3s] -> send [B][max_shard] (padded rank block)
__global__ __launch_bounds__(256) void colbest_pack_kernel(const unsigned long long* src, int batch,
                                                           int n3s, int max_shard,
                                                           unsigned long long* send) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)batch * max_shard) return;
  const int b = (int)(i / max_shard), j = (int)(i - (int64_t)b * max_shard);
  send[i] = j < n3s ? src[(int64_t)b * n3s + j] : 0ull;
}

// Every rank's column winners at their global columns: full [B][n3_total]
__global__ __launch_bounds__(256) void colbest_assemble_kernel(const unsigned long long* recv,
                                                               int world, int64_t block,
                                                               int batch, int n3_total,
                                                               int max_shard,
                                                               unsigned long long* full) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;   // (b, global column)
  if (i >= (int64_t)batch * n3_total) return;
  const int b = (int)(i / n3_total), col = (int)(i - (int64_t)b * n3_total);
  // rank owning col: start_r = floor(n3_total * r / world)
  int r = (int)(((int64_t)col * world) / n3_total);
  while (r + 1 < world && (int64_t)n3_total * (r + 1) / world <= col) ++r;
  while (r > 0 && (int64_t)n3_total * r / world > col) --r;
  const int start = (int)((int64_t)n3_total * r / world);
  full[i] = recv[r * block + (int64_t)b * max_shard + (col - start)];
}

// GraphAttentionLayer (GATs.py:62-123) with include_self=True, with_linear_transform=False,
// additional=False, concat=True, W a folded (h.(W a) == (h W) a):
//   s3 = h3.wa_hi, s2_j = leaf_j.wa_lo, e = LeakyReLU_0.2(s3 + [s3, s2_1..L])
//   alpha = softmax(e), out = ELU(alpha_0 h3 + sum_j alpha_j leaf_j)
// One wave per 3D point over point-major leaves [n3][L][256]: each leaf row is one 1 KB
// coalesced load (a float4 per lane), the L+1 logits are wave reductions, softmax and ELU run
// in registers -- no LDS, every leaf byte crosses HBM once per layer.
//
// The leaf logits s2_j = leaf_j.wa_lo depend on the object alone (the leaves never change
// across layers, GATs_SuperGlue.py:70-72).  onepose_object_prepare stores them for GAT layers
// 1-3 (gat_logits_kernel, kLogitStride per point); a cached forward's GAT then reduces only
// s3.  Both kernels form a logit with gat_dot + gat_wave_sum, so a stored logit has the bits
// the in-kernel one would have.
constexpr int kLogitStride = 16;   // stored leaf logits per point (num_leaf <= 16)

__device__ __forceinline__ float gat_dot(float4 a, float4 w) {
  return fmaf(a.w, w.w, fmaf(a.z, w.z, fmaf(a.y, w.y, a.x * w.x)));
}

template <int MAXL>
__global__ __launch_bounds__(256) void gat_logits_kernel(const float* __restrict__ leaves_pm,
                                                         const float* __restrict__ wa1,
                                                         float* __restrict__ out, int n3, int L) {
  // wa1: GAT layer 1's packed vectors; layers 2 and 3 follow at +kGatFloats (512) each.
  // out[(g - 1)][p][kLogitStride]
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= n3) return;
  const int lane = threadIdx.x & 63;
  const float* lp = leaves_pm + (int64_t)p * L * kDim;
  float4 lf[MAXL];
#pragma unroll
  for (int j = 0; j < MAXL; ++j)
    if (j < L) lf[j] = reinterpret_cast<const float4*>(lp + j * kDim)[lane];
  for (int g = 0; g < 3; ++g) {
    const float4 wl = reinterpret_cast<const float4*>(wa1 + g * 512)[lane];
    float d[MAXL];
#pragma unroll
    for (int j = 0; j < MAXL; ++j) d[j] = (j < L) ? gat_dot(lf[j], wl) : 0.f;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
      for (int j = 0; j < MAXL; ++j) d[j] += __shfl_xor(d[j], o, 64);
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < MAXL; ++j) v = lane == j ? d[j] : v;
    if (lane < L) out[((int64_t)g * n3 + p) * kLogitStride + lane] = v;
  }
}

// slog: the stored leaf logits of this layer ([n3][kLogitStride], shared by the batch) or null.
template <int MAXL>
__global__ __launch_bounds__(256) void gat_kernel(const float* __restrict__ x3,
                                                  const float* __restrict__ leaves_pm,
                                                  int64_t leaves_bs, const float* __restrict__ wa,
                                                  const float* __restrict__ slog,
                                                  float* __restrict__ y3, int n3, int L,
                                                  int batch, uint16_t* __restrict__ y3p,
                                                  int npl) {
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int b = gw / n3, p = gw - b * n3;
  if (b >= batch) return;
  const int lane = threadIdx.x & 63;
  const float4 wh = reinterpret_cast<const float4*>(wa + 256)[lane];
  const float4 h = reinterpret_cast<const float4*>(x3 + ((int64_t)b * n3 + p) * kDim)[lane];
  const float* lp = leaves_pm + b * leaves_bs + (int64_t)p * L * kDim;
  float4 lf[MAXL];
#pragma unroll
  for (int j = 0; j < MAXL; ++j)
    if (j < L) lf[j] = reinterpret_cast<const float4*>(lp + j * kDim)[lane];
  float d[MAXL + 1];
  d[0] = gat_dot(h, wh);
  if (slog != nullptr) {
    // wave-uniform point: the logits come in through scalar loads
    const int pu = __builtin_amdgcn_readfirstlane(p);
    const float* sl = slog + (int64_t)pu * kLogitStride;
#pragma unroll
    for (int j = 0; j < MAXL; ++j) d[j + 1] = (j < L) ? sl[j] : 0.f;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) d[0] += __shfl_xor(d[0], o, 64);
  } else {
    const float4 wl = reinterpret_cast<const float4*>(wa)[lane];
#pragma unroll
    for (int j = 0; j < MAXL; ++j) d[j + 1] = (j < L) ? gat_dot(lf[j], wl) : 0.f;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
      for (int j = 0; j <= MAXL; ++j) d[j] += __shfl_xor(d[j], o, 64);
  }
  const float s3 = d[0];
  float e[MAXL + 1];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j <= MAXL; ++j) {
    if (j > L) break;
    float v = s3 + (j == 0 ? s3 : d[j]);
    v = v > 0.f ? v : v * 0.2f;
    e[j] = v;
    mx = fmaxf(mx, v);
  }
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j <= MAXL; ++j) {
    if (j > L) break;
    e[j] = expf(e[j] - mx);
    sum += e[j];
  }
  const float a0 = e[0] / sum;
  float4 acc = make_float4(a0 * h.x, a0 * h.y, a0 * h.z, a0 * h.w);
#pragma unroll
  for (int j = 0; j < MAXL; ++j) {
    if (j >= L) break;
    const float a = e[j + 1] / sum;
    acc.x += a * lf[j].x;
    acc.y += a * lf[j].y;
    acc.z += a * lf[j].z;
    acc.w += a * lf[j].w;
  }
  const float4 y = make_float4(elu1(acc.x), elu1(acc.y), elu1(acc.z), elu1(acc.w));
  reinterpret_cast<float4*>(y3 + ((int64_t)b * n3 + p) * kDim)[lane] = y;
  if (y3p != nullptr)   // activation planes ([B][3][n3][256]) for the next GEMM's A
    store_planes4(y3p + ((int64_t)b * kPlanesMax * n3 + p) * kDim + lane * 4, (int64_t)n3 * kDim,
                  npl, y);
}

// GAT layers 1-3 of a cached forward from per-object prefix tables (onepose_object_prepare).
// With the leaf logits s_(0) >= ... >= s_(L-1) sorted and c = s_(0), LeakyReLU splits the leaves
// at the point's own logit s3: e_j = s3 + s_j where that is > 0 (a prefix of the sorted order,
// k of them) and 0.2 (s3 + s_j) elsewhere, so
//   sum_j exp(e_j - mx) leaf_j = exp(s3 + c - mx) A_k + exp(0.2 (s3 + c) - mx) B_k,
//   A_k = sum_{i<k} exp(s_(i) - c) leaf_(i),   B_k = sum_{i>=k} exp(0.2 (s_(i) - c)) leaf_(i)
// (both factors <= 1, so nothing overflows).  A frame then reads two table rows per point
// instead of its L leaves (config 2: 16 instead of 42 MB per launch).  The sums differ from
// the direct kernel's (gat_kernel) in rounding only.
// per point 2L rows: A_1..A_L at 0..L-1, B_0..B_(L-1) at L..2L-1

// Tables for the three frame-dependent GAT layers: slogs [3][n3][kLogitStride] (sorted leaf
// logits, descending; equal logits by leaf index), tab [3][n3][2L][256].
__global__ __launch_bounds__(256) void gat_table_kernel(const float* __restrict__ leaves_pm,
                                                        const float* __restrict__ wa1,
                                                        float* __restrict__ slogs,
                                                        float* __restrict__ tab, int n3, int L) {
  constexpr int MAXL = 8;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= n3) return;
  const int lane = threadIdx.x & 63;
  const float* lp = leaves_pm + (int64_t)p * L * kDim;
  float4 lf[MAXL];
#pragma unroll
  for (int j = 0; j < MAXL; ++j)
    lf[j] = j < L ? reinterpret_cast<const float4*>(lp + j * kDim)[lane] : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int g = 0; g < 3; ++g) {
    const float4 wl = reinterpret_cast<const float4*>(wa1 + g * 512)[lane];
    float d[MAXL];
#pragma unroll
    for (int j = 0; j < MAXL; ++j) d[j] = (j < L) ? gat_dot(lf[j], wl) : 0.f;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
      for (int j = 0; j < MAXL; ++j) d[j] += __shfl_xor(d[j], o, 64);
    // rank of leaf j in descending order (ties by index), then the sorted logits / leaves
    int rk[MAXL];
#pragma unroll
    for (int j = 0; j < MAXL; ++j) {
      int r = 0;
#pragma unroll
      for (int i = 0; i < MAXL; ++i)
        r += (i < L && i != j && (d[i] > d[j] || (d[i] == d[j] && i < j))) ? 1 : 0;
      rk[j] = j < L ? r : MAXL;
    }
    float sv[MAXL];
    float4 sl[MAXL];
#pragma unroll
    for (int r = 0; r < MAXL; ++r) {
      float v = 0.f;
      float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int j = 0; j < MAXL; ++j)
        if (rk[j] == r) { v = d[j]; f = lf[j]; }
      sv[r] = v;
      sl[r] = f;
    }
    const float c = sv[0];
    float* out = tab + (((int64_t)g * n3 + p) * 2 * L) * kDim;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int r = 0; r < MAXL; ++r) {
      if (r >= L) break;
      const float wp = expf(sv[r] - c);
      a.x = fmaf(wp, sl[r].x, a.x); a.y = fmaf(wp, sl[r].y, a.y);
      a.z = fmaf(wp, sl[r].z, a.z); a.w = fmaf(wp, sl[r].w, a.w);
      reinterpret_cast<float4*>(out + r * kDim)[lane] = a;   // A_(r+1)
    }
    a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int r = MAXL - 1; r >= 0; --r) {
      if (r >= L) continue;
      const float wn = expf(0.2f * (sv[r] - c));
      a.x = fmaf(wn, sl[r].x, a.x); a.y = fmaf(wn, sl[r].y, a.y);
      a.z = fmaf(wn, sl[r].z, a.z); a.w = fmaf(wn, sl[r].w, a.w);
      reinterpret_cast<float4*>(out + (L + r) * kDim)[lane] = a;   // B_r
    }
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < MAXL; ++r) v = lane == r ? sv[r] : v;
    if (lane < L) slogs[((int64_t)g * n3 + p) * kLogitStride + lane] = v;
  }
}

// One GAT layer from the tables (slogs / tab of this layer, shared by the batch).
__global__ __launch_bounds__(256) void gat_tab_kernel(const float* __restrict__ x3,
                                                      const float* __restrict__ wa,
                                                      const float* __restrict__ slogs,
                                                      const float* __restrict__ tab,
                                                      float* __restrict__ y3, int n3, int L,
                                                      int batch, uint16_t* __restrict__ y3p,
                                                      int npl) {
  constexpr int MAXL = 8;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int b = gw / n3, p = gw - b * n3;
  if (b >= batch) return;
  const int lane = threadIdx.x & 63;
  const float4 wh = reinterpret_cast<const float4*>(wa + 256)[lane];
  const float4 h = reinterpret_cast<const float4*>(x3 + ((int64_t)b * n3 + p) * kDim)[lane];
  // the sorted logits load in the same round trip as h (they do not depend on s3)
  const int pu = __builtin_amdgcn_readfirstlane(p);
  const float* sp = slogs + (int64_t)pu * kLogitStride;
  float sv[MAXL];
#pragma unroll
  for (int r = 0; r < MAXL; ++r) sv[r] = r < L ? sp[r] : 0.f;
  float s3 = gat_dot(h, wh);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s3 += __shfl_xor(s3, o, 64);
  const float c = sv[0];
  float e0 = s3 + s3;
  e0 = e0 > 0.f ? e0 : e0 * 0.2f;
  const float v0 = s3 + c;
  const float mx = fmaxf(e0, v0 > 0.f ? v0 : v0 * 0.2f);
  int k = 0;
#pragma unroll
  for (int r = 0; r < MAXL; ++r) k += (r < L && s3 + sv[r] > 0.f) ? 1 : 0;
  const float E0 = expf(e0 - mx), Fp = expf(v0 - mx), Fn = expf(0.2f * v0 - mx);
  float sp_ = 0.f, sn = 0.f;
#pragma unroll
  for (int r = 0; r < MAXL; ++r) {
    if (r >= L) break;
    if (r < k) sp_ += expf(sv[r] - c);
    else sn += expf(0.2f * (sv[r] - c));
  }
  const float sum = E0 + Fp * sp_ + Fn * sn;
  const float* tp = tab + (int64_t)pu * 2 * L * kDim;
  const float4 A = k > 0 ? reinterpret_cast<const float4*>(tp + (k - 1) * kDim)[lane]
                         : make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 Bv = k < L ? reinterpret_cast<const float4*>(tp + (L + k) * kDim)[lane]
                          : make_float4(0.f, 0.f, 0.f, 0.f);
  const float a0 = E0 / sum, ap = Fp / sum, an = Fn / sum;
  float4 acc;
  acc.x = fmaf(an, Bv.x, fmaf(ap, A.x, a0 * h.x));
  acc.y = fmaf(an, Bv.y, fmaf(ap, A.y, a0 * h.y));
  acc.z = fmaf(an, Bv.z, fmaf(ap, A.z, a0 * h.z));
  acc.w = fmaf(an, Bv.w, fmaf(ap, A.w, a0 * h.w));
  const float4 y = make_float4(elu1(acc.x), elu1(acc.y), elu1(acc.z), elu1(acc.w));
  reinterpret_cast<float4*>(y3 + ((int64_t)b * n3 + p) * kDim)[lane] = y;
  if (y3p != nullptr)
    store_planes4(y3p + ((int64_t)b * kPlanesMax * n3 + p) * kDim + lane * 4, (int64_t)n3 * kDim,
                  npl, y);
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

// One row's (or column's) softmax statistics from its nt per-tile (max, sum exp) partials at p:
// lane l takes partials l, l + 64, ...; the max and the rescaled sum over the wave's lanes.
// Every lane returns the totals.  (conf_kernel's fused form uses the same function, so the
// statistics are the same bits.)
// (tile i's (max, sum exp) at p[i * stride], p[i * stride + 1])
__device__ __forceinline__ float2 softmax_stats_wave(const float* p, int nt, int lane,
                                                     int64_t stride = 2) {
  float mx = -INFINITY;
  for (int i = lane; i < nt; i += 64) mx = fmaxf(mx, p[stride * i]);
  mx = wave_max(mx);
  float s = 0.f;
  for (int i = lane; i < nt; i += 64) s += p[stride * i + 1] * expf(p[stride * i] - mx);
  s = wave_sum(s);
  return make_float2(mx, s);
}

// Combine the score GEMM's per-tile softmax partials: rows over N3 tiles (softmax dim 2),
// columns over N1 tiles (softmax dim 1); one wave per row / column, partials across lanes.
// Also resets the packed argmax words.
__global__ __launch_bounds__(256) void softmax_reduce_kernel(
    const float* rowpart, int ntiles3, const float* colpart, int mtiles1, int batch, int n1,
    int n3, float* rowmax, float* rowsum, float* colmax, float* colsum,
    unsigned long long* rowbest, unsigned long long* colbest) {
  const int64_t idx = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t nr = (int64_t)batch * n1, nc = (int64_t)batch * n3;
  const float* p;
  int nt;
  int64_t stride = 2;
  if (idx < nr) {
    p = rowpart + idx * ntiles3 * 2;
    nt = ntiles3;
  } else if (idx < nr + nc) {   // colpart is tile-major: [b][mtiles1][n3][2]
    const int64_t b = (idx - nr) / n3, c = (idx - nr) % n3;
    p = colpart + (b * mtiles1 * n3 + c) * 2;
    nt = mtiles1;
    stride = (int64_t)n3 * 2;
  } else {
    return;
  }
  const float2 st = softmax_stats_wave(p, nt, lane, stride);
  const float mx = st.x, s = st.y;
  if (lane == 0) {
    if (idx < nr) {
      rowmax[idx] = mx;
      rowsum[idx] = s;
      rowbest[idx] = 0ull;
    } else {
      colmax[idx - nr] = mx;
      colsum[idx - nr] = s;
      colbest[idx - nr] = 0ull;
    }
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
// plus row/column max+argmax (:256).  Workgroup = 32 rows (2D) x 256 columns (3D) on 8 waves
// (4 waves per SIMD at config 2, for the latency; 4 waves of 8 rows gave 2); wave w owns rows
// 4w..4w+3, lane l owns 4 columns (16-byte loads when n3 % 4 == 0), all loads issued before
// any use.  Row winners: in-wave reduction, then one lane per row stores its winner over the
// workgroup's 256 columns to rowpart[b][row][column tile] (plain stores; the consumers take
// the max over the ceil(n3 / 256) parts).  A 64-bit atomicMax per row and workgroup instead
// cost ~3.5 of the kernel's 12.5 us alone (tools/conf_probe.hip: 16 workgroups meet at each
// row's word).  Column winners: per thread over its rows, then over the waves in LDS, one
// atomicMax per column per workgroup (~0.5 us).
// STATS (the whole-frame path): the workgroup derives the softmax statistics it needs from the
// score GEMM's per-tile partials itself -- its 32 rows' (one wave per row, softmax_stats_wave)
// and its 256 columns' (a thread per column, softmax_stats_wave's lane-0 sum tree restated
// for nt <= kConfColTiles partials) -- instead of a softmax_reduce launch before it: the same
// bits, one dependent launch fewer on the frame's chain.  The packed column winners must be
// zero before the launch (transpose_in zeroes them).
constexpr int kConfColTiles = 16;   // column partials (score M-tiles) the fused form takes
constexpr int kConfRowTiles = 64;   // row partials (score N-tiles) the fused form takes
constexpr int kConfWaves = 8, kConfRows = 4;   // 32 rows per workgroup: 8 waves x 4 rows
template <bool VEC, bool STATS>
__global__ __launch_bounds__(kConfWaves * 64) void conf_kernel(float* S, int n1, int n3,
                                                   const float* rowmax, const float* rowsum,
                                                   const float* colmax, const float* colsum,
                                                   unsigned long long* rowpart,
                                                   unsigned long long* colbest, int write_conf,
                                                   int col_offset, const float* srow, int nt3,
                                                   const float* scol, int mt1) {
  constexpr int RW = kConfRows;
  __shared__ unsigned long long cb[kConfWaves][256];
  __shared__ float cst[2][STATS ? 256 : 1];
  const int ct = (n3 + 255) / 256;
  const int tilec = blockIdx.x % ct, tiler = blockIdx.x / ct;
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* Sb = S + (int64_t)b * n1 * n3;
  float rst[STATS ? RW : 1][2];   // STATS: the wave's rows' (max, 1 / sum)
  // The workgroup's S block first: its loads do not depend on the statistics, so they are in
  // flight while the statistics' partials load and reduce (one round trip instead of three).
  int col[4];
  bool cok[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    col[j] = tilec * 256 + (VEC ? lane * 4 + j : lane + 64 * j);
    cok[j] = col[j] < n3;
  }
  float v[RW][4];
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const int n = min(tiler * 32 + wave * RW + i, n1 - 1);
    const float* ps = Sb + (int64_t)n * n3;
    if (VEC && cok[0]) {
      const float4 q = *reinterpret_cast<const float4*>(ps + col[0]);
      v[i][0] = q.x;
      v[i][1] = q.y;
      v[i][2] = q.z;
      v[i][3] = q.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[i][j] = cok[j] ? ps[col[j]] : 0.f;
    }
  }
  if constexpr (STATS) {
    // the wave's rows' partials (nt3 <= 64: one per lane), all RW rows' loads issued together
    float rpm[RW], rps[RW];
    if (nt3 <= 64) {
#pragma unroll
      for (int i = 0; i < RW; ++i) {
        const int n = min(tiler * 32 + wave * RW + i, n1 - 1);
        const float* p = srow + ((int64_t)b * n1 + n) * nt3 * 2;
        rpm[i] = lane < nt3 ? p[2 * lane] : -INFINITY;
        rps[i] = lane < nt3 ? p[2 * lane + 1] : 0.f;
      }
    }
    {   // column tilec * 256 + t: lane 0's butterfly sum of softmax_stats_wave, nt <= 16
      const int cg = tilec * 256 + threadIdx.x;
      if (threadIdx.x < 256 && cg < n3) {
        // (tile-major partials: one 8-B load per tile, a wave's 64 columns contiguous)
        const float2* p = reinterpret_cast<const float2*>(scol) + (int64_t)b * mt1 * n3 + cg;
        float pm[kConfColTiles], ps[kConfColTiles];
#pragma unroll
        for (int i = 0; i < kConfColTiles; ++i) {
          const float2 q = i < mt1 ? p[(int64_t)i * n3] : make_float2(-INFINITY, 0.f);
          pm[i] = q.x;
          ps[i] = q.y;
        }
        float mx = -INFINITY;
#pragma unroll
        for (int i = 0; i < kConfColTiles; ++i) mx = fmaxf(mx, pm[i]);
        float v[kConfColTiles];
#pragma unroll
        for (int i = 0; i < kConfColTiles; ++i) v[i] = i < mt1 ? ps[i] * expf(pm[i] - mx) : 0.f;
        // wave_sum's xor 32 / 16 steps add zeros (lanes >= 16 hold none); xor 8 .. 1 as lane 0
        // sees them
#pragma unroll
        for (int o = kConfColTiles / 2; o >= 1; o >>= 1)
#pragma unroll
          for (int l = 0; l < o; ++l) v[l] = v[l] + v[l + o];
        cst[0][threadIdx.x] = mx;
        cst[1][threadIdx.x] = 1.0f / v[0];
      }
    }
    if (nt3 <= 64) {
      // softmax_stats_wave's arithmetic with its one loop iteration per lane unrolled: the max
      // from -inf, then 0 + the lane's rescaled sum, the same wave reductions -- the same bits
#pragma unroll
      for (int i = 0; i < RW; ++i) {
        const float mx = wave_max(lane < nt3 ? fmaxf(-INFINITY, rpm[i]) : -INFINITY);
        const float s = wave_sum(lane < nt3 ? 0.f + rps[i] * expf(rpm[i] - mx) : 0.f);
        rst[i][0] = mx;
        rst[i][1] = 1.0f / s;
      }
    } else {
#pragma unroll
      for (int i = 0; i < RW; ++i) {   // the wave's rows, one at a time (as softmax_reduce)
        const int n = min(tiler * 32 + wave * RW + i, n1 - 1);
        const float2 r = softmax_stats_wave(srow + ((int64_t)b * n1 + n) * nt3 * 2, nt3, lane);
        rst[i][0] = r.x;
        rst[i][1] = 1.0f / r.y;
      }
    }
    __syncthreads();
  }
  float cmx[4], cinv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if constexpr (STATS) {
      const int cl = VEC ? lane * 4 + j : lane + 64 * j;
      cmx[j] = cok[j] ? cst[0][cl] : 0.f;
      cinv[j] = cok[j] ? cst[1][cl] : 0.f;
    } else {
      cmx[j] = cok[j] ? colmax[(int64_t)b * n3 + col[j]] : 0.f;
      cinv[j] = cok[j] ? 1.0f / colsum[(int64_t)b * n3 + col[j]] : 0.f;
    }
  }
  // Running winners as (conf bits + 1, index): conf >= 0 (or NaN), so 32-bit unsigned order of
  // the bits is pack_best's order, and a strict > over ascending indices keeps the first one
  // (0 = none yet; bits + 1 does not wrap for any conf the kernel can produce).
  unsigned cbu[4] = {0u, 0u, 0u, 0u};
  int cbi[4] = {0, 0, 0, 0};
  unsigned long long rk[RW];   // this lane's best over its 4 columns, per row of the wave
#pragma unroll
  for (int i = 0; i < RW; ++i) rk[i] = 0ull;
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const int n = tiler * 32 + wave * RW + i;
    if (n >= n1) break;   // wave-uniform
    float rmx, rinv;
    if constexpr (STATS) {
      rmx = rst[i][0];
      rinv = rst[i][1];
    } else {
      rmx = rowmax[(int64_t)b * n1 + n];
      rinv = 1.0f / rowsum[(int64_t)b * n1 + n];
    }
    unsigned ru = 0u;
    int ri = 0;
    float c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c[j] = (expf(v[i][j] - cmx[j]) * cinv[j]) * (expf(v[i][j] - rmx) * rinv);
      const unsigned u = __float_as_uint(c[j]) + 1u;
      if (cok[j] && u > ru) { ru = u; ri = col[j]; }
      if (cok[j] && u > cbu[j]) { cbu[j] = u; cbi[j] = n; }
    }
    if (write_conf) {
      float* ps = Sb + (int64_t)n * n3;
      if (VEC && cok[0]) {
        *reinterpret_cast<float4*>(ps + col[0]) = make_float4(c[0], c[1], c[2], c[3]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (cok[j]) ps[col[j]] = c[j];
      }
    }
    rk[i] = ru ? pack_best(__uint_as_float(ru - 1u), ri + col_offset) : 0ull;
  }
  // The RW rows' maxima over the wave's 64 lanes, transposed: at the xor-32 step each lane keeps
  // half of the rows (lanes 0-31 the first half, lanes 32-63 the second) and trades the other
  // half with its partner, at xor 16 a quarter, ...; once one row is left, the remaining xor
  // steps finish it.  Lane l ends with row (l >> (6 - log2 RW))'s maximum: RW - 1 + 6 - log2 RW
  // exchanges instead of RW full butterflies (6 RW).  A max over the same keys, so the same
  // winner.
  {
    constexpr int LG = RW == 8 ? 3 : RW == 4 ? 2 : RW == 2 ? 1 : 0;
    static_assert((1 << LG) == RW, "rows per wave: a power of two <= 8");
#pragma unroll
    for (int st = 0; st < LG; ++st) {
      const int half = (RW / 2) >> st, o = 32 >> st;
      const bool hi = (lane & o) != 0;
#pragma unroll
      for (int j = 0; j < half; ++j) {
        const unsigned long long send = hi ? rk[j] : rk[half + j];
        const unsigned long long mine = hi ? rk[half + j] : rk[j];
        const unsigned long long other = shfl_xor_u64(send, o);
        rk[j] = other > mine ? other : mine;
      }
    }
    unsigned long long key = rk[0];
#pragma unroll
    for (int o = 32 >> LG; o >= 1; o >>= 1) {
      const unsigned long long other = shfl_xor_u64(key, o);
      key = other > key ? other : key;
    }
    const int n = tiler * 32 + wave * RW + (lane >> (6 - LG));
    if ((lane & ((64 >> LG) - 1)) == 0 && n < n1) rowpart[((int64_t)b * n1 + n) * ct + tilec] = key;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    cb[wave][VEC ? lane * 4 + j : lane + 64 * j] =
        cbu[j] ? pack_best(__uint_as_float(cbu[j] - 1u), cbi[j]) : 0ull;
  __syncthreads();
  {
    const int cc = threadIdx.x, cg = tilec * 256 + cc;
    if (cc < 256 && cg < n3) {
      unsigned long long k = cb[0][cc];
      for (int w = 1; w < kConfWaves; ++w) k = cb[w][cc] > k ? cb[w][cc] : k;
      if (k != 0ull) atomicMax(colbest + (int64_t)b * n3 + cg, k);
    }
  }
}

// Mutual nearest neighbour + threshold (GATs_SuperGlue.py:256-267).
// A row's winner over all columns: the max of its conf_kernel parts (ct of them).
// The parts' loads are issued 16 at a time (one round trip at config 2, ct = 16) instead of one
// per loop iteration; the max of the same keys (all >= 0), so the same winner.
__device__ __forceinline__ unsigned long long row_best(const unsigned long long* rowpart, int ct,
                                                       int64_t row) {
  const unsigned long long* q = rowpart + row * ct;
  unsigned long long k = 0ull;
  for (int i0 = 0; i0 < ct; i0 += 16) {
    unsigned long long t[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = i0 + j < ct ? q[i0 + j] : 0ull;
#pragma unroll
    for (int j = 0; j < 16; ++j) k = t[j] > k ? t[j] : k;
  }
  return k;
}

// rowbest[row] = max of the row's parts (the sharded path's exchange sends whole-row winners)
__global__ __launch_bounds__(256) void rowbest_reduce_kernel(const unsigned long long* rowpart,
                                                             int ct, int64_t rows,
                                                             unsigned long long* rowbest) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < rows) rowbest[i] = row_best(rowpart, ct, i);
}

// rowpart != null: the row winners are conf_kernel's parts (ct per row); else rowbest.
__global__ __launch_bounds__(256) void mutual_kernel(const unsigned long long* rowbest,
                                                     const unsigned long long* rowpart, int ct,
                                                     const unsigned long long* colbest,
                                                     int batch, int n1, int n3, float thr,
                                                     int64_t* matches0, int64_t* matches1,
                                                     float* ms0, float* ms1, const unsigned* err) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t nr = (int64_t)batch * n1, nc = (int64_t)batch * n3;
  if (err != nullptr && *err != 0u) {   // the forward read a stale object cache: no match
    if (idx < nr) {
      ms0[idx] = 0.f;
      matches0[idx] = -1;
    } else if (idx < nr + nc) {
      ms1[idx - nr] = 0.f;
      matches1[idx - nr] = -1;
    }
    return;
  }
  if (idx < nr) {
    const int b = (int)(idx / n1), n = (int)(idx - (int64_t)b * n1);
    const unsigned long long p = rowpart ? row_best(rowpart, ct, idx) : rowbest[idx];
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
    const int64_t r1 = (int64_t)b * n1 + i1;
    const unsigned long long p = rowpart ? row_best(rowpart, ct, r1) : rowbest[r1];
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

// MLP conv 1's finalize counters per sample: up to 512 / 32 column blocks (the 64 x 64 tile
// uses the first 512 / 64 of them), then that many per stats group
constexpr int kCntPerSide = 512 / 32;

struct Plan {
  float *x2[2], *x3[2];
  float *kvpart2, *kvpart3, *kspart2, *kspart3;
  float *kv, *ksum, *mf;
  float *phiq2, *phiq3, *y12, *y13;
  // bf16 modes: activation planes of x2 / x3 (ping-pong, as x2 / x3) and of phi(q), each
  // [B][kPlanesMax][n][256] (common.h store_planes4): the attention GEMMs' A operands
  uint16_t *x2p[2], *x3p[2], *phiq2p, *phiq3p;
  float *stats2, *stats3, *mean, *rstd;
  unsigned* cnt;      // in-launch arrival counters: [attention layer][side][B][cps]
  int ncnt, cps;      //   (cps: MLP conv 1's column-block and group counters, gemm.h st_cnt)
  double *grp2, *grp3;   // InstanceNorm group partials of the two sides (gemm.h st_grp)
  float *f2, *f3, *s;
  float *rowpart, *colpart, *rowmax, *rowsum, *colmax, *colsum;
  unsigned long long *rowbest, *colbest;
  unsigned long long* rowwin;    // [B][n1][ceil(n3 / 256)] conf_kernel's row winners per column tile
  float* leaves_pm;   // point-major copy of the leaves (onepose_match only)
  unsigned* err;      // this forward's device-side error word (set by its first kernel)
  size_t bytes;
};

// fp32 QKV tile: 32 rows; 64 rows from 256 64-row tiles of the 3D side (config 2: 384; QKV
// 14% faster alone, +0.3% frames/s) and 128 rows from 4096 (config 3/4 at B = 32).  The tile's
// rows are the KV chunk length, so wider tiles also cut the KV partials the chunk sum reads
// (config 3: 570 MB per launch at 64 rows).
// (bf16 mode: a 64 x 128 / 64-deep tile -- 8 bf16 MFMAs per wave and barrier instead of 2 --
// measured slower in the frame: MLP conv 1 67 vs 42 us per launch at config 5, its accumulators,
// head accumulators and two fragment sets need 256+ VGPRs, one wave per SIMD)
// bf16 mode: QKV and MLP conv 1 on 64 x 128 tiles (4 bf16 MFMAs per wave and stage, W planes by
// global_load_lds; config 5 QKV 0.204 -> 0.181 ms per step, config 2 bf16 1801 -> 2422 frames/s
// with the W planes); MLP conv 2 keeps 64 x 64
// (bf16 MLP conv 1 on 64 x 64 DMA-2 tiles -- 640 workgroups, two stages ahead -- measured
// slower: config 2 2962 -> 2828, config 5 1642 -> 1552 frames/s, profiles/r04/r04d/)
constexpr int kTileBf16 = TILE_64x128;
// The split mode's QKV takes the same 64 x 128 DMA tile (round 4; config 2: QKV 0.210 -> 0.189
// ms per frame, profiles/r04/sw/); its MLP conv 1 keeps 64 x 64 (64 x 128 gives 320 workgroups
// at config 2: 0.273 -> 0.313 ms per frame; a DMA stage's time follows the bytes its workgroup
// moves).
// The bf16 MLP conv 1 runs on the 64 x 128 DMA tile too (a 256 x 128 eight-wave stand-in was
// built bit-identical and measured slower in the frame: DESIGN.md section 8b, tag r05-lab).
constexpr int kTileBf16Mlp1 = kTileBf16;
// The split mode's MLP conv 1 runs on the 8-wave 128 x 128 tile (TILE_128x128W8), standing in
// for its 64 x 64 tiles (the same partials, tickets, acc0 and bits): 160 workgroups at config 2,
// one per CU, leave the other CUs to the other frame's kernels -- split line 1767 / 1772 ->
// 1878 / 1882 frames/s, same box (profiles/r05/wsplit/).  The fp32 MLP
// conv 1 measured slower on it (1699 / 1701 -> 1602 / 1609: its loop is MFMA-bound, so fewer
// CUs cost time; profiles/r05/wf32/) and keeps 64 x 64.
constexpr int kTileSplitMlp1 = TILE_128x128W8;
int mlp1_tile(int pm) {
  return pm == PM_BF16 ? kTileBf16Mlp1 : pm == PM_SPLIT3 ? kTileSplitMlp1 : kTileMLP1;
}
int mlp1_acc_tile(int pm) { return pm == PM_BF16 ? kTileBf16 : kTileMLP1; }
// make_plan sizes MLP conv 1's InstanceNorm partials (stats rows `str`), its arrival counters
// (kCntPerSide column blocks) and group partials once for every precision: each precision's
// MLP conv 1 tile must have those rows and at most that many column blocks over N = 512.
static_assert(gemm_tile_stat_rows(kTileBf16) == gemm_tile_bm(kTileMLP1) &&
                  gemm_tile_stat_rows(kTileBf16Mlp1) == gemm_tile_bm(kTileMLP1) &&
                  gemm_tile_stat_rows(kTileSplitMlp1) == gemm_tile_bm(kTileMLP1),
              "MLP conv 1 tiles of all precisions must share their partials' row count");
static_assert(512 / gemm_tile_bn(kTileMLP1) <= kCntPerSide &&
                  512 / gemm_tile_bn(kTileBf16) <= kCntPerSide &&
                  512 / gemm_tile_bn(kTileBf16Mlp1) <= kCntPerSide &&
                  512 / gemm_tile_bn(kTileSplitMlp1) <= kCntPerSide,
              "MLP conv 1 column blocks exceed the plan's counters");

// the bf16 / split modes' QKV tile (the split mode on the 128 x 128 stand-in measured no faster:
// 1874 / 1847 -> 1838 / 1855 frames/s, profiles/r05/qwide/)
int qkv_tile_planes(int pm) { (void)pm; return kTileBf16; }

int qkv_tile_for(int n3, int B) {
  const int64_t t64 = (int64_t)ceil_div(n3, 64) * 6 * (B > kFusedFoldMaxBatch ? B : 1);
  // (64 x 128 from kQkvWideTiles on through round 5; the 8-wave 128 x 128 stand-in -- 64-row KV
  // chunks, the same bits -- measured +1.1 / +1.4% frames/s at config 2 in profiles/r05/qwide/, and
  // +0.3% at 300 steps / level at 20 on the confirming run, profiles/r05/qconf/: a marginal gain)
  return t64 >= kQkvWiderTiles ? TILE_128x128 : t64 >= kQkvWideTiles ? TILE_128x128W8 : kTileKV;
}

bool valid_precision(int p) {
  return p == ONEPOSE_PREC_FP32 || p == ONEPOSE_PREC_BF16_ATTN || p == ONEPOSE_PREC_FP32_SPLIT;
}

// `planes`: carve the bf16 modes' activation planes (kPlanesMax per tensor); fp32 never reads
// them (match_impl's pl() is null there), so an fp32 plan leaves them out (+75% of
// the per-token footprint otherwise).
Plan make_plan(void* ws, int B, int n1, int n3, int L, bool with_conf, bool planes = true) {
  Carve c(ws);
  Plan p;
  const size_t t2 = (size_t)B * n1, t3 = (size_t)B * n3;
  for (int i = 0; i < 2; ++i) {
    p.x2[i] = c.take<float>(t2 * 256);
    p.x3[i] = c.take<float>(t3 * 256);
  }
  const int ch2 = ceil_div(n1, 64), ch3 = ceil_div(n3, 64);   // score tiles
  const int kvr = gemm_tile_rows(kTileKV), str = gemm_tile_bm(kTileMLP1);   // = every mlp1_tile
  p.kvpart2 = c.take<float>((size_t)B * ceil_div(n1, kvr) * 16384);
  p.kvpart3 = c.take<float>((size_t)B * ceil_div(n3, kvr) * 16384);
  p.kspart2 = c.take<float>((size_t)B * ceil_div(n1, kvr) * 256);
  p.kspart3 = c.take<float>((size_t)B * ceil_div(n3, kvr) * 256);
  p.kv = c.take<float>((size_t)2 * B * 16384);
  p.ksum = c.take<float>((size_t)2 * B * 256);
  p.mf = c.take<float>((size_t)2 * B * kMfFloats);
  p.phiq2 = c.take<float>(t2 * 256);
  p.phiq3 = c.take<float>(t3 * 256);
  p.y12 = c.take<float>(t2 * 512);
  p.y13 = c.take<float>(t3 * 512);
  const size_t npl = planes ? kPlanesMax : 0;
  for (int i = 0; i < 2; ++i) {
    p.x2p[i] = planes ? c.take<uint16_t>(t2 * 256 * npl) : nullptr;
    p.x3p[i] = planes ? c.take<uint16_t>(t3 * 256 * npl) : nullptr;
  }
  p.phiq2p = planes ? c.take<uint16_t>(t2 * 256 * npl) : nullptr;
  p.phiq3p = planes ? c.take<uint16_t>(t3 * 256 * npl) : nullptr;
  p.stats2 = c.take<float>((size_t)B * ceil_div(n1, str) * 1024);
  p.stats3 = c.take<float>((size_t)B * ceil_div(n3, str) * 1024);
  p.mean = c.take<float>((size_t)2 * B * 512);
  p.rstd = c.take<float>((size_t)2 * B * 512);
  p.cps = kCntPerSide * (1 + stats_groups(std::max(n1, n3), str));
  p.ncnt = kApLayers * 2 * B * p.cps;
  p.cnt = c.take<unsigned>((size_t)p.ncnt);
  p.grp2 = c.take<double>((size_t)B * stats_groups(n1, str) * 1024);
  p.grp3 = c.take<double>((size_t)B * stats_groups(n3, str) * 1024);
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
  p.rowwin = c.take<unsigned long long>(t2 * (size_t)ceil_div(n3, 256));
  p.colbest = c.take<unsigned long long>(t3);
  p.leaves_pm = c.take<float>(t3 * L * 256);
  p.err = c.take<unsigned>(1);
  p.bytes = align_up(c.off, 256);
  return p;
}

}  // namespace
}  // namespace onepose

// ------------------------------------------------------------------------------------
// C-ABI
// ------------------------------------------------------------------------------------
using namespace onepose;

extern "C" {

const char* onepose_last_error(void) { return g_last_error.c_str(); }
int onepose_abi_version(void) { return 6; }

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
  g_prof.device = false;
  return ONEPOSE_OK;
}

int onepose_profile_begin_device(uint64_t kind_mask) {
  clear_error();
  // per stamped kind: allocated once (graph nodes keep their sites' addresses), zeroed on
  // every call (all zero = armed)
  OP_HIP(hipDeviceSynchronize());
  for (int k = 0; k < K_NUM_KINDS; ++k) {
    if (!((kind_mask >> k) & 1ull)) continue;
    if (g_prof.acc[k] == nullptr)
      OP_HIP(hipMalloc(&g_prof.acc[k], sizeof(StampAcc) * kStampPool));
    OP_HIP(hipMemset(g_prof.acc[k], 0, sizeof(StampAcc) * kStampPool));
  }
  OP_HIP(hipDeviceSynchronize());
  g_prof.n = 0;
  g_prof.mask = kind_mask;
  g_prof.device = true;
  return ONEPOSE_OK;
}

int onepose_profile_end_device(int64_t* launches, double* total_ms, int n_kinds) {
  clear_error();
  OP_REQUIRE(g_prof.device, "profile_end_device: device stamping not active");
  g_prof.device = false;
  const uint64_t mask = g_prof.mask;
  g_prof.mask = 0;
  OP_HIP(hipDeviceSynchronize());
  std::vector<unsigned long long> tot(K_NUM_KINDS, 0ull), cnt(K_NUM_KINDS, 0ull);
  std::vector<StampAcc> pool(kStampPool);
  for (int k = 0; k < K_NUM_KINDS; ++k) {
    if (!((mask >> k) & 1ull) || g_prof.acc[k] == nullptr) continue;
    OP_HIP(hipMemcpy(pool.data(), g_prof.acc[k], sizeof(StampAcc) * kStampPool,
                     hipMemcpyDeviceToHost));
    for (const StampAcc& s : pool)   // launches past kStampRecs per site (s.overflow) dropped
      for (int e = 0; e < kStampRecs; ++e) {
        unsigned long long st = ~0ull, en = 0ull;
        for (int j = 0; j < kStampShards; ++j) {
          const StampRec& r = s.rec[e][j];
          if (r.end == 0) continue;
          st = std::min(st, ~r.nstart);
          en = std::max(en, r.end);
        }
        if (en == 0) continue;
        tot[k] += en > st ? en - st : 0ull;
        ++cnt[k];
      }
  }
  int dev = 0, khz = 0;
  OP_HIP(hipGetDevice(&dev));
  OP_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  OP_REQUIRE(khz > 0, "profile: wall clock rate unavailable");
  for (int k = 0; k < n_kinds; ++k) {
    const bool ok = k < K_NUM_KINDS;
    if (launches) launches[k] = ok ? (int64_t)cnt[k] : 0;
    if (total_ms) total_ms[k] = ok ? (double)tot[k] / khz : 0.0;
  }
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

size_t onepose_matcher_packed_bytes(void) { return (size_t)kPackedBytes; }

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
    float* wq = p;
    float* wkv = wq + 256 * 256;
    float* bq = p + kApWqkv;
    float* bkv = bq + 256;
    float* w1a = bq + kApBqkv;
    float* cw = w1a + kApW1a;
    float* b1 = cw + kApC;
    float* w2 = b1 + kApB1;
    float* b2 = w2 + kApW2;
    const float* pw[3];
    const float* pb[3];
    for (int j = 0; j < 3; ++j) {
      pw[j] = tensors[ti++];
      pb[j] = tensors[ti++];
    }
    const float* mw = tensors[ti++];   // merge [256][256]
    const float* mb = tensors[ti++];
    const float* m0w = tensors[ti++];  // mlp.0 [512][512]
    const float* m0b = tensors[ti++];
    const float* m3w = tensors[ti++];  // mlp.3 [256][512]
    const float* m3b = tensors[ti++];
    // q: packed row h*64+d <- reference row d*4+h (view(B, 64, 4, N), :116)
    for (int cp = 0; cp < 256; ++cp) {
      const int h = cp / 64, d = cp % 64, cr = d * 4 + h;
      memcpy(wq + (int64_t)cp * 256, pw[0] + (int64_t)cr * 256, 256 * sizeof(float));
      bq[cp] = pb[0][cr];
    }
    // k / v interleaved per head: rows [128h, 128h+64) = k_h, [128h+64, 128h+128) = v_h
    for (int h = 0; h < 4; ++h)
      for (int d = 0; d < 64; ++d) {
        const int cr = d * 4 + h;
        memcpy(wkv + (int64_t)(128 * h + d) * 256, pw[1] + (int64_t)cr * 256, 256 * sizeof(float));
        memcpy(wkv + (int64_t)(128 * h + 64 + d) * 256, pw[2] + (int64_t)cr * 256,
               256 * sizeof(float));
        bkv[128 * h + d] = pb[1][cr];
        bkv[128 * h + 64 + d] = pb[2][cr];
      }
    // MLP conv 1 split: x part as is; message part folded with the merge conv.  Each output is
    // one double chain over j in ascending order; the merge weight is read through a
    // transposed double copy (packed column order) and eight chains run side by side, so the
    // fold is not bound by strided loads and one dependent chain (1.09 -> 0.19 s per model on
    // this container's CPU; the same chains, the same bits).
    std::vector<double> mwt((size_t)256 * 256);   // [cp][j] = merge[j][cr(cp)]
    for (int cp = 0; cp < 256; ++cp) {   // merge input channel q*4+h -> packed h*64+q
      const int h = cp / 64, q = cp % 64, cr = q * 4 + h;
      for (int j = 0; j < 256; ++j) mwt[(size_t)cp * 256 + j] = (double)mw[(int64_t)j * 256 + cr];
    }
    for (int o = 0; o < 512; ++o) {
      memcpy(w1a + (int64_t)o * 256, m0w + (int64_t)o * 512, 256 * sizeof(float));
      const float* mo = m0w + (int64_t)o * 512 + 256;
      double bacc = (double)m0b[o];
      for (int j = 0; j < 256; ++j) bacc += (double)mo[j] * mb[j];
      b1[o] = (float)bacc;
      double arow[256];
      for (int j = 0; j < 256; ++j) arow[j] = (double)mo[j];
      for (int cp0 = 0; cp0 < 256; cp0 += 8) {
        double acc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        const double* wt = mwt.data() + (size_t)cp0 * 256;
        for (int j = 0; j < 256; ++j)
          for (int k = 0; k < 8; ++k) acc[k] += arow[j] * wt[(size_t)k * 256 + j];
        for (int k = 0; k < 8; ++k) cw[(int64_t)o * 256 + cp0 + k] = (float)acc[k];
      }
    }
    memcpy(w2, m3w, kApW2 * sizeof(float));
    memcpy(b2, m3b, kApB2 * sizeof(float));
    float* ct = b2 + kApB2;
    for (int o = 0; o < 512; ++o)
      for (int cp = 0; cp < 256; ++cp) ct[(int64_t)cp * 512 + o] = cw[(int64_t)o * 256 + cp];
    uint16_t* pl = reinterpret_cast<uint16_t*>(out + kPackedFloats) + (int64_t)ap * kApPlanes;
    split_planes(wq, kPlWqkv, pl);   // wq: the whole [768][256] panel (q rows, then k_h / v_h)
    split_planes(w1a, kPlW1a, pl + 3 * kPlWqkv);
    split_planes(w2, kPlW2, pl + 3 * (kPlWqkv + kPlW1a));
    ++ap;
  }
  float* fin = out + kApLayers * kApFloats + kGatLayers * kGatFloats;
  memcpy(fin, tensors[ti++], 256 * 256 * sizeof(float));
  memcpy(fin + 256 * 256, tensors[ti++], 256 * sizeof(float));
  return ONEPOSE_OK;
}

size_t onepose_match_workspace_bytes(int batch, int n1, int n3, int num_leaf, int with_conf) {
  clear_error();
  if (batch <= 0 || n1 <= 0 || n3 <= 0) return 0;
  OP_REQUIRE(num_leaf >= 1 && num_leaf <= 16, "workspace: num_leaf=%d", num_leaf);
  return make_plan(nullptr, batch, n1, n3, num_leaf, with_conf != 0).bytes;   // every precision
}

size_t onepose_match_workspace_bytes_ex(int batch, int n1, int n3, int num_leaf, int with_conf,
                                        int precision) {
  clear_error();
  if (batch <= 0 || n1 <= 0 || n3 <= 0 || !valid_precision(precision)) return 0;
  OP_REQUIRE(num_leaf >= 1 && num_leaf <= 16, "workspace: num_leaf=%d", num_leaf);
  return make_plan(nullptr, batch, n1, n3, num_leaf, with_conf != 0,
                   precision != ONEPOSE_PREC_FP32).bytes;
}

}  // extern "C"

extern "C" {

}  // extern "C"

namespace onepose {
namespace {

// N3-sharded execution context (onepose_match_sharded); null for a whole frame.
struct ShardCtx {
  int world, rank, n3_total, offset, max_shard;
  char* send;          // caller's exchange buffers: this rank's block / world blocks, rank-major
  char* recv;
  size_t cap;          // bytes per rank block
  onepose_allgather_fn fn;
  void* user;
  unsigned long long* colbest_full;   // [B][n3_total]
};

void shard_range(int n3_total, int world, int rank, int* start, int* count) {
  const int s0 = (int)((int64_t)n3_total * rank / world);
  const int s1 = (int)((int64_t)n3_total * (rank + 1) / world);
  *start = s0;
  *count = s1 - s0;
}

size_t shard_xchg_bytes(int B, int n1, int n3_total, int world) {
  const size_t max_shard = (size_t)(n3_total + world - 1) / world;
  size_t b = (size_t)B * (16384 + 256) * sizeof(float);      // KV + sum phi(k)
  b = std::max(b, (size_t)B * 512 * 3 * sizeof(double));     // InstanceNorm (n, mean, M2)
  b = std::max(b, (size_t)B * n1 * 8);                       // row (max, sum) / row winners
  b = std::max(b, (size_t)B * max_shard * 8);                // column winners
  return align_up(b, 256);
}

int shard_exchange(const ShardCtx& sh, size_t bytes, hipStream_t st) {
  if (bytes > sh.cap) {
    set_error("match_sharded: exchange of %zu bytes > buffer %zu", bytes, sh.cap);
    return ONEPOSE_ERR_WORKSPACE;
  }
  const int rc = sh.fn(bytes, static_cast<void*>(st), sh.user);
  if (rc != 0) {
    set_error("match_sharded: all-gather callback returned %d", rc);
    return ONEPOSE_ERR_HIP;
  }
  return ONEPOSE_OK;
}

int attention_pm(int precision) {
  return precision == ONEPOSE_PREC_BF16_ATTN ? PM_BF16
         : precision == ONEPOSE_PREC_FP32_SPLIT ? PM_SPLIT3 : PM_F32;
}
// activation planes the producers write for a GEMM operand mode (0: none, fp32)
int planes_of(int pm) { return pm == PM_BF16 ? 1 : pm == PM_SPLIT3 ? 3 : 0; }

// W of a GEMM as the packed bf16 planes (bf16 modes; gemm.h GemmProb::Wp)
void set_w_planes(GemmProb& g, const uint16_t* wp, int64_t rows_x_cols) {
  g.Wp = wp;
  g.wp_bs = 0;
  g.wpl = rows_x_cols;
}
// A of a GEMM as activation planes ([B][kPlanesMax][n][256]; bs per sample, 0 = shared)
void set_a_planes(GemmProb& g, const uint16_t* ap, int64_t bs, int n) {
  g.Ap = ap;
  g.ap_bs = bs;
  g.apl = (int64_t)n * 256;
  g.ldap = 256;
}
// the stored output's activation planes ([B][kPlanesMax][n][256])
void set_y_planes(GemmProb& g, uint16_t* yp, int n, int B) {
  (void)B;
  g.Yp = yp;
  g.yp_bs = (int64_t)kPlanesMax * n * 256;
  g.ypl = (int64_t)n * 256;
}
// MLP conv 1's second K range: the Mf planes of a Mf region (kMfFloats per sample; bs 0: shared)
void set_mf_planes(GemmProb& g, const float* mf, int64_t sample_floats) {
  g.Wp1 = reinterpret_cast<const uint16_t*>(mf);
  g.wp1_bs = sample_floats * 2;
  g.wpl1 = kMfElems;
}

// One side of an attention layer: its input state (x_bs 0 = shared by the batch: the object
// cache), where the residual output goes, its per-layer scratch, and which slot's KV it
// attends to.  Slot i of kv / ksum / mf / mean / rstd belongs to side i of the launch.
struct Side {
  const float* x;
  int64_t x_bs;
  float* xo;
  float *phiq, *kvpart, *kspart, *y1, *stats;
  int n;        // tokens (this rank's)
  float len;    // the side's full length as an attention source (Ns, v / Ns)
  int src;      // slot of the side this one attends to
  int ntile;    // token count the tile choices use (n; a sharded 3D side: the largest shard,
                // so that every rank picks the same tiles and rounds alike)
  // bf16 modes: activation planes ([B][kPlanesMax][n][256], plane stride n * 256) of x (xp,
  // xp_bs per sample; null: QKV / MLP conv 1 stage A through registers), of the output xo
  // (written by MLP conv 2) and of phi(q) (written by QKV, read by MLP conv 1)
  const uint16_t* xp = nullptr;
  int64_t xp_bs = 0;
  uint16_t* xop = nullptr;
  uint16_t* phiqp = nullptr;
};

// Choices of one attention layer that change a side's summation order: the QKV tile of the
// side (its rows are the side's KV chunk length), kv_fold vs kv_reduce + m_fold for the side as
// a source slot, and the MLP-conv-2 tile of the side.  A side's bits depend on these (and on
// nothing else about the launches), so launches whose results must agree bit for bit get the
// same choices: the object prefix (B = 1) and the 3D side of layers 1-2 in every forward; a
// cached and an uncached forward's 2D side; every rank of a sharded frame.  attention_layer
// groups the sides with equal choices into one launch per step.
struct LayerTiles {
  int qkv[2];
  bool fused_fold[2];   // indexed by source slot (= side index)
  int mlp2[2];
};

int mlp2_tile_for(int64_t t64, int pm) {
  // fp32: the 64x32 K-split tile doubles the workgroup count where 64x64 tiles would leave
  // CUs idle (config 2: 320 -> 640 tiles, 23.2 -> 19.7 us); with >= 4 tiles per CU anyway
  // (batched configs) 64x64 moves less data per FLOP (config 3: 9.5 vs 12.3 ms per step)
  // (bf16: 64 x 128 tiles -- 32- or 64-deep stages on the DMA loop -- measured slower for MLP
  // conv 2 in the frame than the register-staged 64 x 64: N = 256 gives them half the
  // workgroups; config 2: 0.138 vs 0.108 ms per step)
  if (pm == PM_SPLIT3) return t64 < kMlp2WideTiles ? kTileMLP2Split : kTileMLP2;
  if (pm == PM_BF16) return kTileMLP2;
  return t64 < kMlp2WideTiles ? kTileMLP2F32 : kTileMLP2;
}

// Every side the same choices, from the launch as a whole (layers 4-11, sharded frames).
LayerTiles layer_tiles(int qkv_n3, const Side* sd, int nside, int B, int pm, bool sharded) {
  LayerTiles t;
  const int q = pm == PM_F32 ? qkv_tile_for(qkv_n3, B) : qkv_tile_planes(pm);
  // kv_fold re-reads the whole 128 KB C_h panel per workgroup (64 of them per side and
  // sample): one launch instead of two pays at small batches; at B = 32 the separate MFMA
  // m_fold (16 KB of C per workgroup) is cheaper (config 3: 1.68 vs 2.02 ms per step).
  // Sharded: the 3D source's KV is summed over the ranks between the two.
  const bool fused = !sharded && B <= kFusedFoldMaxBatch;
  int64_t t64 = 0;
  for (int i = 0; i < nside; ++i) t64 += (int64_t)ceil_div(sd[i].ntile, 64) * 4 * B;
  const int m2 = mlp2_tile_for(t64, pm);
  for (int i = 0; i < 2; ++i) {
    t.qkv[i] = q;
    t.fused_fold[i] = fused;
    t.mlp2[i] = m2;
  }
  return t;
}

// Layers 1-2 of a whole frame: each side by itself.  The 3D side takes the object prefix's
// choices (B = 1, so the cache serves any batch), the 2D side those of its tokens alone (a
// 2D-only launch of 1024 tokens gets 32-row QKV tiles: 192 workgroups instead of 96).  Cross-
// attention 1 runs both sides' MLP conv 2 in one launch (its 3D half is per frame), so both
// take the choice over both sides there.
LayerTiles side_tiles(int n1, int n3, int B, int pm, bool cross) {
  LayerTiles t;
  t.qkv[0] = pm == PM_F32 ? qkv_tile_for(n1, B) : qkv_tile_planes(pm);
  t.qkv[1] = pm == PM_F32 ? qkv_tile_for(n3, 1) : qkv_tile_planes(pm);
  t.fused_fold[0] = B <= kFusedFoldMaxBatch;
  t.fused_fold[1] = true;
  const int64_t t2 = (int64_t)ceil_div(n1, 64) * 4 * B, t3 = (int64_t)ceil_div(n3, 64) * 4;
  t.mlp2[0] = mlp2_tile_for(cross ? t2 + t3 * B : t2, pm);
  t.mlp2[1] = cross ? t.mlp2[0] : mlp2_tile_for(t3, pm);
  return t;
}

// Object cache layout (floats; onepose_object_cache_bytes): the 3D state entering layer 2,
// GAT layers 1-3's leaf logits, cross-attention 1's frame-independent 3D half (SideCache), then,
// with ONEPOSE_OBJ_GAT_TABLES and num_leaf <= 8, GAT layers 1-3's prefix tables (sorted logits
// [3][n3][16] and [3][n3][2L][256] rows, gat_tab_kernel).
bool obj_tables(int num_leaf, int flags) {
  return (flags & ONEPOSE_OBJ_GAT_TABLES) != 0 && num_leaf <= 8;
}
struct ObjLayout {
  int64_t logits, phiq, acc, ksum, mf, phiqp, slogs, tab, hdr, total;
  bool tables;
};
ObjLayout obj_layout(int n3, int num_leaf, int flags, bool planes) {
  ObjLayout L;
  L.tables = obj_tables(num_leaf, flags);
  L.logits = (int64_t)n3 * 256;
  L.phiq = L.logits + (int64_t)3 * n3 * kLogitStride;
  L.acc = L.phiq + (int64_t)n3 * 256;
  L.ksum = L.acc + (int64_t)ceil_div(n3, 64) * 64 * 512;   // TILE_64x64 tiles of N = 512
  L.mf = L.ksum + 256;
  // phi(q)'s activation planes [kPlanesMax][n3][256] uint16 (bf16 modes only: onepose_
  // object_cache_bytes reserves them in every precision, _ex only for the bf16 ones)
  L.phiqp = L.mf + kMfFloats;
  L.slogs = L.phiqp + (planes ? (int64_t)kPlanesMax * n3 * 256 / 2 : 0);
  L.tab = L.slogs + (L.tables ? (int64_t)3 * n3 * kLogitStride : 0);
  L.hdr = L.tab + (L.tables ? (int64_t)3 * n3 * 2 * num_leaf * 256 : 0);   // CacheHdr (64 B)
  L.total = L.hdr + 16;
  return L;
}

// Cross-attention 1's frame-independent half (object cache, onepose_object_prepare): the 3D
// side enters layer 2 with the cached state, so its q projection (phi(q)), its k / v as the 2D
// side's source (sum phi(k), and the 2D side's folded weights Mf = C KV_3D) and the x range of
// its MLP conv 1 (W1a x, as raw accumulators) are the same for every frame.
struct SideCache {
  const float* phiq;   // [n3][256]  phi(q) of the 3D side
  const float* acc;    // MLP conv 1 accumulators over K [0, 256) (EPI_ACC layout, TILE_64x64)
  const float* ksum;   // [256]      sum phi(k) of the 3D side
  const float* mf;     // [512][256] the 2D side's Mf
  const uint16_t* phiqp;   // [3][n3][256] phi(q)'s activation planes (bf16 modes)
};

void launch_kv_fold(const KvFoldArgs& ka, int nslot, int B, float* kv, float* ksum, hipStream_t st) {
  hipLaunchKernelGGL(kv_fold256_kernel, dim3(nslot * B * (64 * KVF_OSPLIT + 1)), dim3(256), 0, st, ka, kv, ksum, B);
}

// AttentionPropagation (GATs_SuperGlue.py:123-132) for 1 or 2 sides, grouped into one launch
// per step wherever the sides' choices (LayerTiles) agree.  Each side's arithmetic is
// independent of the others' (per-problem tiles, per-slot reductions), so a side gives the
// same bits alone or grouped.  Sharded runs have two sides, slot 1 being the 3D shard.
// xc (cross-attention 1 of a cached forward, sides 2D / 3D): the 3D side's frame-independent
// half comes from the object cache -- QKV and the KV fold run for the 2D side only, MLP conv 1
// starts the 3D side from its cached accumulators.
int attention_layer(const ApW& w, const Side* sd, int nside, int B, const Plan& p,
                    unsigned* cnt, hipStream_t st, int pm, const ShardCtx* sh,
                    const LayerTiles& tl, const SideCache* xc = nullptr) {
  int rc;
  OP_REQUIRE(!xc || (nside == 2 && !sh), "attention layer: cached cross half");
  OP_REQUIRE(!sh || (!tl.fused_fold[0] && !tl.fused_fold[1] && tl.qkv[0] == tl.qkv[1]),
             "attention layer: sharded choices");
  const int nsrc = xc ? 1 : nside;   // sides whose QKV and KV fold run here
  // sides [i0, i1) with equal choices form one launch
  auto groups = [&](int n, auto same, auto body) -> int {
    for (int i0 = 0; i0 < n;) {
      int i1 = i0 + 1;
      while (i1 < n && same(i0, i1)) ++i1;
      const int r = body(i0, i1);
      if (r != ONEPOSE_OK) return r;
      i0 = i1;
    }
    return ONEPOSE_OK;
  };
  // 1. [q | k_h v_h ...]: phi(q) stored, per-chunk KV / ksum partials
  // activation planes (bf16 modes): A by DMA where every side of a launch has them; phi(q)'s
  // planes written where every side has a buffer for them
  auto all_of = [&](int i0, int i1, auto pred) {
    for (int i = i0; i < i1; ++i)
      if (!pred(i)) return false;
    return true;
  };
  rc = groups(nsrc, [&](int a, int b) { return tl.qkv[a] == tl.qkv[b]; }, [&](int i0, int i1) -> int {
    GemmArgs a;
    a.nprob = i1 - i0;
    const bool ap = pm != PM_F32 && all_of(i0, i1, [&](int i) { return sd[i].xp != nullptr; });
    const bool yp = pm != PM_F32 && all_of(i0, i1, [&](int i) { return sd[i].phiqp != nullptr; });
    for (int i = i0; i < i1; ++i) {
      const Side& s = sd[i];
      GemmProb& g = a.p[i - i0];
      g = gemm_prob(s.x, 256, w.wqkv, 256, w.bqkv, s.phiq, 256, s.n, 768, 256, B);
      g.a0_bs = s.x_bs;
      g.vdiv = s.len;
      g.kvpart = s.kvpart;
      g.kspart = s.kspart;
      g.y_bs = (int64_t)s.n * 256;
      if (pm != PM_F32) set_w_planes(g, w.wqkv_p, kPlWqkv);
      if (ap) set_a_planes(g, s.xp, s.xp_bs, s.n);
      if (yp) set_y_planes(g, s.phiqp, s.n, B);
    }
    return gemm_launch(EPI_QKV, PRO_PLAIN, tl.qkv[i0], a, st, K_QKV_GEMM, pm);
  });
  if (rc != ONEPOSE_OK) return rc;
  // 2+3. KV[slot], ksum[slot] and the folded message weights Mf of the side attending to the
  // slot: kv_fold (one launch), or kv_reduce + m_fold (sharded: the 3D source's KV is summed
  // over the ranks between the two).  A launch over slots [i0, i1) writes their KV / ksum at
  // their own slot offsets.
  int reader[2] = {-1, -1};   // the side attending to slot i
  for (int i = 0; i < nside; ++i) reader[sd[i].src] = i;
  for (int i = 0; i < nsrc; ++i)
    OP_REQUIRE(reader[i] >= 0, "attention layer: source slot %d has no reader", i);
  auto mf_of = [&](int side) { return p.mf + (size_t)side * B * kMfFloats; };
  // bf16 modes: W operands as bf16 planes (gemm.h GemmProb::Wp)
  const bool planes = pm != PM_F32;
  auto chunks = [&](int i) { return ceil_div(sd[i].n, gemm_tile_stat_rows(tl.qkv[i])); };
  rc = groups(nsrc, [&](int a, int b) { return tl.fused_fold[a] == tl.fused_fold[b]; },
              [&](int i0, int i1) -> int {
    float* kv = p.kv + (size_t)i0 * B * 16384;
    float* ksum = p.ksum + (size_t)i0 * B * 256;
    const int ns = i1 - i0;
    if (tl.fused_fold[i0]) {
      KvFoldArgs ka;
      ka.ct = w.ct;
      ka.planes = planes ? 1 : 0;
      for (int i = i0; i < i1; ++i) {
        ka.p[i - i0] = {sd[i].kvpart, sd[i].kspart, chunks(i)};
        ka.mf[i - i0] = mf_of(reader[i]);
      }
      prof_pre(K_KV_REDUCE, st);
      launch_kv_fold(ka, ns, B, kv, ksum, st);
      prof_post(K_KV_REDUCE, st);
      OP_LAUNCHED();
      return (int)ONEPOSE_OK;
    }
    KvArgs kva;
    for (int i = i0; i < i1; ++i) kva.p[i - i0] = {sd[i].kvpart, sd[i].kspart, chunks(i)};
    OP_LAUNCH(K_KV_REDUCE, st, kv_reduce_kernel, dim3(ns * B * 65), dim3(256), 0, st, kva, kv,
              ksum, B);
    if (sh && i1 == 2) {   // the 3D side's KV / sum phi(k) over every rank's points
      const int64_t nkv = (int64_t)B * 16384, nks = (int64_t)B * 256;
      OP_HIP(hipMemcpyAsync(sh->send, p.kv + nkv, nkv * 4, hipMemcpyDeviceToDevice, st));
      OP_HIP(hipMemcpyAsync(sh->send + nkv * 4, p.ksum + nks, nks * 4, hipMemcpyDeviceToDevice,
                            st));
      int r = shard_exchange(*sh, (nkv + nks) * 4, st);
      if (r != ONEPOSE_OK) return r;
      const float* rv = reinterpret_cast<const float*>(sh->recv);
      OP_LAUNCH(K_KV_REDUCE, st, shard_sum_kernel, dim3((unsigned)ceil_div((int)nkv, 256)),
                dim3(256), 0, st, rv, sh->world, nkv + nks, (int64_t)0, nkv, p.kv + nkv);
      OP_LAUNCH(K_KV_REDUCE, st, shard_sum_kernel, dim3((unsigned)ceil_div((int)nks, 256)),
                dim3(256), 0, st, rv, sh->world, nkv + nks, nkv, nks, p.ksum + nks);
    }
    FoldArgs fa;   // Mf of the sides attending to these slots
    fa.c = w.c;
    fa.planes = planes ? 1 : 0;
    for (int i = i0; i < i1; ++i)
      fa.p[i - i0] = {p.kv + (size_t)i * B * 16384, mf_of(reader[i])};
    OP_LAUNCH(K_MFOLD, st, m_fold_kernel, dim3(ns * B * 32), dim3(256), 0, st, fa, B);
    return (int)ONEPOSE_OK;
  });
  if (rc != ONEPOSE_OK) return rc;
  {  // 4. MLP conv 1 on [x ; phi(q)] with [W1a | Mf], the phi(q) heads scaled by Z * Ns
     //    in-kernel (PRO_HEADZ), + InstanceNorm partials
    GemmArgs a;
    a.nprob = nside;
    // A planes: x's (the cached 3D half of cross-attention 1 starts from acc0 and never reads
    // its x range) and phi(q)'s
    const bool ap = pm != PM_F32 && all_of(0, nside, [&](int i) {
      const bool cached = xc && i == 1;
      return (cached || sd[i].xp != nullptr) &&
             (cached ? xc->phiqp != nullptr : sd[i].phiqp != nullptr);
    });
    for (int i = 0; i < nside; ++i) {
      const Side& s = sd[i];
      a.p[i] = gemm_prob(s.x, 256, w.w1a, 256, w.b1, s.y1, 512, s.n, 512, 512, B);
      a.p[i].a0_bs = s.x_bs;
      a.p[i].A1 = s.phiq;
      a.p[i].lda1 = 256;
      a.p[i].a1_bs = (int64_t)s.n * 256;
      a.p[i].ksplit = 256;
      a.p[i].W1 = mf_of(i);
      a.p[i].ldw1 = 256;
      a.p[i].w1_bs = kMfFloats;
      if (planes) {
        set_w_planes(a.p[i], w.w1a_p, kPlW1a);
        set_mf_planes(a.p[i], mf_of(i), kMfFloats);
      }
      a.p[i].stats = s.stats;
      a.p[i].st_cnt = cnt + (size_t)i * B * p.cps;
      a.p[i].st_cnt_bs = p.cps;
      a.p[i].st_grp = s.stats == p.stats2 ? p.grp2 : p.grp3;
      a.p[i].st_mean = p.mean + (size_t)i * B * 512;
      a.p[i].st_rstd = p.rstd + (size_t)i * B * 512;
      a.p[i].ksum = p.ksum + (size_t)s.src * B * 256;
      a.p[i].ksum_bs = 256;
      a.p[i].ns = sd[s.src].len;
    }
    if (xc) {   // the object's halves: shared by the batch (batch stride 0)
      a.p[0].W1 = xc->mf;
      a.p[0].w1_bs = 0;
      if (planes) set_mf_planes(a.p[0], xc->mf, 0);
      a.p[0].ksum = xc->ksum;
      a.p[0].ksum_bs = 0;
      a.p[1].A1 = xc->phiq;
      a.p[1].a1_bs = 0;
      a.p[1].acc0 = xc->acc;
      a.p[1].acc0_bs = 0;
    }
    if (ap) {
      for (int i = 0; i < nside; ++i) {
        const bool cached = xc && i == 1;
        const uint16_t* qp = cached ? xc->phiqp : sd[i].phiqp;
        const int64_t qbs = cached ? 0 : (int64_t)kPlanesMax * sd[i].n * 256;
        // (the cached side's x range is skipped: its A0 planes are never read)
        set_a_planes(a.p[i], cached ? qp : sd[i].xp, cached ? 0 : sd[i].xp_bs, sd[i].n);
        a.p[i].Ap1 = qp;
        a.p[i].ap1_bs = qbs;
        a.p[i].apl1 = (int64_t)sd[i].n * 256;
        a.p[i].ldap1 = 256;
      }
    }
    // (the bf16 / split modes' wide tiles read A from its planes: without them, the tile of
    // the EPI_ACC launch)
    const int t1 = (pm != PM_F32 && !ap) ? mlp1_acc_tile(pm) : mlp1_tile(pm);
    if ((rc = gemm_launch(EPI_STATS, PRO_HEADZ, t1, a, st, K_MLP1, pm)) != ONEPOSE_OK)
      return rc;
  }
  // 5. InstanceNorm statistics: finalized inside MLP conv 1 by each column block's last
  //    M-tile (st_cnt); a sharded 3D side is re-merged over the ranks' (n, mean, M2)
  if (sh) {
    StatsArgs sa;
    const int str = gemm_tile_rows(kTileMLP1);
    for (int i = 0; i < nside; ++i)
      sa.p[i] = {sd[i].stats, p.mean + (size_t)i * B * 512, p.rstd + (size_t)i * B * 512,
                 sd[i].n, ceil_div(sd[i].n, str), str};
    {
      OP_LAUNCH(K_STATS, st, stats_partial_kernel, dim3(B * 32), dim3(256), 0, st, sa.p[1], B,
                reinterpret_cast<double*>(sh->send));
      const int64_t nst = (int64_t)B * 512 * 3;
      if ((rc = shard_exchange(*sh, nst * 8, st)) != ONEPOSE_OK) return rc;
      OP_LAUNCH(K_STATS, st, stats_merge_kernel, dim3(ceil_div(B * 512, 256)), dim3(256), 0, st,
                reinterpret_cast<const double*>(sh->recv), sh->world, nst, B,
                p.mean + (size_t)B * 512, p.rstd + (size_t)B * 512);
    }
  }
  // 6. MLP conv 2 on ReLU(InstanceNorm(.)) + residual: desc + delta
  return groups(nside, [&](int a, int b) { return tl.mlp2[a] == tl.mlp2[b]; }, [&](int i0, int i1) -> int {
    GemmArgs a;
    a.nprob = i1 - i0;
    const bool yp = pm != PM_F32 && all_of(i0, i1, [&](int i) { return sd[i].xop != nullptr; });
    for (int i = i0; i < i1; ++i) {
      const Side& s = sd[i];
      GemmProb& g = a.p[i - i0];
      g = gemm_prob(s.y1, 512, w.w2, 512, w.b2, s.xo, 256, s.n, 256, 512, B);
      g.R = s.x;
      g.ldr = 256;
      g.r_bs = s.x_bs;
      g.pro_mean = p.mean + (size_t)i * B * 512;
      g.pro_rstd = p.rstd + (size_t)i * B * 512;
      g.pro_bs = 512;
      if (pm != PM_F32) set_w_planes(g, w.w2_p, kPlW2);
      if (yp) set_y_planes(g, s.xop, s.n, B);
    }
    return gemm_launch(EPI_RESID, PRO_NORM_RELU, tl.mlp2[i0], a, st, K_MLP2, pm);
  });
}

// The matcher forward on point-major leaves [*, n3*L, 256] (leaves_pm_bs elements per sample).
// obj_cache (onepose_match_cached): the 3D side entering layer 2, [n3][256] shared by the
// batch (onepose_object_prepare) -- GAT 0 and the 3D half of self-attention 1 are skipped.
// desc_dt (ONEPOSE_DT_*): the element type of desc2d and of an uncached desc3d.
int match_impl(const void* packed_weights, const void* desc2d, int64_t desc2d_bstride,
               const void* desc3d, int64_t desc3d_bstride, const float* leaves_pm,
               int64_t leaves_pm_bs, int batch, int n1, int n3, int num_leaf, float scale_factor,
               float match_threshold, int64_t* matches0, int64_t* matches1, float* mscores0,
               float* mscores1, float* conf, const Plan& p, hipStream_t st, int precision,
               const ShardCtx* sh = nullptr, const float* obj_cache = nullptr,
               int obj_flags = 0, int desc_dt = ONEPOSE_DT_F32,
               const CacheHdr* obj_hdr = nullptr, int first_stage = ONEPOSE_STAGE_INPUTS,
               int last_stage = ONEPOSE_STAGE_WINNERS) {
  // the stages [first_stage, last_stage] of the forward (onepose_match_cached_stages)
  auto in_range = [&](int stage) { return stage >= first_stage && stage <= last_stage; };
  const bool with_conf = conf != nullptr;
  const int n3g = sh ? sh->n3_total : n3;   // the 3D side's full length (softmax / attention)
  const int pm = attention_pm(precision);   // attention-layer GEMM operand mode
  const int pm_out = precision == ONEPOSE_PREC_FP32_SPLIT ? PM_SPLIT3 : PM_F32;   // final, score
  const float* wbase = static_cast<const float*>(packed_weights);
  const int B = batch;
  float* S = with_conf ? conf : p.s;
  const float* leaves = leaves_pm;
  const int64_t leaves_bstride = leaves_pm_bs;

  // bf16 modes: every producer of an attention GEMM's A operand also writes its activation
  // planes (the token states x2 / x3, phi(q)), which those GEMMs then move by DMA
  const int npl = planes_of(pm);
  auto pl = [&](uint16_t* q) { return npl ? q : nullptr; };
  // the dual softmax's statistics inside conf_kernel (whole frames, few score M-tiles, at most
  // kConfRowTiles score tiles per row): no softmax_reduce launch; the packed column winners are
  // zeroed by the first kernel instead.  Every conf workgroup re-derives its rows' statistics
  // from all of the row's partials, so above 64 score tiles per row (configs 3 and 5) those
  // re-reads (n3 / 256 times each) cost more than the separate softmax_reduce launch: config 5
  // conf 55.7 -> 36.4 + 7.6 us, config 3 1.91 -> 0.76 ms per step, the same bits
  // (profiles/r05/conf_rpl/, profiles/r05/smx/)
  const int score_mt = ceil_div(n1, pm_out == PM_F32 ? kScoreBM : 64);   // colpart per column
  const bool conf_stats = !sh && score_mt <= kConfColTiles && ceil_div(n3, 64) <= kConfRowTiles;
  // the dual softmax's winners and the mutual check (ONEPOSE_STAGE_WINNERS): the score GEMM's
  // partials and S in the workspace -> matches / scores
  auto winners = [&]() -> int {
    int rc;
    const int ch3 = ceil_div(n3, 64);
    const int64_t total = (int64_t)B * (n1 + n3);
    if (!conf_stats)
      OP_LAUNCH(K_SMX_REDUCE, st, softmax_reduce_kernel, dim3((unsigned)((total + 3) / 4)),
                dim3(256), 0, st, p.rowpart, ch3, p.colpart, score_mt, B, n1, n3, p.rowmax,
                p.rowsum, p.colmax, p.colsum, p.rowbest, p.colbest);
    const int64_t nr = (int64_t)B * n1;
    if (sh) {   // row softmax over every rank's columns
      OP_HIP(hipMemcpyAsync(sh->send, p.rowmax, nr * 4, hipMemcpyDeviceToDevice, st));
      OP_HIP(hipMemcpyAsync(sh->send + nr * 4, p.rowsum, nr * 4, hipMemcpyDeviceToDevice, st));
      if ((rc = shard_exchange(*sh, nr * 8, st)) != ONEPOSE_OK) return rc;
      OP_LAUNCH(K_SMX_REDUCE, st, rowstat_merge_kernel, dim3((unsigned)((nr + 255) / 256)),
                dim3(256), 0, st, reinterpret_cast<const float*>(sh->recv), sh->world, 2 * nr, nr,
                p.rowmax, p.rowsum);
    }
    const int coff = sh ? sh->offset : 0;
    const dim3 cgrid(ceil_div(n1, 32) * ceil_div(n3, 256), B);
#define CONF_LAUNCH(V, ST)                                                                   \
  OP_LAUNCH(K_CONF, st, (conf_kernel<V, ST>), cgrid, dim3(kConfWaves * 64), 0, st, S, n1, n3,  \
            p.rowmax,                                                                       \
            p.rowsum, p.colmax, p.colsum, p.rowwin, p.colbest, with_conf ? 1 : 0, coff,     \
            p.rowpart, ch3, p.colpart, score_mt)
    if (n3 % 4 == 0) {
      if (conf_stats) CONF_LAUNCH(true, true);
      else CONF_LAUNCH(true, false);
    } else {
      if (conf_stats) CONF_LAUNCH(false, true);
      else CONF_LAUNCH(false, false);
    }
#undef CONF_LAUNCH
    const unsigned long long* colbest = p.colbest;
    const unsigned long long* rowwin = p.rowwin;
    if (sh) {   // row winners over all columns; every rank's column winners at global columns
      OP_LAUNCH(K_MUTUAL, st, rowbest_reduce_kernel, dim3((unsigned)((nr + 255) / 256)), dim3(256),
                0, st, p.rowwin, ceil_div(n3, 256), nr,
                reinterpret_cast<unsigned long long*>(sh->send));
      rowwin = nullptr;
      if ((rc = shard_exchange(*sh, nr * 8, st)) != ONEPOSE_OK) return rc;
      OP_LAUNCH(K_MUTUAL, st, best_max_kernel, dim3((unsigned)((nr + 255) / 256)), dim3(256), 0, st,
                reinterpret_cast<const unsigned long long*>(sh->recv), sh->world, nr, nr,
                p.rowbest);
      const int64_t nc = (int64_t)B * sh->max_shard;
      OP_LAUNCH(K_MUTUAL, st, colbest_pack_kernel, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0,
                st, p.colbest, B, n3, sh->max_shard,
                reinterpret_cast<unsigned long long*>(sh->send));
      if ((rc = shard_exchange(*sh, nc * 8, st)) != ONEPOSE_OK) return rc;
      const int64_t nf = (int64_t)B * n3g;
      OP_LAUNCH(K_MUTUAL, st, colbest_assemble_kernel, dim3((unsigned)((nf + 255) / 256)),
                dim3(256), 0, st, reinterpret_cast<const unsigned long long*>(sh->recv), sh->world,
                nc, B, n3g, sh->max_shard, sh->colbest_full);
      colbest = sh->colbest_full;
    }
    const int64_t tot_g = (int64_t)B * (n1 + n3g);
    OP_LAUNCH(K_MUTUAL, st, mutual_kernel, dim3((unsigned)((tot_g + 255) / 256)), dim3(256), 0, st,
                       p.rowbest, rowwin, ceil_div(n3, 256), colbest, B, n1, n3g,
                       match_threshold, matches0, matches1,
                       mscores0, mscores1, p.err);
    return ONEPOSE_OK;
  };
  {
    TransArgs ta;
    ta.p[0] = {desc2d, desc2d_bstride, n1, ceil_div(n1, 64) * 4, p.x2[0], pl(p.x2p[0])};
    ta.p[1] = {desc3d, desc3d_bstride, n3, obj_cache ? 0 : ceil_div(n3, 64) * 4, p.x3[0],
               pl(p.x3p[0])};
    ta.p[0].f16 = desc_dt == ONEPOSE_DT_F16;
    ta.p[1].f16 = !obj_cache && desc_dt == ONEPOSE_DT_F16;
    ta.zero = p.cnt;
    ta.nzero = p.ncnt;
    ta.npl = npl;
    if (conf_stats) {
      ta.zero64 = p.colbest;
      ta.nzero64 = (int64_t)B * n3;
    }
    ta.err = p.err;
    if (obj_cache != nullptr && obj_hdr != nullptr) {
      ta.hdr = reinterpret_cast<const unsigned*>(
          obj_cache + obj_layout(n3, num_leaf, obj_flags, npl != 0).hdr);
      ta.expect = *obj_hdr;
    }
    if (in_range(ONEPOSE_STAGE_INPUTS))
      OP_LAUNCH(K_TRANSPOSE, st, transpose_in_kernel, dim3((ta.p[0].tiles + ta.p[1].tiles) * B),
                dim3(256), 0, st, ta, B);
  }
  if (last_stage < ONEPOSE_STAGE_LAYER0 || first_stage > ONEPOSE_STAGE_SCORE)
    return in_range(ONEPOSE_STAGE_WINNERS) ? winners() : ONEPOSE_OK;

  // Current states: side x is read from x?r (batch stride x?bs) and written to p.x?[c? ^ 1];
  // their activation planes (bf16 modes) from x?pr (null: the object cache's state, which only
  // cached halves read)
  int c2 = 0, c3 = 0, ap = 0, gat = 0;
  const float* x2r = p.x2[0];
  const float* x3r = obj_cache ? obj_cache : p.x3[0];
  int64_t x3bs = obj_cache ? 0 : (int64_t)n3 * 256;
  const uint16_t* x2pr = pl(p.x2p[0]);
  const uint16_t* x3pr = obj_cache ? nullptr : pl(p.x3p[0]);
  for (int layer = 0; layer < kLayers; ++layer) {
    if (last_stage < ONEPOSE_STAGE_LAYER0 + layer) return ONEPOSE_OK;
    // a layer outside the range ran in an earlier call on the same workspace (or runs in a
    // later one): the loop only tracks which buffers hold the states
    const bool run_layers = in_range(ONEPOSE_STAGE_LAYER0 + layer);
    const int kind = layer % 3;  // 0 GATs, 1 self, 2 cross
    const bool cached3 = obj_cache && layer < 2;   // the 3D side comes from the cache
    if (kind == 0) {
      if (!cached3) {
        const dim3 ggrid(ceil_div(B * n3, 4));
        // the object's stored leaf logits (one object for the whole batch: leaves stride 0)
        const float* slog = obj_cache && leaves_bstride == 0 && gat >= 1
                                ? obj_cache + (int64_t)n3 * 256 +
                                      (int64_t)(gat - 1) * n3 * kLogitStride
                                : nullptr;
        const ObjLayout OL = obj_layout(n3, num_leaf, obj_flags, npl != 0);
        uint16_t* yp = pl(p.x3p[c3 ^ 1]);
        if (!run_layers) {
        } else if (slog != nullptr && OL.tables) {
          OP_LAUNCH(K_GAT, st, gat_tab_kernel, ggrid, dim3(256), 0, st, x3r, gat_weights(wbase, gat),
                    obj_cache + OL.slogs + (int64_t)(gat - 1) * n3 * kLogitStride,
                    obj_cache + OL.tab + (int64_t)(gat - 1) * n3 * 2 * num_leaf * 256,
                    p.x3[c3 ^ 1], n3, num_leaf, B, yp, npl);
        } else if (num_leaf <= 8)
          OP_LAUNCH(K_GAT, st, gat_kernel<8>, ggrid, dim3(256), 0, st, x3r, leaves,
                    leaves_bstride, gat_weights(wbase, gat), slog, p.x3[c3 ^ 1], n3, num_leaf, B,
                    yp, npl);
        else
          OP_LAUNCH(K_GAT, st, gat_kernel<16>, ggrid, dim3(256), 0, st, x3r, leaves,
                    leaves_bstride, gat_weights(wbase, gat), slog, p.x3[c3 ^ 1], n3, num_leaf, B,
                    yp, npl);
        x3r = p.x3[c3 ^ 1];
        x3pr = yp;
        c3 ^= 1;
      }
      ++gat;
      continue;
    }
    const ApW w = ap_weights(wbase, ap++);
    // self: each side attends to itself; cross: 2D <-> 3D
    Side sd[2];
    sd[0] = {x2r, (int64_t)n1 * 256, p.x2[c2 ^ 1], p.phiq2, p.kvpart2, p.kspart2, p.y12,
             p.stats2, n1, (float)n1, kind == 1 ? 0 : 1, n1};
    sd[1] = {x3r, x3bs, p.x3[c3 ^ 1], p.phiq3, p.kvpart3, p.kspart3, p.y13, p.stats3, n3,
             (float)n3g, kind == 1 ? 1 : 0, sh ? sh->max_shard : n3};
    const int64_t pbs2 = (int64_t)kPlanesMax * n1 * 256, pbs3 = (int64_t)kPlanesMax * n3 * 256;
    sd[0].xp = x2pr;
    sd[0].xp_bs = pbs2;
    sd[0].xop = pl(p.x2p[c2 ^ 1]);
    sd[0].phiqp = pl(p.phiq2p);
    sd[1].xp = x3pr;
    sd[1].xp_bs = pbs3;
    sd[1].xop = pl(p.x3p[c3 ^ 1]);
    sd[1].phiqp = pl(p.phiq3p);
    const int qkv_n3 = sh ? sh->max_shard : n3;
    unsigned* lcnt = p.cnt + (size_t)(ap - 1) * 2 * B * p.cps;
    // layers 1-2 of a whole frame: per-side choices (the 3D side's are the object prefix's,
    // so cached and uncached forwards agree bit for bit at any batch); later layers and
    // sharded frames: one set for the launch
    const LayerTiles tl = !sh && ap <= 2 ? side_tiles(n1, n3, B, pm, kind == 2)
                                         : layer_tiles(qkv_n3, sd, 2, B, pm, sh);
    int rc = ONEPOSE_OK;
    if (!run_layers) {
    } else if (cached3) {   // self-attention 1, 2D half (the 3D half is in the object cache)
      rc = attention_layer(w, sd, 1, B, p, lcnt, st, pm, sh, tl);
    } else if (obj_cache && layer == 2 && !sh) {
      // cross-attention 1: the 3D side's frame-independent half from the object cache
      const ObjLayout L = obj_layout(n3, num_leaf, obj_flags, npl != 0);
      const SideCache xc = {obj_cache + L.phiq, obj_cache + L.acc, obj_cache + L.ksum,
                            obj_cache + L.mf,
                            npl ? reinterpret_cast<const uint16_t*>(obj_cache + L.phiqp) : nullptr};
      rc = attention_layer(w, sd, 2, B, p, lcnt, st, pm, nullptr, tl, &xc);
    } else {
      rc = attention_layer(w, sd, 2, B, p, lcnt, st, pm, sh, tl);
    }
    if (rc != ONEPOSE_OK) return rc;
    x2r = p.x2[c2 ^ 1];
    x2pr = sd[0].xop;
    c2 ^= 1;
    if (!cached3) {
      x3r = p.x3[c3 ^ 1];
      x3pr = sd[1].xop;
      x3bs = (int64_t)n3 * 256;
      c3 ^= 1;
    }
  }

  if (last_stage < ONEPOSE_STAGE_FINAL) return ONEPOSE_OK;
  int rc;
  if (in_range(ONEPOSE_STAGE_FINAL)) {  // final_proj on both sides, then L2 normalise
    const float* fw = final_weights(wbase);
    GemmArgs a;
    a.nprob = 2;
    a.p[0] = gemm_prob(x2r, 256, fw, 256, fw + 65536, p.f2, 256, n1, 256, 256, B);
    a.p[1] = gemm_prob(x3r, 256, fw, 256, fw + 65536, p.f3, 256, n3, 256, 256, B);
    if (pm_out == PM_F32) {
      // fp32: whole-row tiles normalise in the epilogue (l2norm_kernel's arithmetic, the same
      // bits), one launch and one pass over f2 / f3 fewer; half the workgroups of 64 x 64,
      // which leaves CUs to the other match stream
      if ((rc = gemm_launch(EPI_BIAS_L2, PRO_PLAIN, kTileFinalL2, a, st, K_FINAL, pm_out)) !=
          ONEPOSE_OK)
        return rc;
    } else {
      if ((rc = gemm_launch(EPI_BIAS, PRO_PLAIN, kTileFinal, a, st, K_FINAL, pm_out)) != ONEPOSE_OK)
        return rc;
      const int rows = B * (n1 + n3);
      OP_LAUNCH(K_L2NORM, st, l2norm_kernel, dim3(ceil_div(rows, 4)), dim3(256), 0, st, p.f2,
                B * n1, p.f3, B * n3);
    }
  }
  if (!in_range(ONEPOSE_STAGE_SCORE)) return ONEPOSE_OK;   // (a range: no winners either)
  // score tile: 128 x 64 on 8 waves in fp32 (K = 256 is short; fewer operand loads per FLOP
  // than 64 x 64), 64 x 64 in the split mode (its LDS images are three bf16 planes)
  const int score_tile = pm_out == PM_F32 ? kTileScore : TILE_64x64;
  {  // S = D2^T D3 / scale_factor with softmax partials
    GemmArgs a;
    a.nprob = 1;
    a.p[0] = gemm_prob(p.f2, 256, p.f3, 256, nullptr, S, n3, n1, n3, 256, B);
    a.p[0].w_bs = (int64_t)n3 * 256;
    a.p[0].scale = scale_factor;
    a.p[0].rowstat = p.rowpart;
    a.p[0].colstat = p.colpart;
    if ((rc = gemm_launch(EPI_SCORE, PRO_PLAIN, score_tile, a, st, K_SCORE, pm_out)) != ONEPOSE_OK)
      return rc;
  }
  return in_range(ONEPOSE_STAGE_WINNERS) ? winners() : ONEPOSE_OK;
}

// The frame-independent prefix of the 3D side (onepose_object_prepare): transpose, GAT 0
// (GATs.py:62-123 on the object's own leaves) and the 3D half of self-attention 1 (the 3D
// side attends only to itself there) -> cache [n3][256], the state entering layer 2.
// The same kernels and tiles as the grouped forward, so the cached state is bit-identical
// to what onepose_match computes in place.
int object_prepare_impl(const void* packed_weights, const void* desc3d, int desc_dt,
                        const float* leaves_pm, int n3, int num_leaf, int precision, int flags,
                        float* cache, const Plan& p, hipStream_t st) {
  const float* wbase = static_cast<const float*>(packed_weights);
  const int pm = attention_pm(precision);
  const int npl = planes_of(pm);   // activation planes (bf16 modes), as in match_impl
  auto pl = [&](uint16_t* q) { return npl ? q : nullptr; };
  {
    TransArgs ta;
    ta.p[0] = {desc3d, 0, n3, ceil_div(n3, 64) * 4, p.x3[0]};
    ta.p[1] = {desc3d, 0, n3, 0, p.x3[0]};
    ta.p[0].f16 = desc_dt == ONEPOSE_DT_F16;
    ta.zero = p.cnt;
    ta.nzero = p.ncnt;
    OP_LAUNCH(K_TRANSPOSE, st, transpose_in_kernel, dim3(ta.p[0].tiles), dim3(256), 0, st, ta, 1);
  }
  const dim3 ggrid(ceil_div(n3, 4));
  const float* nolog = nullptr;
  float* slog = cache + (int64_t)n3 * 256;   // leaf logits of GAT layers 1-3
  if (num_leaf <= 8) {
    OP_LAUNCH(K_GAT, st, gat_kernel<8>, ggrid, dim3(256), 0, st, p.x3[0], leaves_pm, (int64_t)0,
              gat_weights(wbase, 0), nolog, p.x3[1], n3, num_leaf, 1, pl(p.x3p[1]), npl);
    OP_LAUNCH(K_GAT, st, gat_logits_kernel<8>, ggrid, dim3(256), 0, st, leaves_pm,
              gat_weights(wbase, 1), slog, n3, num_leaf);
    const ObjLayout OL = obj_layout(n3, num_leaf, flags, npl != 0);
    if (OL.tables)
      OP_LAUNCH(K_GAT, st, gat_table_kernel, ggrid, dim3(256), 0, st, leaves_pm,
                gat_weights(wbase, 1), cache + OL.slogs, cache + OL.tab, n3, num_leaf);
  } else {
    OP_LAUNCH(K_GAT, st, gat_kernel<16>, ggrid, dim3(256), 0, st, p.x3[0], leaves_pm, (int64_t)0,
              gat_weights(wbase, 0), nolog, p.x3[1], n3, num_leaf, 1, pl(p.x3p[1]), npl);
    OP_LAUNCH(K_GAT, st, gat_logits_kernel<16>, ggrid, dim3(256), 0, st, leaves_pm,
              gat_weights(wbase, 1), slog, n3, num_leaf);
  }
  Side s3 = {p.x3[1], (int64_t)n3 * 256, cache, p.phiq3, p.kvpart3, p.kspart3, p.y13,
             p.stats3, n3, (float)n3, 0, n3};
  s3.xp = pl(p.x3p[1]);
  s3.xp_bs = (int64_t)kPlanesMax * n3 * 256;
  s3.xop = pl(p.x3p[0]);   // the cached state's planes: cross-attention 1's QKV below reads them
  s3.phiqp = pl(p.phiq3p);
  int rc = attention_layer(ap_weights(wbase, 0), &s3, 1, 1, p, p.cnt, st, pm, nullptr,
                           layer_tiles(n3, &s3, 1, 1, pm, false));
  if (rc != ONEPOSE_OK) return rc;

  // Cross-attention 1 (layer 2), the 3D side's frame-independent half, with the choices a
  // cached forward's layer 2 makes (batch <= kFusedFoldMaxBatch: QKV tile from n3 alone, one
  // kv_fold launch), so that its bits are the ones the uncached forward computes in place.
  const ObjLayout L = obj_layout(n3, num_leaf, flags, npl != 0);
  const ApW w = ap_weights(wbase, 1);
  const Side x3 = {cache, 0, nullptr, cache + L.phiq, p.kvpart3, p.kspart3, nullptr, nullptr, n3,
                   (float)n3, 0, n3};
  const LayerTiles tl = layer_tiles(n3, &x3, 1, 1, pm, false);   // = side_tiles' 3D choices
  {  // phi(q) into the cache; KV / sum phi(k) chunk partials
    GemmArgs a;
    a.nprob = 1;
    a.p[0] = gemm_prob(cache, 256, w.wqkv, 256, w.bqkv, cache + L.phiq, 256, n3, 768, 256, 1);
    a.p[0].vdiv = (float)n3;
    a.p[0].kvpart = p.kvpart3;
    a.p[0].kspart = p.kspart3;
    if (pm != PM_F32) {
      set_w_planes(a.p[0], w.wqkv_p, kPlWqkv);
      set_a_planes(a.p[0], p.x3p[0], 0, n3);
      // phi(q)'s planes into the cache: a cached frame's MLP conv 1 reads them as its A1
      set_y_planes(a.p[0], reinterpret_cast<uint16_t*>(cache + L.phiqp), n3, 1);
    }
    if ((rc = gemm_launch(EPI_QKV, PRO_PLAIN, tl.qkv[0], a, st, K_QKV_GEMM, pm)) != ONEPOSE_OK)
      return rc;
  }
  {  // sum phi(k) into the cache, and the 2D side's Mf = C KV_3D
    KvFoldArgs ka;
    ka.ct = w.ct;
    ka.planes = pm != PM_F32 ? 1 : 0;
    ka.p[0] = {p.kvpart3, p.kspart3, ceil_div(n3, gemm_tile_stat_rows(tl.qkv[0]))};
    ka.mf[0] = cache + L.mf;
    ka.mf[1] = nullptr;
    prof_pre(K_KV_REDUCE, st);
    launch_kv_fold(ka, 1, 1, p.kv, cache + L.ksum, st);
    prof_post(K_KV_REDUCE, st);
    OP_LAUNCHED();
  }
  {  // MLP conv 1's x range: W1a x3 as raw accumulators of the TILE_64x64 MFMA sequence
    GemmArgs a;
    a.nprob = 1;
    a.p[0] = gemm_prob(cache, 256, w.w1a, 256, nullptr, cache + L.acc, 512, n3, 512, 256, 1);
    if (pm != PM_F32) set_w_planes(a.p[0], w.w1a_p, kPlW1a);
    if ((rc = gemm_launch(EPI_ACC, PRO_PLAIN, mlp1_acc_tile(pm), a, st, K_MLP1, pm)) != ONEPOSE_OK)
      return rc;
  }
  return ONEPOSE_OK;
}

int check_match_args(const void* packed_weights, const void* desc2d, const void* desc3d,
                     const void* leaves, int batch, int n1, int n3, int num_leaf,
                     float scale_factor, const int64_t* matches0, const int64_t* matches1,
                     const float* mscores0, const float* mscores1, const void* workspace) {
  OP_REQUIRE(packed_weights && desc2d && desc3d && leaves, "match: null input");
  OP_REQUIRE(matches0 && matches1 && mscores0 && mscores1, "match: null output");
  OP_REQUIRE(batch >= 1 && n1 >= 1 && n3 >= 1, "match: batch=%d n1=%d n3=%d", batch, n1, n3);
  OP_REQUIRE(num_leaf >= 1 && num_leaf <= 16, "match: num_leaf=%d not in [1,16]", num_leaf);
  OP_REQUIRE(scale_factor != 0.f, "match: scale_factor 0");
  OP_REQUIRE(workspace != nullptr, "match: null workspace");
  return ONEPOSE_OK;
}

}  // namespace
}  // namespace onepose

extern "C" {

size_t onepose_leaves_prepared_bytes(int batch, int n3, int num_leaf) {
  if (batch <= 0 || n3 <= 0 || num_leaf <= 0) return 0;
  return (size_t)batch * n3 * num_leaf * 256 * sizeof(float);
}

int onepose_prepare_leaves(const float* leaves, int64_t leaves_bstride, int batch, int n3,
                           int num_leaf, float* out, void* stream_) {
  return onepose_prepare_leaves_dt(leaves, ONEPOSE_DT_F32, leaves_bstride, batch, n3, num_leaf,
                                   out, stream_);
}

int onepose_prepare_leaves_dt(const void* leaves, int dtype, int64_t leaves_bstride, int batch,
                              int n3, int num_leaf, float* out, void* stream_) {
  clear_error();
  OP_REQUIRE(leaves && out, "prepare_leaves: null pointer");
  OP_REQUIRE(dtype == ONEPOSE_DT_F32 || dtype == ONEPOSE_DT_F16, "prepare_leaves: dtype %d", dtype);
  OP_REQUIRE(batch >= 1 && n3 >= 1 && num_leaf >= 1 && num_leaf <= 16,
             "prepare_leaves: batch=%d n3=%d num_leaf=%d", batch, n3, num_leaf);
  hipStream_t st = static_cast<hipStream_t>(stream_);
  const int ncol = n3 * num_leaf;
  TransArgs ta;
  ta.p[0] = {leaves, leaves_bstride, ncol, ceil_div(ncol, 64) * 4, out};
  ta.p[1] = {leaves, 0, 1, 0, out};
  ta.p[0].f16 = dtype == ONEPOSE_DT_F16;
  ta.zero = nullptr;
  ta.nzero = 0;
  OP_LAUNCH(K_TRANSPOSE, st, transpose_in_kernel, dim3(ta.p[0].tiles * batch), dim3(256), 0, st,
            ta, batch);
  return ONEPOSE_OK;
}

int onepose_match_ex(const void* packed_weights, const float* desc2d, int64_t desc2d_bstride,
                     const float* desc3d, int64_t desc3d_bstride, const float* leaves,
                     int64_t leaves_bstride, int batch, int n1, int n3, int num_leaf,
                     float scale_factor, float match_threshold, int precision,
                     int64_t* matches0, int64_t* matches1, float* mscores0, float* mscores1,
                     float* conf, void* workspace, size_t workspace_bytes, void* stream_) {
  return onepose_match_dt(packed_weights, desc2d, desc2d_bstride, desc3d, desc3d_bstride, leaves,
                          leaves_bstride, ONEPOSE_DT_F32, batch, n1, n3, num_leaf, scale_factor,
                          match_threshold, precision, matches0, matches1, mscores0, mscores1,
                          conf, workspace, workspace_bytes, stream_);
}

int onepose_match_dt(const void* packed_weights, const void* desc2d, int64_t desc2d_bstride,
                     const void* desc3d, int64_t desc3d_bstride, const void* leaves,
                     int64_t leaves_bstride, int desc_dtype, int batch, int n1, int n3,
                     int num_leaf, float scale_factor, float match_threshold, int precision,
                     int64_t* matches0, int64_t* matches1, float* mscores0, float* mscores1,
                     float* conf, void* workspace, size_t workspace_bytes, void* stream_) {
  clear_error();
  OP_REQUIRE(valid_precision(precision),
             "match: precision %d", precision);
  OP_REQUIRE(desc_dtype == ONEPOSE_DT_F32 || desc_dtype == ONEPOSE_DT_F16, "match: dtype %d",
             desc_dtype);
  int rc = check_match_args(packed_weights, desc2d, desc3d, leaves, batch, n1, n3, num_leaf,
                            scale_factor, matches0, matches1, mscores0, mscores1, workspace);
  if (rc != ONEPOSE_OK) return rc;
  const bool planes = precision != ONEPOSE_PREC_FP32;
  const Plan need = make_plan(nullptr, batch, n1, n3, num_leaf, conf != nullptr, planes);
  if (workspace_bytes < need.bytes) {
    set_error("match: workspace %zu < %zu bytes", workspace_bytes, need.bytes);
    return ONEPOSE_ERR_WORKSPACE;
  }
  hipStream_t st = static_cast<hipStream_t>(stream_);
  const Plan p = make_plan(workspace, batch, n1, n3, num_leaf, conf != nullptr, planes);
  // reference layout [*, 256, n3*L] -> point-major copy in the workspace
  const int lb = leaves_bstride == 0 ? 1 : batch;
  if ((rc = onepose_prepare_leaves_dt(leaves, desc_dtype, leaves_bstride, lb, n3, num_leaf,
                                      p.leaves_pm, stream_)) != ONEPOSE_OK)
    return rc;
  const int64_t pm_bs = leaves_bstride == 0 ? 0 : (int64_t)n3 * num_leaf * 256;
  return match_impl(packed_weights, desc2d, desc2d_bstride, desc3d, desc3d_bstride, p.leaves_pm,
                    pm_bs, batch, n1, n3, num_leaf, scale_factor, match_threshold, matches0,
                    matches1, mscores0, mscores1, conf, p, st, precision, nullptr, nullptr, 0,
                    desc_dtype);
}

int onepose_match(const void* packed_weights, const float* desc2d, int64_t desc2d_bstride,
                  const float* desc3d, int64_t desc3d_bstride, const float* leaves,
                  int64_t leaves_bstride, int batch, int n1, int n3, int num_leaf,
                  float scale_factor, float match_threshold, int64_t* matches0,
                  int64_t* matches1, float* mscores0, float* mscores1, float* conf,
                  void* workspace, size_t workspace_bytes, void* stream_) {
  return onepose_match_ex(packed_weights, desc2d, desc2d_bstride, desc3d, desc3d_bstride, leaves,
                          leaves_bstride, batch, n1, n3, num_leaf, scale_factor, match_threshold,
                          ONEPOSE_PREC_FP32, matches0, matches1, mscores0, mscores1, conf,
                          workspace, workspace_bytes, stream_);
}

int onepose_match_prepared_ex(const void* packed_weights, const float* desc2d,
                              int64_t desc2d_bstride, const float* desc3d, int64_t desc3d_bstride,
                              const float* leaves_prepared, int64_t prepared_bstride, int batch,
                              int n1, int n3, int num_leaf, float scale_factor,
                              float match_threshold, int precision, int64_t* matches0,
                              int64_t* matches1, float* mscores0, float* mscores1, float* conf,
                              void* workspace, size_t workspace_bytes, void* stream_) {
  clear_error();
  OP_REQUIRE(valid_precision(precision),
             "match: precision %d", precision);
  int rc = check_match_args(packed_weights, desc2d, desc3d, leaves_prepared, batch, n1, n3,
                            num_leaf, scale_factor, matches0, matches1, mscores0, mscores1,
                            workspace);
  if (rc != ONEPOSE_OK) return rc;
  const bool planes = precision != ONEPOSE_PREC_FP32;
  const Plan need = make_plan(nullptr, batch, n1, n3, num_leaf, conf != nullptr, planes);
  if (workspace_bytes < need.bytes) {
    set_error("match: workspace %zu < %zu bytes", workspace_bytes, need.bytes);
    return ONEPOSE_ERR_WORKSPACE;
  }
  const Plan p = make_plan(workspace, batch, n1, n3, num_leaf, conf != nullptr, planes);
  return match_impl(packed_weights, desc2d, desc2d_bstride, desc3d, desc3d_bstride,
                    leaves_prepared, prepared_bstride, batch, n1, n3, num_leaf, scale_factor,
                    match_threshold, matches0, matches1, mscores0, mscores1, conf, p,
                    static_cast<hipStream_t>(stream_), precision);
}

int onepose_match_prepared(const void* packed_weights, const float* desc2d,
                           int64_t desc2d_bstride, const float* desc3d, int64_t desc3d_bstride,
                           const float* leaves_prepared, int64_t prepared_bstride, int batch,
                           int n1, int n3, int num_leaf, float scale_factor,
                           float match_threshold, int64_t* matches0, int64_t* matches1,
                           float* mscores0, float* mscores1, float* conf, void* workspace,
                           size_t workspace_bytes, void* stream_) {
  return onepose_match_prepared_ex(packed_weights, desc2d, desc2d_bstride, desc3d, desc3d_bstride,
                                   leaves_prepared, prepared_bstride, batch, n1, n3, num_leaf,
                                   scale_factor, match_threshold, ONEPOSE_PREC_FP32, matches0,
                                   matches1, mscores0, mscores1, conf, workspace, workspace_bytes,
                                   stream_);
}

size_t onepose_object_cache_bytes(int n3, int num_leaf, int flags) {
  if (n3 <= 0 || num_leaf < 1 || num_leaf > 16) return 0;
  if ((flags & ~ONEPOSE_OBJ_GAT_TABLES) != 0) return 0;   // the flags prepare / match refuse
  return (size_t)obj_layout(n3, num_leaf, flags, true).total * sizeof(float);   // any precision
}

size_t onepose_object_cache_bytes_ex(int n3, int num_leaf, int flags, int precision) {
  if (n3 <= 0 || num_leaf < 1 || num_leaf > 16 || !valid_precision(precision)) return 0;
  if ((flags & ~ONEPOSE_OBJ_GAT_TABLES) != 0) return 0;
  return (size_t)obj_layout(n3, num_leaf, flags, precision != ONEPOSE_PREC_FP32).total *
         sizeof(float);
}

size_t onepose_object_prepare_workspace_bytes(int n3, int num_leaf) {
  clear_error();
  if (n3 <= 0 || num_leaf < 1 || num_leaf > 16) return 0;
  return make_plan(nullptr, 1, 1, n3, num_leaf, false).bytes;
}

}  // extern "C"

namespace onepose {
namespace {
// What onepose_object_prepare built into each cache, keyed by the cache's device address. The
// cache's layout depends on (n3, num_leaf, flags) and its Mf region's format on the precision
// (fp32, or bf16 planes), and the device copy cannot be read back without a synchronisation,
// which a graph-captured launch must not do. So the host records them at prepare time and
// onepose_match_cached refuses a cache whose record is missing or differs from its arguments.
struct CacheRecord {
  int n3, num_leaf, precision, flags;
  unsigned long long gen;   // also in the cache's device header (CacheHdr)
};
std::mutex g_cache_mu;
std::unordered_map<const void*, CacheRecord> g_caches;
unsigned long long g_cache_gen = 0;
}  // namespace
}  // namespace onepose

extern "C" {

int onepose_object_prepare(const void* packed_weights, const float* desc3d,
                           const float* leaves_prepared, int n3, int num_leaf, int precision,
                           int flags, float* cache, void* workspace, size_t workspace_bytes,
                           void* stream_) {
  return onepose_object_prepare_dt(packed_weights, desc3d, ONEPOSE_DT_F32, leaves_prepared, n3,
                                   num_leaf, precision, flags, cache, workspace, workspace_bytes,
                                   stream_);
}

int onepose_object_prepare_dt(const void* packed_weights, const void* desc3d, int desc_dtype,
                              const float* leaves_prepared, int n3, int num_leaf, int precision,
                              int flags, float* cache, void* workspace, size_t workspace_bytes,
                              void* stream_) {
  clear_error();
  OP_REQUIRE(desc_dtype == ONEPOSE_DT_F32 || desc_dtype == ONEPOSE_DT_F16,
             "object_prepare: dtype %d", desc_dtype);
  OP_REQUIRE(packed_weights && desc3d && leaves_prepared && cache, "object_prepare: null pointer");
  OP_REQUIRE(valid_precision(precision),
             "object_prepare: precision %d", precision);
  OP_REQUIRE(n3 >= 1 && num_leaf >= 1 && num_leaf <= 16, "object_prepare: n3=%d num_leaf=%d", n3,
             num_leaf);
  OP_REQUIRE((flags & ~ONEPOSE_OBJ_GAT_TABLES) == 0, "object_prepare: flags %d", flags);
  OP_REQUIRE(workspace != nullptr, "object_prepare: null workspace");
  const size_t need = onepose_object_prepare_workspace_bytes(n3, num_leaf);
  if (workspace_bytes < need) {
    set_error("object_prepare: workspace %zu < %zu bytes", workspace_bytes, need);
    return ONEPOSE_ERR_WORKSPACE;
  }
  const Plan p = make_plan(workspace, 1, 1, n3, num_leaf, false);
  {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    g_caches.erase(cache);   // whatever it held before is gone from here on
  }
  const int rc = object_prepare_impl(packed_weights, desc3d, desc_dtype, leaves_prepared, n3,
                                     num_leaf, precision, flags, cache, p,
                                     static_cast<hipStream_t>(stream_));
  if (rc != ONEPOSE_OK) return rc;
  unsigned long long gen;
  {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    gen = ++g_cache_gen;
  }
  const CacheHdr h = cache_hdr(n3, num_leaf, precision, flags, gen);
  hipStream_t st = static_cast<hipStream_t>(stream_);
  unsigned* hdr = reinterpret_cast<unsigned*>(
      cache + obj_layout(n3, num_leaf, flags, precision != ONEPOSE_PREC_FP32).hdr);
  OP_LAUNCH(K_TRANSPOSE, st, cache_hdr_kernel, dim3(1), dim3(64), 0, st, hdr, h);
  {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    g_caches[cache] = {n3, num_leaf, precision, flags, gen};
  }
  return rc;
}

void onepose_object_release(const float* cache) {
  std::lock_guard<std::mutex> lk(g_cache_mu);
  g_caches.erase(cache);
}

int onepose_match_cached(const void* packed_weights, const float* desc2d, int64_t desc2d_bstride,
                         const float* object_cache, const float* leaves_prepared,
                         int64_t prepared_bstride, int batch, int n1, int n3, int num_leaf,
                         float scale_factor, float match_threshold, int precision,
                         int object_flags, int64_t* matches0, int64_t* matches1, float* mscores0,
                         float* mscores1, float* conf, void* workspace, size_t workspace_bytes,
                         void* stream_) {
  return onepose_match_cached_dt(packed_weights, desc2d, ONEPOSE_DT_F32, desc2d_bstride,
                                 object_cache, leaves_prepared, prepared_bstride, batch, n1, n3,
                                 num_leaf, scale_factor, match_threshold, precision, object_flags,
                                 matches0, matches1, mscores0, mscores1, conf, workspace,
                                 workspace_bytes, stream_);
}

int onepose_match_cached_dt(const void* packed_weights, const void* desc2d, int desc_dtype,
                            int64_t desc2d_bstride, const float* object_cache,
                            const float* leaves_prepared, int64_t prepared_bstride, int batch,
                            int n1, int n3, int num_leaf, float scale_factor,
                            float match_threshold, int precision, int object_flags,
                            int64_t* matches0, int64_t* matches1, float* mscores0,
                            float* mscores1, float* conf, void* workspace, size_t workspace_bytes,
                            void* stream_) {
  return onepose_match_cached_stages(packed_weights, desc2d, desc_dtype, desc2d_bstride,
                                    object_cache, leaves_prepared, prepared_bstride, batch, n1,
                                    n3, num_leaf, scale_factor, match_threshold, precision,
                                    object_flags, matches0, matches1, mscores0, mscores1, conf,
                                    workspace, workspace_bytes, ONEPOSE_STAGE_INPUTS,
                                    ONEPOSE_STAGE_WINNERS, stream_);
}

int onepose_match_cached_stages(const void* packed_weights, const void* desc2d, int desc_dtype,
                               int64_t desc2d_bstride, const float* object_cache,
                               const float* leaves_prepared, int64_t prepared_bstride, int batch,
                               int n1, int n3, int num_leaf, float scale_factor,
                               float match_threshold, int precision, int object_flags,
                               int64_t* matches0, int64_t* matches1, float* mscores0,
                               float* mscores1, float* conf, void* workspace,
                               size_t workspace_bytes, int first_stage, int last_stage,
                               void* stream_) {
  clear_error();
  OP_REQUIRE(first_stage >= ONEPOSE_STAGE_INPUTS && first_stage <= last_stage &&
                 last_stage <= ONEPOSE_STAGE_WINNERS,
             "match_cached: stages [%d, %d]", first_stage, last_stage);
  OP_REQUIRE(desc_dtype == ONEPOSE_DT_F32 || desc_dtype == ONEPOSE_DT_F16,
             "match_cached: dtype %d", desc_dtype);
  OP_REQUIRE(valid_precision(precision),
             "match_cached: precision %d", precision);
  OP_REQUIRE((object_flags & ~ONEPOSE_OBJ_GAT_TABLES) == 0, "match_cached: flags %d",
             object_flags);
  int rc = check_match_args(packed_weights, desc2d, object_cache, leaves_prepared, batch, n1, n3,
                            num_leaf, scale_factor, matches0, matches1, mscores0, mscores1,
                            workspace);
  if (rc != ONEPOSE_OK) return rc;
  CacheHdr hdr;
  {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    const auto it = g_caches.find(object_cache);
    OP_REQUIRE(it != g_caches.end(),
               "match_cached: object_cache was not built by onepose_object_prepare (or was "
               "released)");
    const CacheRecord& c = it->second;
    OP_REQUIRE(c.n3 == n3 && c.num_leaf == num_leaf && c.precision == precision &&
                   c.flags == object_flags,
               "match_cached: cache prepared for n3=%d num_leaf=%d precision=%d flags=%d, "
               "called with n3=%d num_leaf=%d precision=%d flags=%d",
               c.n3, c.num_leaf, c.precision, c.flags, n3, num_leaf, precision, object_flags);
    hdr = cache_hdr(c.n3, c.num_leaf, c.precision, c.flags, c.gen);
  }
  const bool planes = precision != ONEPOSE_PREC_FP32;
  const Plan need = make_plan(nullptr, batch, n1, n3, num_leaf, conf != nullptr, planes);
  if (workspace_bytes < need.bytes) {
    set_error("match_cached: workspace %zu < %zu bytes", workspace_bytes, need.bytes);
    return ONEPOSE_ERR_WORKSPACE;
  }
  const Plan p = make_plan(workspace, batch, n1, n3, num_leaf, conf != nullptr, planes);
  return match_impl(packed_weights, desc2d, desc2d_bstride, object_cache, 0, leaves_prepared,
                    prepared_bstride, batch, n1, n3, num_leaf, scale_factor, match_threshold,
                    matches0, matches1, mscores0, mscores1, conf, p,
                    static_cast<hipStream_t>(stream_), precision, nullptr, object_cache,
                    object_flags, desc_dtype, &hdr, first_stage, last_stage);
}

int onepose_device_errors(int clear, unsigned* bits) {
  clear_error();
  OP_REQUIRE(bits != nullptr, "device_errors: null pointer");
  unsigned v = 0u;
  OP_HIP(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_device_errors), sizeof(v)));
  if (clear && v != 0u) {
    const unsigned z = 0u;
    OP_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_device_errors), &z, sizeof(z)));
  }
  *bits = v;
  return ONEPOSE_OK;
}

void onepose_shard_range(int n3_total, int world, int rank, int* start, int* count) {
  if (!start || !count || world <= 0 || rank < 0 || rank >= world || n3_total < 0) {
    if (start) *start = 0;
    if (count) *count = 0;
    return;
  }
  shard_range(n3_total, world, rank, start, count);
}

size_t onepose_match_sharded_xchg_bytes(int batch, int n1, int n3_total, int world) {
  if (batch <= 0 || n1 <= 0 || n3_total <= 0 || world <= 0) return 0;
  return shard_xchg_bytes(batch, n1, n3_total, world);
}

size_t onepose_match_sharded_workspace_bytes(int batch, int n1, int n3_total, int world, int rank,
                                             int num_leaf, int with_conf) {
  if (batch <= 0 || n1 <= 0 || n3_total <= 0 || world <= 0 || rank < 0 || rank >= world) return 0;
  int s0, n3s;
  shard_range(n3_total, world, rank, &s0, &n3s);
  if (n3s <= 0) return 0;
  return make_plan(nullptr, batch, n1, n3s, num_leaf, with_conf != 0).bytes +
         align_up((size_t)batch * n3_total * 8, 256);
}

int onepose_match_sharded(const void* packed_weights, const float* desc2d, int64_t desc2d_bstride,
                          const float* desc3d_shard, int64_t desc3d_bstride,
                          const float* leaves_shard_prepared, int64_t prepared_bstride, int batch,
                          int n1, int n3_total, int num_leaf, int world, int rank,
                          float scale_factor, float match_threshold, int precision,
                          void* xchg_send, void* xchg_recv, size_t xchg_bytes,
                          onepose_allgather_fn allgather, void* user, int64_t* matches0,
                          int64_t* matches1, float* mscores0, float* mscores1, float* conf_shard,
                          void* workspace, size_t workspace_bytes, void* stream_) {
  clear_error();
  OP_REQUIRE(valid_precision(precision),
             "match_sharded: precision %d", precision);
  OP_REQUIRE(world >= 1 && rank >= 0 && rank < world, "match_sharded: rank %d of %d", rank, world);
  OP_REQUIRE(xchg_send && xchg_recv && allgather, "match_sharded: null exchange buffer/callback");
  int off, n3s;
  shard_range(n3_total, world, rank, &off, &n3s);
  OP_REQUIRE(n3s >= 1, "match_sharded: empty shard (n3_total %d, world %d)", n3_total, world);
  int rc = check_match_args(packed_weights, desc2d, desc3d_shard, leaves_shard_prepared, batch, n1,
                            n3s, num_leaf, scale_factor, matches0, matches1, mscores0, mscores1,
                            workspace);
  if (rc != ONEPOSE_OK) return rc;
  const size_t need_x = shard_xchg_bytes(batch, n1, n3_total, world);
  if (xchg_bytes < need_x) {
    set_error("match_sharded: exchange buffers %zu < %zu bytes per rank", xchg_bytes, need_x);
    return ONEPOSE_ERR_WORKSPACE;
  }
  const size_t need = onepose_match_sharded_workspace_bytes(batch, n1, n3_total, world, rank,
                                                            num_leaf, conf_shard != nullptr);
  if (workspace_bytes < need) {
    set_error("match_sharded: workspace %zu < %zu bytes", workspace_bytes, need);
    return ONEPOSE_ERR_WORKSPACE;
  }
  const Plan p = make_plan(workspace, batch, n1, n3s, num_leaf, conf_shard != nullptr);
  ShardCtx sh;
  sh.world = world;
  sh.rank = rank;
  sh.n3_total = n3_total;
  sh.offset = off;
  sh.max_shard = (n3_total + world - 1) / world;
  sh.send = static_cast<char*>(xchg_send);
  sh.recv = static_cast<char*>(xchg_recv);
  sh.cap = xchg_bytes;
  sh.fn = allgather;
  sh.user = user;
  sh.colbest_full = reinterpret_cast<unsigned long long*>(static_cast<char*>(workspace) +
                                                          align_up(p.bytes, 256));
  return match_impl(packed_weights, desc2d, desc2d_bstride, desc3d_shard, desc3d_bstride,
                    leaves_shard_prepared, prepared_bstride, batch, n1, n3s, num_leaf, scale_factor,
                    match_threshold, matches0, matches1, mscores0, mscores1, conf_shard, p,
                    static_cast<hipStream_t>(stream_), precision, &sh);
}

}  // extern "C"
