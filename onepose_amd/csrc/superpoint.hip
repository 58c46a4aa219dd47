// SuperPoint detector + descriptor (src/models/extractors/SuperPoint/superpoint.py:170-224)
// on gfx950: image [B][H][W] -> keypoints (x, y), scores, L2-normalised descriptors [256][k].
//
// Feature maps are NHWC fp32 (a pixel's channels contiguous).  Every 3x3 / 1x1 convolution is
// an implicit GEMM on v_mfma_f32_32x32x2_f32 (exact fp32 products, like the reference's
// conv2d up to summation order): tile = 64 output pixels x BN output channels, K = taps x
// Cin in 32-deep stages, operands staged through padded LDS (register prefetch two stages
// ahead, as in gemm.hip).  The 2x2 max-pool after conv1b/2b/3b is fused into the conv's
// epilogue: a tile's 64 rows are 16 pooled pixels x their 4 inputs, ordered so that one
// pooling window is a lane's 4 consecutive accumulator registers.  The score head's 1x1
// conv (65 logits, padded to 128) ends in softmax + pixel shuffle straight into the
// full-resolution score map.  NMS (simple_nms, :47-64) is five separable max-pool passes;
// keypoint selection keeps the reference's order (raster order when at most max_keypoints
// survive, torch.topk's score-descending order otherwise; equal scores by raster index).
#include "common.h"

namespace onepose {

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

struct SpLayer {
  int cin, cout, k, cout_pad;
};
constexpr int kSpLayers = 12;
// conv1a 1b 2a 2b 3a 3b 4a 4b Pa Pb Da Db   (superpoint.py:147-162)
constexpr SpLayer kSp[kSpLayers] = {{1, 64, 3, 64},     {64, 64, 3, 64},    {64, 64, 3, 64},
                                    {64, 64, 3, 64},    {64, 128, 3, 128},  {128, 128, 3, 128},
                                    {128, 128, 3, 128}, {128, 128, 3, 128}, {128, 256, 3, 256},
                                    {256, 65, 1, 128},  {128, 256, 3, 256}, {256, 256, 1, 256}};
const char* const kSpNames[kSpLayers] = {"conv1a", "conv1b", "conv2a", "conv2b",
                                         "conv3a", "conv3b", "conv4a", "conv4b",
                                         "convPa", "convPb", "convDa", "convDb"};

// packed: per layer W [cout_pad][k*k][cin] (zero rows past cout) then bias [cout_pad]
constexpr int64_t layer_floats(int i) {
  return (int64_t)kSp[i].cout_pad * kSp[i].k * kSp[i].k * kSp[i].cin + kSp[i].cout_pad;
}
constexpr int64_t layer_offset(int i) {
  int64_t o = 0;
  for (int j = 0; j < i; ++j) o += layer_floats(j);
  return o;
}
constexpr int64_t kSpPackedFloats = layer_offset(kSpLayers);

enum ConvEpi { CE_RELU = 0, CE_BIAS = 1, CE_SOFTMAX = 2 };

struct ConvArgs {
  const float* x;     // [B][H][W][cin]
  int64_t x_bs;
  const float* w;     // [cout_pad][taps][cin]
  const float* bias;  // [cout_pad]
  float* y;           // [B][Ho][Wo][cout]  (CE_SOFTMAX: score map [B][8H][8W])
  int64_t y_bs;
  int H, W, cin, cout, ks, mtiles, ntiles;
  StampAcc* stamp;
};

constexpr int CBM = 64, CBK = 32, CPITCH = CBK + 4;

template <int BN>
struct ConvStage {
  float4 a[2];
  float4 w[BN / 32];
  bool ok[2];
};

// Pixel of tile row m: raster order, or (POOL) pooled pixel m>>2 and its 2x2 input m&3.
template <bool POOL>
__device__ __forceinline__ void row_pixel(const ConvArgs& a, int mt, int m, int& y, int& x,
                                          bool& valid) {
  if (!POOL) {
    const int p = mt * CBM + m;
    valid = p < a.H * a.W;
    const int pc = valid ? p : 0;
    y = pc / a.W;
    x = pc - y * a.W;
  } else {
    const int wp = a.W >> 1, hp = a.H >> 1;
    const int pp = mt * (CBM / 4) + (m >> 2);
    valid = pp < hp * wp;
    const int pc = valid ? pp : 0;
    const int py = pc / wp, px = pc - py * wp;
    y = 2 * py + ((m >> 1) & 1);
    x = 2 * px + (m & 1);
  }
}

template <int BN, bool POOL, int EPI>
__global__ __launch_bounds__(256) void conv_kernel(ConvArgs a) {
  constexpr int FN = BN / 64;
  constexpr int STAGE = (CBM + BN) * CPITCH;
  __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];
  stamp_begin(a.stamp);
  const int b = blockIdx.y;
  const int mt = blockIdx.x / a.ntiles, nt = blockIdx.x - mt * a.ntiles;
  const int n0 = nt * BN;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, wm = wave >> 1, wn = wave & 1;
  const float* X = a.x + b * a.x_bs;
  const int taps = a.ks * a.ks, half = a.ks >> 1;
  const int chunks = a.cin / CBK;
  const int nk = taps * chunks;
  const int kq = (t & 7) * 4;
  int py[2], px[2];
  bool pv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) row_pixel<POOL>(a, mt, (t >> 3) + 32 * i, py[i], px[i], pv[i]);

  auto load = [&](int s, ConvStage<BN>& st) __attribute__((always_inline)) {
    const int tap = s / chunks, c0 = (s - tap * chunks) * CBK;
    const int dy = tap / a.ks - half, dx = tap - (tap / a.ks) * a.ks - half;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int yy = py[i] + dy, xx = px[i] + dx;
      st.ok[i] = pv[i] && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;   // zero padding
      const int yc = min(max(yy, 0), a.H - 1), xc = min(max(xx, 0), a.W - 1);
      st.a[i] = *reinterpret_cast<const float4*>(X + ((int64_t)yc * a.W + xc) * a.cin + c0 + kq);
    }
#pragma unroll
    for (int i = 0; i < BN / 32; ++i) {
      const int o = n0 + (t >> 3) + 32 * i;   // cout_pad rows exist for every tile row
      st.w[i] = *reinterpret_cast<const float4*>(a.w + ((int64_t)o * taps + tap) * a.cin + c0 + kq);
    }
  };
  auto store = [&](float* la, ConvStage<BN>& st) __attribute__((always_inline)) {
    float* lw = la + CBM * CPITCH;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(la + ((t >> 3) + 32 * i) * CPITCH + kq) = st.ok[i] ? st.a[i] : z;
    }
#pragma unroll
    for (int i = 0; i < BN / 32; ++i)
      *reinterpret_cast<float4*>(lw + ((t >> 3) + 32 * i) * CPITCH + kq) = st.w[i];
  };

  floatx16 acc[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;

  ConvStage<BN> s0, s1;
  load(0, s0);
  load(min(1, nk - 1), s1);
  store(lds, s0);
  __syncthreads();
  auto step = [&](int kt, ConvStage<BN>& next, ConvStage<BN>& spare)
      __attribute__((always_inline)) {
    load(min(kt + 2, nk - 1), spare);
    const float* la = lds + (kt & 1) * STAGE;
    const float* pa = la + (wm * 32 + (lane & 31)) * CPITCH + (lane >> 5) * 4;
    const float* pw = la + CBM * CPITCH + (wn * (BN / 2) + (lane & 31)) * CPITCH + (lane >> 5) * 4;
#pragma unroll
    for (int kk = 0; kk < CBK / 8; ++kk) {
      const float4 av = *reinterpret_cast<const float4*>(pa + kk * 8);
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const float4 wv = *reinterpret_cast<const float4*>(pw + j * 32 * CPITCH + kk * 8);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, wv.x, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, wv.y, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, wv.z, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, wv.w, acc[j], 0, 0, 0);
      }
    }
    store(lds + ((kt + 1) & 1) * STAGE, next);   // (unused after the last stage)
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += 2) {   // nk even: taps x cin/32 with cin % 64 == 0
    step(kt, s1, s0);
    step(kt + 1, s0, s1);
  }

  float* Y = a.y + b * a.y_bs;
  if (EPI != CE_SOFTMAX) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * (BN / 2) + j * 32 + (lane & 31);
      const bool n_ok = n < a.cout;
      const float bias = n_ok ? a.bias[n] : 0.f;
      if (!POOL) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int m = wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
          const int p = mt * CBM + m;
          float v = acc[j][i] + bias;
          if (EPI == CE_RELU) v = fmaxf(v, 0.f);
          if (n_ok && p < a.H * a.W) Y[(int64_t)p * a.cout + n] = v;
        }
      } else {
        const int hp = a.H >> 1, wp = a.W >> 1;
#pragma unroll
        for (int g = 0; g < 4; ++g) {   // registers 4g..4g+3 = one 2x2 window
          const int m = wm * 32 + 8 * g + 4 * (lane >> 5);
          const int pp = mt * (CBM / 4) + (m >> 2);
          float v = fmaxf(fmaxf(acc[j][4 * g], acc[j][4 * g + 1]),
                          fmaxf(acc[j][4 * g + 2], acc[j][4 * g + 3])) + bias;
          if (EPI == CE_RELU) v = fmaxf(v, 0.f);   // relu(max(.)) == max(relu(.))
          if (n_ok && pp < hp * wp) Y[(int64_t)pp * a.cout + n] = v;
        }
      }
    }
    stamp_end(a.stamp);
    return;
  }
  // CE_SOFTMAX: 64 cells x 65 logits -> softmax over 65, drop the dustbin, pixel shuffle
  // (scores.permute(0,2,3,1).reshape(b,h,w,8,8).permute(0,1,3,2,4).reshape(b,8h,8w), :181-183)
  static_assert(EPI != CE_SOFTMAX || BN == 128, "softmax head tile holds all 65 logits");
  float* tile = lds;   // [64][129]
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = wn * (BN / 2) + j * 32 + (lane & 31);
    const float bias = n < a.cout ? a.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int m = wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
      tile[m * 129 + n] = acc[j][i] + bias;
    }
  }
  __syncthreads();
  {
    const int m = t >> 2, q = t & 3;   // 4 threads per cell, 16 channels each
    const float* row = tile + m * 129;
    float mx = -INFINITY;
    for (int c = 0; c < 65; ++c) mx = fmaxf(mx, row[c]);
    float sum = 0.f;
    for (int c = 0; c < 65; ++c) sum += expf(row[c] - mx);
    const int p = mt * CBM + m;
    if (p < a.H * a.W) {
      const int cy = p / a.W, cx = p - cy * a.W;
      const int W8 = a.W * 8;
#pragma unroll
      for (int cc = 0; cc < 16; ++cc) {
        const int c = q * 16 + cc;
        Y[(int64_t)(cy * 8 + (c >> 3)) * W8 + cx * 8 + (c & 7)] = expf(row[c] - mx) / sum;
      }
    }
  }
  stamp_end(a.stamp);
}

// conv1a (1 -> 64, 3x3, pad 1) + ReLU, direct: one thread per pixel, weights in LDS.
__global__ __launch_bounds__(256) void conv1a_kernel(const float* __restrict__ img, int64_t img_bs,
                                                     const float* __restrict__ w,
                                                     const float* __restrict__ bias, int H, int W,
                                                     float* __restrict__ y, int64_t y_bs) {
  __shared__ float sw[64 * 9], sb[64];
  for (int i = threadIdx.x; i < 64 * 9; i += 256) sw[i] = w[i];
  if (threadIdx.x < 64) sb[threadIdx.x] = bias[threadIdx.x];
  __syncthreads();
  const int b = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= H * W) return;
  const int py = p / W, px = p - py * W;
  const float* I = img + b * img_bs;
  float v[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = py + k / 3 - 1, xx = px + k % 3 - 1;
    v[k] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? I[yy * W + xx] : 0.f;
  }
  float4* out = reinterpret_cast<float4*>(y + b * y_bs + (int64_t)p * 64);
#pragma unroll
  for (int c4 = 0; c4 < 16; ++c4) {
    float r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c4 * 4 + j;
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 9; ++k) s += v[k] * sw[c * 9 + k];
      r[j] = fmaxf(s + sb[c], 0.f);
    }
    out[c4] = make_float4(r[0], r[1], r[2], r[3]);
  }
}

// ---- simple_nms (superpoint.py:47-64): max_pool2d(k=2r+1, stride 1, pad r) passes ----
enum NmsMode { NMS_INIT = 0, NMS_SUPP = 1, NMS_GROW = 2 };
struct NmsArgs {
  const float* s;   // scores [B][H][W]
  float* mask;      // max_mask (0/1)
  float* supp;      // supp_mask (0/1)
  float* ss;        // supp_scores
  int H, W, r;
  int64_t bs;
};
constexpr int NT = 32, NMAXR = 8;

// One 32x32 output tile: the pass's input over the tile + halo r is staged in LDS, the
// (2r+1)^2 max is taken separably (rows, then columns); padding counts as -inf.
template <int MODE>
__global__ __launch_bounds__(256) void nms_kernel(NmsArgs a) {
  __shared__ float in[NT + 2 * NMAXR][NT + 2 * NMAXR + 1];
  __shared__ float rowmax[NT + 2 * NMAXR][NT + 1];
  const int b = blockIdx.z, y0 = blockIdx.y * NT, x0 = blockIdx.x * NT, r = a.r;
  const int E = NT + 2 * r;
  const int64_t o = b * a.bs;
  for (int e = threadIdx.x; e < E * E; e += 256) {
    const int ey = e / E, ex = e - ey * E;
    const int yy = y0 + ey - r, xx = x0 + ex - r;
    float v = -INFINITY;
    if (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W) {
      const int64_t i = o + (int64_t)yy * a.W + xx;
      v = MODE == NMS_INIT ? a.s[i] : MODE == NMS_SUPP ? a.mask[i] : a.ss[i];
    }
    in[ey][ex] = v;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < E * NT; e += 256) {
    const int ey = e / NT, ox = e - ey * NT;
    float m = -INFINITY;
    for (int d = 0; d <= 2 * r; ++d) m = fmaxf(m, in[ey][ox + d]);
    rowmax[ey][ox] = m;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < NT * NT; e += 256) {
    const int oy = e / NT, ox = e - oy * NT;
    const int yy = y0 + oy, xx = x0 + ox;
    if (yy >= a.H || xx >= a.W) continue;
    float m = -INFINITY;
    for (int d = 0; d <= 2 * r; ++d) m = fmaxf(m, rowmax[oy + d][ox]);
    const int64_t i = o + (int64_t)yy * a.W + xx;
    const float c = in[oy + r][ox + r];
    if (MODE == NMS_INIT) {
      a.mask[i] = (c == m) ? 1.f : 0.f;                       // scores == max_pool(scores)
    } else if (MODE == NMS_SUPP) {
      const bool sp = m > 0.f;                                // max_pool(max_mask) > 0
      a.supp[i] = sp ? 1.f : 0.f;
      a.ss[i] = sp ? 0.f : a.s[i];                            // where(supp, 0, scores)
    } else {
      const bool nm = c == m;                                 // supp == max_pool(supp)
      if (nm && a.supp[i] == 0.f) a.mask[i] = 1.f;            // max_mask |= new & ~supp
    }
  }
}

// ---- keypoint selection: threshold + borders, raster-order compaction, top-k ----
constexpr int kSelChunk = 4096;
struct SelArgs {
  const float* s;       // scores [B][H][W]
  const float* mask;    // NMS max_mask
  int H, W, border, max_kp;
  float thr;
  int64_t bs;
  int chunks;           // per sample
  int* chunk_count;     // [B][chunks]
  int* chunk_off;       // [B][chunks]
  int* total;           // [B]
  float* cand_score;    // [B][H*W] raster-order candidates
  int* cand_idx;
  float* kpts;          // [B][max_kp][2] (x, y)
  float* kscores;       // [B][max_kp]
  int* counts;          // [B]
};

__device__ __forceinline__ bool is_cand(const SelArgs& a, int64_t o, int p, float& v) {
  const int y = p / a.W, x = p - (p / a.W) * a.W;
  // nms score = where(max_mask, scores, 0) > threshold; remove_borders (:66-76)
  v = a.mask[o + p] != 0.f ? a.s[o + p] : 0.f;
  return v > a.thr && y >= a.border && y < a.H - a.border && x >= a.border &&
         x < a.W - a.border;
}

__global__ __launch_bounds__(256) void sel_count_kernel(SelArgs a) {
  __shared__ int red[4];
  const int b = blockIdx.y, ch = blockIdx.x;
  const int64_t o = b * a.bs;
  int c = 0;
  for (int p = ch * kSelChunk + threadIdx.x; p < min((ch + 1) * kSelChunk, a.H * a.W); p += 256) {
    float v;
    c += is_cand(a, o, p, v) ? 1 : 0;
  }
  for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) a.chunk_count[b * a.chunks + ch] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(64) void sel_scan_kernel(SelArgs a) {
  const int b = blockIdx.x;
  if (threadIdx.x != 0) return;
  int run = 0;
  for (int c = 0; c < a.chunks; ++c) {
    a.chunk_off[b * a.chunks + c] = run;
    run += a.chunk_count[b * a.chunks + c];
  }
  a.total[b] = run;
}

// Scatter candidates in raster order: each wave compacts 64 pixels with a ballot.
__global__ __launch_bounds__(256) void sel_scatter_kernel(SelArgs a) {
  __shared__ int wbase[4][kSelChunk / 256];
  const int b = blockIdx.y, ch = blockIdx.x;
  const int64_t o = b * a.bs;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int p0 = ch * kSelChunk;
  // pass 1: per (wave, round) counts; rounds cover 256 pixels each
  constexpr int R = kSelChunk / 256;
  bool c[R];
  float v[R];
  for (int rr = 0; rr < R; ++rr) {
    const int p = p0 + rr * 256 + wave * 64 + lane;
    c[rr] = p < a.H * a.W && is_cand(a, o, p, v[rr]);
    const unsigned long long bal = __ballot(c[rr]);
    if (lane == 0) wbase[wave][rr] = __popcll(bal);
  }
  __syncthreads();
  if (threadIdx.x == 0) {   // exclusive scan in raster order: round-major, wave-minor
    int run = a.chunk_off[b * a.chunks + ch];
    for (int rr = 0; rr < R; ++rr)
      for (int w = 0; w < 4; ++w) {
        const int n = wbase[w][rr];
        wbase[w][rr] = run;
        run += n;
      }
  }
  __syncthreads();
  float* cs = a.cand_score + o;
  int* ci = a.cand_idx + o;
  for (int rr = 0; rr < R; ++rr) {
    const unsigned long long bal = __ballot(c[rr]);
    if (c[rr]) {
      const int pos = wbase[wave][rr] + __popcll(bal & ((1ull << lane) - 1ull));
      cs[pos] = v[rr];
      ci[pos] = p0 + rr * 256 + wave * 64 + lane;
    }
  }
}

// One workgroup per sample.  total <= max_kp: the candidates as they are (raster order, the
// reference's nonzero order).  Otherwise torch.topk(k): radix-select the k-th largest score
// on its bit pattern (scores > 0), gather the winners (ties by raster index) and bitonic-sort
// them by (score desc, raster index asc) in LDS.
__global__ __launch_bounds__(1024) void sel_final_kernel(SelArgs a) {
  extern __shared__ unsigned long long keys[];   // [pow2 >= max_kp]
  __shared__ int hist[256];
  __shared__ unsigned prefix_s, mask_s;
  __shared__ int need_s, ngt_s, neq_s;
  const int b = blockIdx.x, t = threadIdx.x;
  const int total = a.total[b], k = a.max_kp;
  const int64_t o = b * a.bs;
  const float* cs = a.cand_score + o;
  const int* ci = a.cand_idx + o;
  float* kp = a.kpts + (int64_t)b * k * 2;
  float* ks = a.kscores + (int64_t)b * k;
  if (total <= k) {
    for (int i = t; i < k; i += 1024) {
      const bool on = i < total;
      const int p = on ? ci[i] : 0;
      kp[2 * i] = on ? (float)(p % a.W) : 0.f;   // flip (y, x) -> (x, y)
      kp[2 * i + 1] = on ? (float)(p / a.W) : 0.f;
      ks[i] = on ? cs[i] : 0.f;
    }
    if (t == 0) a.counts[b] = total;
    return;
  }
  // radix select: the k-th largest bit pattern, 8 bits at a time from the top
  if (t == 0) {
    prefix_s = 0u;
    mask_s = 0u;
    need_s = k;
  }
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = t; i < 256; i += 1024) hist[i] = 0;
    __syncthreads();
    const unsigned pre = prefix_s, msk = mask_s;
    for (int i = t; i < total; i += 1024) {
      const unsigned u = __float_as_uint(cs[i]);
      if ((u & msk) == pre) atomicAdd(&hist[(u >> shift) & 255], 1);
    }
    __syncthreads();
    if (t == 0) {
      int need = need_s, d = 255;
      for (; d > 0; --d) {
        if (hist[d] >= need) break;
        need -= hist[d];
      }
      prefix_s = pre | ((unsigned)d << shift);
      mask_s = msk | (255u << shift);
      need_s = need;   // how many of the bin's pattern (the threshold) are still needed
    }
    __syncthreads();
  }
  const unsigned thr_u = prefix_s;
  if (t == 0) {
    ngt_s = 0;
    neq_s = 0;
  }
  int P = 1;
  while (P < k) P <<= 1;
  for (int i = t; i < P; i += 1024) keys[i] = 0ull;
  __syncthreads();
  // winners: every score above the threshold, and the first need_s equal to it (raster order)
  const int n_eq = need_s;
  const int n_gt = k - n_eq;
  for (int base = 0; base < total; base += 1024) {
    const int i = base + t;
    const unsigned u = i < total ? __float_as_uint(cs[i]) : 0u;
    const bool gt = i < total && u > thr_u, eq = i < total && u == thr_u;
    // equal ones must be taken in raster order: rank them within this round, in order
    __shared__ int eq_rank[1024];
    eq_rank[t] = eq ? 1 : 0;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {   // inclusive scan
      const int v = t >= off ? eq_rank[t - off] : 0;
      __syncthreads();
      eq_rank[t] += v;
      __syncthreads();
    }
    const int eq_before = neq_s;
    if (gt) {
      const int slot = atomicAdd(&ngt_s, 1);
      keys[slot] = ((unsigned long long)u << 32) | (0xFFFFFFFFu - (unsigned)ci[i]);
    }
    if (eq) {
      const int r = eq_before + eq_rank[t] - 1;
      if (r < n_eq) keys[n_gt + r] = ((unsigned long long)u << 32) | (0xFFFFFFFFu - (unsigned)ci[i]);
    }
    __syncthreads();
    if (t == 1023) neq_s = eq_before + eq_rank[1023];
    __syncthreads();
  }
  // bitonic sort, descending by key (score desc, raster index asc)
  for (int size = 2; size <= P; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = t; i < P; i += 1024) {
        const int j = i ^ stride;
        if (j > i) {
          const unsigned long long ki = keys[i], kj = keys[j];
          const bool desc = (i & size) == 0;
          if (desc ? (ki < kj) : (ki > kj)) {
            keys[i] = kj;
            keys[j] = ki;
          }
        }
      }
      __syncthreads();
    }
  for (int i = t; i < k; i += 1024) {
    const unsigned long long key = keys[i];
    const int p = (int)(0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull));
    kp[2 * i] = (float)(p % a.W);
    kp[2 * i + 1] = (float)(p / a.W);
    ks[i] = __uint_as_float((unsigned)(key >> 32));
  }
  if (t == 0) a.counts[b] = k;
}

// ---- descriptors: normalise the dense map per cell, then sample at the keypoints ----
__global__ __launch_bounds__(256) void desc_norm_kernel(float* d, int cells) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= cells) return;
  float4* p = reinterpret_cast<float4*>(d + (int64_t)c * 256) + lane;
  float4 v = *p;
  const float ss = wave_sum(v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w);
  const float n = fmaxf(sqrtf(ss), 1e-12f);   // F.normalize(p=2, dim=1)
  *p = make_float4(v.x / n, v.y / n, v.z / n, v.w / n);
}

// sample_descriptors (superpoint.py:95-113) on the NHWC dense map [h][w][256]: one wave per
// keypoint (4 channels per lane), the same arithmetic order as frame_ops.hip's NCHW kernel;
// 64 keypoints per workgroup are written through LDS as [256][k] columns.
__global__ __launch_bounds__(256) void sample_nhwc_kernel(const float* __restrict__ kpts,
                                                          const int* __restrict__ counts,
                                                          const float* __restrict__ dense,
                                                          int max_kp, int h, int w, int s,
                                                          int align_corners,
                                                          float* __restrict__ out) {
#pragma clang fp contract(off)
  __shared__ float tile[256][65];
  const int b = blockIdx.y, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int k0 = blockIdx.x * 64;
  const int cnt = counts[b];
  const float* D = dense + (int64_t)b * h * w * 256;
  for (int kk = wave; kk < 64; kk += 4) {
    const int k = k0 + kk;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (k < cnt) {
      const float hs = (float)s / 2.0f;
      float x = kpts[((int64_t)b * max_kp + k) * 2 + 0];
      float y = kpts[((int64_t)b * max_kp + k) * 2 + 1];
      x = (x - hs) + 0.5f;
      y = (y - hs) + 0.5f;
      x = x / (float)((double)w * s - s / 2.0 - 0.5);
      y = y / (float)((double)h * s - s / 2.0 - 0.5);
      x = x * 2.0f - 1.0f;
      y = y * 2.0f - 1.0f;
      float ix, iy;
      if (align_corners) {
        ix = ((x + 1.0f) / 2.0f) * (float)(w - 1);
        iy = ((y + 1.0f) / 2.0f) * (float)(h - 1);
      } else {
        ix = ((x + 1.0f) * (float)w - 1.0f) / 2.0f;
        iy = ((y + 1.0f) * (float)h - 1.0f) / 2.0f;
      }
      const int x0 = (int)floorf(ix), y0 = (int)floorf(iy), x1 = x0 + 1, y1 = y0 + 1;
      const float wnw = ((float)x1 - ix) * ((float)y1 - iy);
      const float wne = (ix - (float)x0) * ((float)y1 - iy);
      const float wsw = ((float)x1 - ix) * (iy - (float)y0);
      const float wse = (ix - (float)x0) * (iy - (float)y0);
      auto corner = [&](int cx, int cy, float wt, float4& acc) {
        if (cx >= 0 && cx < w && cy >= 0 && cy < h) {
          const float4 q = reinterpret_cast<const float4*>(D + ((int64_t)cy * w + cx) * 256)[lane];
          acc.x += q.x * wt;
          acc.y += q.y * wt;
          acc.z += q.z * wt;
          acc.w += q.w * wt;
        }
      };
      corner(x0, y0, wnw, v);
      corner(x1, y0, wne, v);
      corner(x0, y1, wsw, v);
      corner(x1, y1, wse, v);
      // the NCHW kernel sums lane-strided channels; the norm's summation order differs only
      const float ss = wave_sum(v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w);
      const float nrm = fmaxf(sqrtf(ss), 1e-12f);
      v = make_float4(v.x / nrm, v.y / nrm, v.z / nrm, v.w / nrm);
    }
    tile[lane * 4 + 0][kk] = v.x;
    tile[lane * 4 + 1][kk] = v.y;
    tile[lane * 4 + 2][kk] = v.z;
    tile[lane * 4 + 3][kk] = v.w;
  }
  __syncthreads();
  float* O = out + (int64_t)b * 256 * max_kp;
  for (int e = threadIdx.x; e < 256 * 64; e += 256) {
    const int c = e >> 6, kk = e & 63;
    if (k0 + kk < max_kp) O[(int64_t)c * max_kp + k0 + kk] = tile[c][kk];
  }
}

// ---- plan ----
struct DetPlan {   // NMS + selection scratch
  float *mask, *supp, *ss;        // [H][W]
  float* cand_score;
  int *cand_idx, *chunk_count, *chunk_off, *total;
};
struct SpPlan {
  float *f0, *f1;                 // ping-pong feature maps (largest: H*W*64)
  float *x4, *head;               // encoder output [H/8][W/8][128], head hidden [H/8][W/8][256]
  float *dense;                   // [H/8][W/8][256]
  float* score;                   // [H][W]
  DetPlan det;
  size_t bytes;
};

DetPlan det_plan(Carve& c, int B, int H, int W) {
  DetPlan p;
  const size_t hw = (size_t)H * W;
  const int chunks = (int)((hw + kSelChunk - 1) / kSelChunk);
  p.mask = c.take<float>(B * hw);
  p.supp = c.take<float>(B * hw);
  p.ss = c.take<float>(B * hw);
  p.cand_score = c.take<float>(B * hw);
  p.cand_idx = c.take<int>(B * hw);
  p.chunk_count = c.take<int>((size_t)B * chunks);
  p.chunk_off = c.take<int>((size_t)B * chunks);
  p.total = c.take<int>(B);
  return p;
}

SpPlan sp_plan(void* ws, int B, int H, int W) {
  Carve c(ws);
  SpPlan p;
  const size_t hw = (size_t)H * W, hw8 = (size_t)(H / 8) * (W / 8);
  p.f0 = c.take<float>(B * hw * 64);
  p.f1 = c.take<float>(B * hw / 4 * 64 + 64);
  p.x4 = c.take<float>(B * hw8 * 128);
  p.head = c.take<float>(B * hw8 * 256);
  p.dense = c.take<float>(B * hw8 * 256);
  p.score = c.take<float>(B * hw);
  p.det = det_plan(c, B, H, W);
  p.bytes = align_up(c.off, 256);
  return p;
}

size_t det_bytes(int B, int H, int W) {
  Carve c(nullptr);
  det_plan(c, B, H, W);
  return align_up(c.off, 256);
}

template <int BN, bool POOL, int EPI>
int conv_launch(const float* x, int B, int H, int W, const float* packed, int layer, float* y,
                hipStream_t st) {
  const SpLayer& L = kSp[layer];
  ConvArgs a;
  a.x = x;
  a.x_bs = (int64_t)H * W * L.cin;
  a.w = packed + layer_offset(layer);
  a.bias = a.w + (int64_t)L.cout_pad * L.k * L.k * L.cin;
  a.y = y;
  a.H = H;
  a.W = W;
  a.cin = L.cin;
  a.cout = L.cout;
  a.ks = L.k;
  const int pix = POOL ? (H / 2) * (W / 2) : H * W;
  a.mtiles = ceil_div(pix, POOL ? CBM / 4 : CBM);
  a.ntiles = L.cout_pad / BN;
  a.stamp = prof_stamp_slot(K_SP_CONV);
  a.y_bs = EPI == CE_SOFTMAX ? (int64_t)H * W * 64 : (int64_t)pix * L.cout;
  OP_LAUNCH(K_SP_CONV, st, (conv_kernel<BN, POOL, EPI>), dim3(a.mtiles * a.ntiles, B), dim3(256),
            0, st, a);
  return ONEPOSE_OK;
}

constexpr int kMaxSortKeypoints = 16384;

int check_detect_args(int batch, int h, int w, int nms_radius, int remove_borders,
                      int max_keypoints) {
  OP_REQUIRE(batch >= 1 && h >= 16 && w >= 16 && h % 8 == 0 && w % 8 == 0,
             "superpoint: image %dx%d (batch %d): sides must be multiples of 8, >= 16", h, w,
             batch);
  OP_REQUIRE(nms_radius >= 0 && nms_radius <= NMAXR, "superpoint: nms_radius %d not in [0,%d]",
             nms_radius, NMAXR);
  OP_REQUIRE(remove_borders >= 0, "superpoint: remove_borders %d", remove_borders);
  // top-k sorts in LDS; a capacity of every pixel (max_keypoints -1) never needs the sort
  OP_REQUIRE(max_keypoints >= 1 &&
                 (max_keypoints <= kMaxSortKeypoints || (int64_t)max_keypoints >= (int64_t)h * w),
             "superpoint: max_keypoints %d not in [1, %d] nor >= h*w", max_keypoints,
             kMaxSortKeypoints);
  return ONEPOSE_OK;
}

// simple_nms -> threshold/borders -> top-k -> descriptor sampling, from a score map
// [B][h][w] and a normalised NHWC dense descriptor map [B][h/8][w/8][256].
int detect_impl(const float* score, const float* dense, int B, int h, int w, int nms_radius,
                float thr, int border, int max_kp, int align_corners, float* keypoints,
                float* scores, float* descriptors, int* counts, const DetPlan& p,
                hipStream_t st) {
  // simple_nms: mask = s == mp(s); twice { supp = mp(mask) > 0; ss = supp ? 0 : s;
  //                                        mask |= (ss == mp(ss)) & ~supp }
  NmsArgs na{score, p.mask, p.supp, p.ss, h, w, nms_radius, (int64_t)h * w};
  const dim3 ng(ceil_div(w, NT), ceil_div(h, NT), B);
  OP_LAUNCH(K_SP_NMS, st, nms_kernel<NMS_INIT>, ng, dim3(256), 0, st, na);
  for (int it = 0; it < 2; ++it) {
    OP_LAUNCH(K_SP_NMS, st, nms_kernel<NMS_SUPP>, ng, dim3(256), 0, st, na);
    OP_LAUNCH(K_SP_NMS, st, nms_kernel<NMS_GROW>, ng, dim3(256), 0, st, na);
  }
  SelArgs sa;
  sa.s = score;
  sa.mask = p.mask;
  sa.H = h;
  sa.W = w;
  sa.border = border;
  sa.max_kp = max_kp;
  sa.thr = thr;
  sa.bs = (int64_t)h * w;
  sa.chunks = ceil_div(h * w, kSelChunk);
  sa.chunk_count = p.chunk_count;
  sa.chunk_off = p.chunk_off;
  sa.total = p.total;
  sa.cand_score = p.cand_score;
  sa.cand_idx = p.cand_idx;
  sa.kpts = keypoints;
  sa.kscores = scores;
  sa.counts = counts;
  OP_LAUNCH(K_SP_SELECT, st, sel_count_kernel, dim3(sa.chunks, B), dim3(256), 0, st, sa);
  OP_LAUNCH(K_SP_SELECT, st, sel_scan_kernel, dim3(B), dim3(64), 0, st, sa);
  OP_LAUNCH(K_SP_SELECT, st, sel_scatter_kernel, dim3(sa.chunks, B), dim3(256), 0, st, sa);
  size_t shm = 0;
  if (max_kp <= kMaxSortKeypoints) {
    int P2 = 1;
    while (P2 < max_kp) P2 <<= 1;
    shm = (size_t)P2 * 8;
  }
  static bool attr_set = false;
  if (!attr_set) {
    OP_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(sel_final_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               kMaxSortKeypoints * 8));
    attr_set = true;
  }
  OP_LAUNCH(K_SP_SELECT, st, sel_final_kernel, dim3(B), dim3(1024), shm, st, sa);
  OP_LAUNCH(K_SP_DESC, st, sample_nhwc_kernel, dim3(ceil_div(max_kp, 64), B), dim3(256), 0, st,
            keypoints, counts, dense, max_kp, h / 8, w / 8, 8, align_corners, descriptors);
  return ONEPOSE_OK;
}

}  // namespace
}  // namespace onepose

using namespace onepose;

extern "C" {

int onepose_superpoint_num_tensors(void) { return 2 * kSpLayers; }

const char* onepose_superpoint_tensor_name(int i) {
  static std::string names[2 * kSpLayers];
  if (i < 0 || i >= 2 * kSpLayers) return nullptr;
  if (names[i].empty()) names[i] = std::string(kSpNames[i / 2]) + (i % 2 ? ".bias" : ".weight");
  return names[i].c_str();
}

size_t onepose_superpoint_packed_bytes(void) { return (size_t)kSpPackedFloats * sizeof(float); }

int onepose_superpoint_pack(const float* const* tensors, int n_tensors, void* packed_host) {
  clear_error();
  OP_REQUIRE(tensors != nullptr && packed_host != nullptr, "superpoint_pack: null pointer");
  OP_REQUIRE(n_tensors == 2 * kSpLayers, "superpoint_pack: expected %d tensors, got %d",
             2 * kSpLayers, n_tensors);
  float* out = static_cast<float*>(packed_host);
  for (int l = 0; l < kSpLayers; ++l) {
    const SpLayer& L = kSp[l];
    const float* w = tensors[2 * l];       // torch [cout][cin][k][k]
    const float* bias = tensors[2 * l + 1];
    OP_REQUIRE(w != nullptr && bias != nullptr, "superpoint_pack: tensor %d null", 2 * l);
    float* dw = out + layer_offset(l);
    const int taps = L.k * L.k;
    float* db = dw + (int64_t)L.cout_pad * taps * L.cin;
    for (int o = 0; o < L.cout_pad; ++o) {
      for (int tp = 0; tp < taps; ++tp)
        for (int c = 0; c < L.cin; ++c)
          dw[((int64_t)o * taps + tp) * L.cin + c] =
              o < L.cout ? w[((int64_t)o * L.cin + c) * taps + tp] : 0.f;
      db[o] = o < L.cout ? bias[o] : 0.f;
    }
  }
  return ONEPOSE_OK;
}

size_t onepose_superpoint_workspace_bytes(int batch, int h, int w) {
  if (batch <= 0 || h <= 0 || w <= 0) return 0;
  return sp_plan(nullptr, batch, h, w).bytes;
}

int onepose_superpoint(const void* packed, const float* image, int batch, int h, int w,
                       int nms_radius, float keypoint_threshold, int remove_borders,
                       int max_keypoints, int align_corners, float* keypoints, float* scores,
                       float* descriptors, int* counts, float* score_map, float* dense_desc,
                       void* workspace, size_t workspace_bytes, void* stream_) {
  clear_error();
  OP_REQUIRE(packed && image && keypoints && scores && descriptors && counts,
             "superpoint: null pointer");
  int rc;
  if ((rc = check_detect_args(batch, h, w, nms_radius, remove_borders, max_keypoints)))
    return rc;
  const SpPlan need = sp_plan(nullptr, batch, h, w);
  OP_REQUIRE(workspace != nullptr, "superpoint: null workspace");
  if (workspace_bytes < need.bytes) {
    set_error("superpoint: workspace %zu < %zu bytes", workspace_bytes, need.bytes);
    return ONEPOSE_ERR_WORKSPACE;
  }
  hipStream_t st = static_cast<hipStream_t>(stream_);
  const SpPlan p = sp_plan(workspace, batch, h, w);
  const float* P = static_cast<const float*>(packed);
  const int B = batch;
  // shared encoder: conv1a, [1b+pool], 2a, [2b+pool], 3a, [3b+pool], 4a, 4b
  OP_LAUNCH(K_SP_CONV, st, conv1a_kernel, dim3(ceil_div(h * w, 256), B), dim3(256), 0, st, image,
            (int64_t)h * w, P + layer_offset(0), P + layer_offset(0) + 64 * 9, h, w, p.f0,
            (int64_t)h * w * 64);
  if ((rc = conv_launch<64, true, CE_RELU>(p.f0, B, h, w, P, 1, p.f1, st))) return rc;
  if ((rc = conv_launch<64, false, CE_RELU>(p.f1, B, h / 2, w / 2, P, 2, p.f0, st))) return rc;
  if ((rc = conv_launch<64, true, CE_RELU>(p.f0, B, h / 2, w / 2, P, 3, p.f1, st))) return rc;
  if ((rc = conv_launch<64, false, CE_RELU>(p.f1, B, h / 4, w / 4, P, 4, p.f0, st))) return rc;
  if ((rc = conv_launch<64, true, CE_RELU>(p.f0, B, h / 4, w / 4, P, 5, p.f1, st))) return rc;
  if ((rc = conv_launch<64, false, CE_RELU>(p.f1, B, h / 8, w / 8, P, 6, p.f0, st))) return rc;
  if ((rc = conv_launch<64, false, CE_RELU>(p.f0, B, h / 8, w / 8, P, 7, p.x4, st))) return rc;
  // score head: convPa + ReLU, convPb -> softmax(65)[:64] -> pixel shuffle -> [H][W]
  if ((rc = conv_launch<64, false, CE_RELU>(p.x4, B, h / 8, w / 8, P, 8, p.head, st))) return rc;
  if ((rc = conv_launch<128, false, CE_SOFTMAX>(p.head, B, h / 8, w / 8, P, 9, p.score, st)))
    return rc;
  // descriptor head: convDa + ReLU, convDb, normalise (the score head's hidden map is dead)
  if ((rc = conv_launch<64, false, CE_RELU>(p.x4, B, h / 8, w / 8, P, 10, p.head, st))) return rc;
  if ((rc = conv_launch<64, false, CE_BIAS>(p.head, B, h / 8, w / 8, P, 11, p.dense, st)))
    return rc;
  const int cells = B * (h / 8) * (w / 8);
  OP_LAUNCH(K_SP_DESC, st, desc_norm_kernel, dim3(ceil_div(cells, 4)), dim3(256), 0, st, p.dense,
            cells);
  if ((rc = detect_impl(p.score, p.dense, B, h, w, nms_radius, keypoint_threshold,
                        remove_borders, max_keypoints, align_corners, keypoints, scores,
                        descriptors, counts, p.det, st)))
    return rc;
  if (score_map)
    OP_HIP(hipMemcpyAsync(score_map, p.score, sizeof(float) * B * h * w,
                          hipMemcpyDeviceToDevice, st));
  if (dense_desc)
    OP_HIP(hipMemcpyAsync(dense_desc, p.dense, sizeof(float) * cells * 256,
                          hipMemcpyDeviceToDevice, st));
  return ONEPOSE_OK;
}

size_t onepose_superpoint_detect_workspace_bytes(int batch, int h, int w) {
  if (batch <= 0 || h <= 0 || w <= 0) return 0;
  return det_bytes(batch, h, w);
}

int onepose_superpoint_detect(const float* score_map, const float* dense_desc, int batch, int h,
                              int w, int nms_radius, float keypoint_threshold, int remove_borders,
                              int max_keypoints, int align_corners, float* keypoints,
                              float* scores, float* descriptors, int* counts, void* workspace,
                              size_t workspace_bytes, void* stream) {
  clear_error();
  OP_REQUIRE(score_map && dense_desc && keypoints && scores && descriptors && counts &&
                 workspace,
             "superpoint_detect: null pointer");
  int rc;
  if ((rc = check_detect_args(batch, h, w, nms_radius, remove_borders, max_keypoints)))
    return rc;
  if (workspace_bytes < det_bytes(batch, h, w)) {
    set_error("superpoint_detect: workspace %zu < %zu bytes", workspace_bytes,
              det_bytes(batch, h, w));
    return ONEPOSE_ERR_WORKSPACE;
  }
  Carve c(workspace);
  const DetPlan p = det_plan(c, batch, h, w);
  return detect_impl(score_map, dense_desc, batch, h, w, nms_radius, keypoint_threshold,
                     remove_borders, max_keypoints, align_corners, keypoints, scores, descriptors,
                     counts, p, static_cast<hipStream_t>(stream));
}

}  // extern "C"
