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

#include <cstdlib>

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

constexpr int CBK = 32, CPITCH = CBK + 4;

// Tile shape: WM x WN waves, each owning 32 rows x 32*FN output channels, times KS groups of
// such waves that split the K stages (taps x channel chunks) and reduce through LDS at the end.
template <int WM_, int WN_, int FN_, int KS_>
struct ConvTile {
  static constexpr int WM = WM_, WN = WN_, FN = FN_, KS = KS_;
  static constexpr int BM = 32 * WM, BN = 32 * FN * WN;
  static constexpr int NTG = 64 * WM * WN, NT = NTG * KS;      // threads per group / total
  static constexpr int AV = BM * 8 / NTG, WV = BN * 8 / NTG;   // float4 loads per thread
  static constexpr int STAGE = (BM + BN) * CPITCH;
  static_assert(AV >= 1 && WV >= 1 && BM * 8 % NTG == 0 && BN * 8 % NTG == 0, "tile/threads");
  static_assert(KS == 1 || (KS - 1) * WM * WN * FN * 16 * 64 <= KS * 2 * STAGE, "reduction");
};
using TileBig = ConvTile<2, 2, 1, 1>;    // 64 x 64, 256 threads: the 512^2 .. 128^2 layers
using TileSmall = ConvTile<1, 2, 1, 2>;  // 32 x 64, 2 K-groups: the 64^2 layers (fills CUs)
using TileHead = ConvTile<1, 2, 2, 2>;   // 32 x 128, 2 K-groups: convPb's 65 logits

template <class TL>
struct ConvStage {
  float4 a[TL::AV];
  float4 w[TL::WV];
  int ok;   // bit i: A row i is inside the image (else zero padding)
};

// Pixel of tile row m: raster order, or (POOL) pooled pixel m>>2 and its 2x2 input m&3.
template <bool POOL, int BM>
__device__ __forceinline__ void row_pixel(const ConvArgs& a, int mt, int m, int& y, int& x,
                                          bool& valid) {
  if (!POOL) {
    const int p = mt * BM + m;
    valid = p < a.H * a.W;
    const int pc = valid ? p : 0;
    y = pc / a.W;
    x = pc - y * a.W;
  } else {
    const int wp = a.W >> 1, hp = a.H >> 1;
    const int pp = mt * (BM / 4) + (m >> 2);
    valid = pp < hp * wp;
    const int pc = valid ? pp : 0;
    const int py = pc / wp, px = pc - py * wp;
    y = 2 * py + ((m >> 1) & 1);
    x = 2 * px + (m & 1);
  }
}

template <int CIN, int KS, class TL, bool POOL, int EPI>
__global__ __launch_bounds__(TL::NT) void conv_kernel(ConvArgs a) {
  constexpr int BM = TL::BM, BN = TL::BN, NTG = TL::NTG, FN = TL::FN;
  constexpr int CH = CIN / CBK, TAPS = KS * KS, NK = TAPS * CH, HALF = KS / 2;
  constexpr int NKG = NK / TL::KS;   // stages per K-group
  static_assert(NK % TL::KS == 0 && NKG >= 2, "stages must split evenly over the K-groups");
  __shared__ __attribute__((aligned(16))) float lds[TL::KS * 2 * TL::STAGE];
  __shared__ StampLds sl;
  const StampTick tk = stamp_begin(a.stamp, &sl);
  const int b = blockIdx.y;
  const int mt = blockIdx.x / a.ntiles, nt = blockIdx.x - mt * a.ntiles;
  const int n0 = nt * BN;
  const int t = threadIdx.x, grp = t / NTG, tg = t - grp * NTG;
  const int lane = t & 63, wave = tg >> 6;
  const int wm = wave / TL::WN, wn = wave - wm * TL::WN;
  const int kq = (tg & 7) * 4, r0 = tg >> 3;
  constexpr int RSTEP = NTG / 8;   // rows covered by one load instruction
  const float* X = a.x + (int64_t)b * a.x_bs + kq;
  int py[TL::AV], px[TL::AV], roff[TL::AV];
  bool pv[TL::AV];
#pragma unroll
  for (int i = 0; i < TL::AV; ++i) {
    row_pixel<POOL, BM>(a, mt, r0 + RSTEP * i, py[i], px[i], pv[i]);
    roff[i] = (py[i] * a.W + px[i]) * CIN;
  }
  const float* Wt = a.w + (n0 + r0) * (TAPS * CIN) + kq;
  float* glds = lds + grp * 2 * TL::STAGE;
  const int s_base = grp * NKG;

  auto load = [&](int s, ConvStage<TL>& st) __attribute__((always_inline)) {
    const int tap = s / CH, c0 = (s - tap * CH) * CBK;
    const int dy = tap / KS - HALF, dx = tap - (tap / KS) * KS - HALF;
    const int delta = (dy * a.W + dx) * CIN + c0;
    int ok = 0;
#pragma unroll
    for (int i = 0; i < TL::AV; ++i) {
      const bool in = pv[i] & ((unsigned)(py[i] + dy) < (unsigned)a.H) &
                      ((unsigned)(px[i] + dx) < (unsigned)a.W);
      ok |= in ? (1 << i) : 0;
      st.a[i] = *reinterpret_cast<const float4*>(X + roff[i] + (in ? delta : c0));
    }
    st.ok = ok;
#pragma unroll
    for (int i = 0; i < TL::WV; ++i)
      st.w[i] = *reinterpret_cast<const float4*>(Wt + (i * RSTEP) * (TAPS * CIN) + tap * CIN + c0);
  };
  auto store = [&](float* la, const ConvStage<TL>& st) __attribute__((always_inline)) {
    float* lw = la + BM * CPITCH;
#pragma unroll
    for (int i = 0; i < TL::AV; ++i) {
      float4 v = st.a[i];
      const bool in = (st.ok >> i) & 1;
      v.x = in ? v.x : 0.f;
      v.y = in ? v.y : 0.f;
      v.z = in ? v.z : 0.f;
      v.w = in ? v.w : 0.f;
      *reinterpret_cast<float4*>(la + (r0 + RSTEP * i) * CPITCH + kq) = v;
    }
#pragma unroll
    for (int i = 0; i < TL::WV; ++i)
      *reinterpret_cast<float4*>(lw + (r0 + RSTEP * i) * CPITCH + kq) = st.w[i];
  };

  floatx16 acc[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;

  ConvStage<TL> s0, s1;
  load(s_base, s0);
  load(s_base + 1, s1);
  store(glds, s0);
  __syncthreads();
  auto step = [&](int kt, ConvStage<TL>& next, ConvStage<TL>& spare)
      __attribute__((always_inline)) {
    load(s_base + min(kt + 2, NKG - 1), spare);
    const float* la = glds + (kt & 1) * TL::STAGE;
    const float* pa = la + (wm * 32 + (lane & 31)) * CPITCH + (lane >> 5) * 4;
    const float* pw = la + BM * CPITCH + (wn * 32 * FN + (lane & 31)) * CPITCH + (lane >> 5) * 4;
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
    store(glds + ((kt + 1) & 1) * TL::STAGE, next);   // (unused after the last stage)
    __syncthreads();
  };
  for (int kt = 0; kt + 1 < NKG; kt += 2) {
    step(kt, s1, s0);
    step(kt + 1, s0, s1);
  }
  if (NKG & 1) step(NKG - 1, s1, s0);
  if (TL::KS > 1) {   // K-groups 1.. hand their partial sums to group 0 (fixed order)
    constexpr int PER = TL::WM * TL::WN * FN * 16 * 64;
    if (grp > 0) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          lds[(grp - 1) * PER + ((wave * FN + j) * 16 + i) * 64 + lane] = acc[j][i];
    }
    __syncthreads();
    if (grp == 0) {
      for (int g = 1; g < TL::KS; ++g)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            acc[j][i] += lds[(g - 1) * PER + ((wave * FN + j) * 16 + i) * 64 + lane];
    }
    __syncthreads();
  }

  float* Y = a.y + (int64_t)b * a.y_bs;
  if (EPI != CE_SOFTMAX) {
    if (grp == 0) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * 32 * FN + j * 32 + (lane & 31);
        const bool n_ok = n < a.cout;
        const float bias = n_ok ? a.bias[n] : 0.f;
        if (!POOL) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int m = wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
            const int p = mt * BM + m;
            float v = acc[j][i] + bias;
            if (EPI == CE_RELU) v = fmaxf(v, 0.f);
            if (n_ok && p < a.H * a.W) Y[p * a.cout + n] = v;
          }
        } else {
          const int hp = a.H >> 1, wp = a.W >> 1;
#pragma unroll
          for (int g = 0; g < 4; ++g) {   // registers 4g..4g+3 = one 2x2 window
            const int m = wm * 32 + 8 * g + 4 * (lane >> 5);
            const int pp = mt * (BM / 4) + (m >> 2);
            float v = fmaxf(fmaxf(acc[j][4 * g], acc[j][4 * g + 1]),
                            fmaxf(acc[j][4 * g + 2], acc[j][4 * g + 3])) + bias;
            if (EPI == CE_RELU) v = fmaxf(v, 0.f);   // relu(max(.)) == max(relu(.))
            if (n_ok && pp < hp * wp) Y[pp * a.cout + n] = v;
          }
        }
      }
    }
    stamp_end(a.stamp, tk, &sl);
    return;
  }
  // CE_SOFTMAX: BM cells x 65 logits -> softmax over 65, drop the dustbin, pixel shuffle
  // (scores.permute(0,2,3,1).reshape(b,h,w,8,8).permute(0,1,3,2,4).reshape(b,8h,8w), :181-183)
  static_assert(EPI != CE_SOFTMAX || (BN == 128 && NTG == 4 * BM), "softmax head tile");
  float* tile = lds;   // [BM][129]
  if (grp == 0) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = wn * 32 * FN + j * 32 + (lane & 31);
      const float bias = n < a.cout ? a.bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
        tile[m * 129 + n] = acc[j][i] + bias;
      }
    }
  }
  __syncthreads();
  if (grp == 0) {
    const int m = tg >> 2, q = tg & 3;   // 4 threads per cell, 16 channels each
    const float* row = tile + m * 129;
    float mx = -INFINITY;
    for (int c = 0; c < 65; ++c) mx = fmaxf(mx, row[c]);
    float sum = 0.f;
    for (int c = 0; c < 65; ++c) sum += expf(row[c] - mx);
    const int p = mt * BM + m;
    if (p < a.H * a.W) {
      const int cy = p / a.W, cx = p - cy * a.W;
      const int W8 = a.W * 8;
#pragma unroll
      for (int cc = 0; cc < 16; ++cc) {
        const int c = q * 16 + cc;
        Y[(cy * 8 + (c >> 3)) * W8 + cx * 8 + (c & 7)] = expf(row[c] - mx) / sum;
      }
    }
  }
  stamp_end(a.stamp, tk, &sl);
}

// conv1a (1 -> 64, 3x3, pad 1) + ReLU, direct: 16 threads per pixel, 4 output channels each,
// so a wave writes 4 whole NHWC pixels (1 KB) per store; each thread keeps its 36 weights.
__global__ __launch_bounds__(256) void conv1a_kernel(const float* __restrict__ img, int64_t img_bs,
                                                     const float* __restrict__ w,
                                                     const float* __restrict__ bias, int H, int W,
                                                     float* __restrict__ y, int64_t y_bs) {
  const int b = blockIdx.y, g = threadIdx.x & 15;
  float wr[4][9], br[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int k = 0; k < 9; ++k) wr[j][k] = w[(4 * g + j) * 9 + k];
    br[j] = bias[4 * g + j];
  }
  const float* I = img + b * img_bs;
  float* Y = y + b * y_bs;
  constexpr int kPix = 4;   // pixels per thread group, amortising the weight loads
#pragma unroll
  for (int r = 0; r < kPix; ++r) {
    const int p = (blockIdx.x * kPix + r) * 16 + (threadIdx.x >> 4);
    if (p >= H * W) return;
    const int py = p / W, px = p - py * W;
    float v[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int yy = py + k / 3 - 1, xx = px + k % 3 - 1;
      v[k] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? I[yy * W + xx] : 0.f;
    }
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 9; ++k) s += v[k] * wr[j][k];
      o[j] = fmaxf(s + br[j], 0.f);
    }
    *reinterpret_cast<float4*>(Y + (int64_t)p * 64 + 4 * g) = make_float4(o[0], o[1], o[2], o[3]);
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

// simple_nms fused: one 32x32 output tile per workgroup evaluates all five max-pool passes
// in LDS over windows that shrink by R per pass, from scores loaded with a 5R halo.  Arrays
// live in tile coordinates [E][E]; positions outside the image are -inf to every pool, as
// max_pool2d's padding is.  Writes max_mask (0/1) for the tile.
template <int R>
__global__ __launch_bounds__(256) void nms_fused_kernel(NmsArgs a) {
  constexpr int E = NT + 10 * R, K = 2 * R + 1;
  __shared__ float S[E * E], M[E * E], SP[E * E], SS[E * E], TMP[E * E];
  const int b = blockIdx.z, gy0 = blockIdx.y * NT - 5 * R, gx0 = blockIdx.x * NT - 5 * R;
  const int64_t o = b * a.bs;
  auto inside = [&](int y, int x) {
    return (unsigned)(gy0 + y) < (unsigned)a.H && (unsigned)(gx0 + x) < (unsigned)a.W;
  };
  for (int e = threadIdx.x; e < E * E; e += 256) {
    const int y = e / E, x = e - y * E;
    S[e] = inside(y, x) ? a.s[o + (int64_t)(gy0 + y) * a.W + gx0 + x] : -INFINITY;
  }
  __syncthreads();
  // max_pool(IN) over the window [lo, E - lo)^2 into TMP (rows then columns, via TMP rows)
  auto pool = [&](const float* IN, int lo, auto&& finish) {
    const int hi = E - lo, n = hi - lo;
    float* rowm = TMP;   // rows [lo - R, hi + R) x cols [lo, hi)
    for (int e = threadIdx.x; e < (n + 2 * R) * n; e += 256) {
      const int y = lo - R + e / n, x = lo + e % n;
      float m = -INFINITY;
#pragma unroll
      for (int d = 0; d < K; ++d) m = fmaxf(m, IN[y * E + x - R + d]);
      rowm[y * E + x] = m;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < n * n; e += 256) {
      const int y = lo + e / n, x = lo + e % n;
      float m = -INFINITY;
#pragma unroll
      for (int d = 0; d < K; ++d) m = fmaxf(m, rowm[(y - R + d) * E + x]);
      finish(y * E + x, m, inside(y, x));
    }
    __syncthreads();
  };
  // mask = scores == max_pool(scores)
  pool(S, R, [&](int i, float m, bool in) { M[i] = in ? (S[i] == m ? 1.f : 0.f) : -INFINITY; });
  for (int it = 0; it < 2; ++it) {
    // supp = max_pool(mask) > 0; ss = supp ? 0 : scores
    pool(M, (2 + 2 * it) * R, [&](int i, float m, bool in) {
      SP[i] = m > 0.f ? 1.f : 0.f;
      SS[i] = in ? (m > 0.f ? 0.f : S[i]) : -INFINITY;
    });
    // mask |= (ss == max_pool(ss)) & ~supp
    pool(SS, (3 + 2 * it) * R, [&](int i, float m, bool in) {
      if (in && SS[i] == m && SP[i] == 0.f) M[i] = 1.f;
    });
  }
  for (int e = threadIdx.x; e < NT * NT; e += 256) {
    const int y = 5 * R + e / NT, x = 5 * R + e % NT;
    if (inside(y, x)) a.mask[o + (int64_t)(gy0 + y) * a.W + gx0 + x] = M[y * E + x] > 0.f ? 1.f : 0.f;
  }
}

// ---- keypoint selection: threshold + borders, raster-order compaction, top-k ----
// Candidates (score > threshold after NMS, outside the border) are compacted in raster order
// (torch.nonzero's order).  When more than max_keypoints survive, torch.topk(k) keeps the k
// best in descending order: a 16384-bin histogram of the scores' order-preserving keys (binned
// over the sample's own key range, so bins hold a handful of candidates) finds the cutoff
// bin; every candidate at or above it is scattered into bin-descending order, and
// its final position is its bin's start plus the number of bin mates with a larger key
// (score, then lower raster index first).  Equal scores therefore keep raster order.
constexpr int kSelChunk = 4096;
constexpr int kCutBins = 16384;      // histogram bins over [min key, max key]
constexpr int kCutBits = 14;
constexpr int kMaxBinRank = 2048;    // larger tie bins take the single-workgroup sort path
constexpr int kMaxSortKeys = 16384;  // LDS sort capacity of that path (128 KB of keys)
constexpr int kUnroll = 8;           // candidate loads in flight per thread

enum SelMode { SEL_DONE = 0, SEL_RANK = 1, SEL_SORT = 2 };

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
  int* mode;            // [B] SelMode
  int* n_cut;           // [B] candidates at or above the cutoff bin
  float* cand_score;    // [B][H*W] raster-order candidates
  int* cand_idx;
  unsigned long long* cut_key;   // [B][H*W] cutoff set, bin-descending
  int2* cut_range;      // [B][H*W] the element's bin range in cut_key
  float* kpts;          // [B][max_kp][2] (x, y)
  float* kscores;       // [B][max_kp]
  int* counts;          // [B]
};

// Order-preserving uint key of a float (any sign), and its inverse.
__device__ __forceinline__ unsigned ord_key(float v) {
  const unsigned u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord_val(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}
// Sort key: score descending, then raster index ascending.
__device__ __forceinline__ unsigned long long sort_key(unsigned ordv, int idx) {
  return ((unsigned long long)ordv << 32) | (0xFFFFFFFFu - (unsigned)idx);
}
__device__ __forceinline__ void emit(const SelArgs& a, int b, int slot,
                                     unsigned long long key) {
  const int p = (int)(0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull));
  float* kp = a.kpts + ((int64_t)b * a.max_kp + slot) * 2;
  kp[0] = (float)(p % a.W);   // flip (y, x) -> (x, y)
  kp[1] = (float)(p / a.W);
  a.kscores[(int64_t)b * a.max_kp + slot] = ord_val((unsigned)(key >> 32));
}

__device__ __forceinline__ bool is_cand(const SelArgs& a, int64_t o, int p, float& v) {
  const int y = p / a.W, x = p - y * a.W;
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

// Exclusive scan of the chunk counts (one workgroup per sample).
__global__ __launch_bounds__(256) void sel_scan_kernel(SelArgs a) {
  __shared__ int sc[256];
  const int b = blockIdx.x, t = threadIdx.x;
  const int per = (a.chunks + 255) / 256, c0 = t * per, c1 = min(c0 + per, a.chunks);
  const int* cnt = a.chunk_count + (int64_t)b * a.chunks;
  int sum = 0;
  for (int c = c0; c < c1; ++c) sum += cnt[c];
  sc[t] = sum;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {   // inclusive scan
    const int v = t >= off ? sc[t - off] : 0;
    __syncthreads();
    sc[t] += v;
    __syncthreads();
  }
  int run = sc[t] - sum;
  for (int c = c0; c < c1; ++c) {
    a.chunk_off[(int64_t)b * a.chunks + c] = run;
    run += cnt[c];
  }
  if (t == 255) a.total[b] = sc[255];
}

// Scatter candidates in raster order: each wave compacts 64 pixels with a ballot.
__global__ __launch_bounds__(256) void sel_scatter_kernel(SelArgs a) {
  __shared__ int wbase[4][kSelChunk / 256];
  const int b = blockIdx.y, ch = blockIdx.x;
  const int64_t o = b * a.bs;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int p0 = ch * kSelChunk;
  constexpr int R = kSelChunk / 256;   // rounds of 256 pixels
  bool c[R];
  float v[R];
#pragma unroll
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
#pragma unroll
  for (int rr = 0; rr < R; ++rr) {
    const unsigned long long bal = __ballot(c[rr]);
    if (c[rr]) {
      const int pos = wbase[wave][rr] + __popcll(bal & ((1ull << lane) - 1ull));
      cs[pos] = v[rr];
      ci[pos] = p0 + rr * 256 + wave * 64 + lane;
    }
  }
}

// One workgroup per sample: raster output when total <= k; otherwise the cutoff histogram and
// the bin-grouped cutoff set for sel_rank (or SEL_SORT when a tie bin is too large).
__global__ __launch_bounds__(1024) void sel_cut_kernel(SelArgs a) {
  __shared__ int cnt[kCutBins];     // per-bin count, then a countdown cursor
  __shared__ int start[kCutBins];   // candidates in higher bins
  __shared__ int tsum[1024];
  __shared__ int cut_bin, max_bin;
  __shared__ unsigned kmin, kmax;
  const int b = blockIdx.x, t = threadIdx.x;
  const int total = a.total[b], k = a.max_kp;
  const int64_t o = b * a.bs;
  const float* cs = a.cand_score + o;
  const int* ci = a.cand_idx + o;
  if (total <= k) {
    for (int i = t; i < k; i += 1024) {
      const bool on = i < total;
      const int p = on ? ci[i] : 0;
      float* kp = a.kpts + ((int64_t)b * k + i) * 2;
      kp[0] = on ? (float)(p % a.W) : 0.f;   // flip (y, x) -> (x, y)
      kp[1] = on ? (float)(p / a.W) : 0.f;
      a.kscores[(int64_t)b * k + i] = on ? cs[i] : 0.f;
    }
    if (t == 0) {
      a.counts[b] = total;
      a.mode[b] = SEL_DONE;
      a.n_cut[b] = 0;
    }
    return;
  }
  for (int i = t; i < kCutBins; i += 1024) cnt[i] = 0;
  if (t == 0) {
    max_bin = 0;
    kmin = 0xFFFFFFFFu;
    kmax = 0u;
  }
  __syncthreads();
  {   // key range -> bin = (key - kmin) >> shift, monotone, at most kCutBins bins
    unsigned lo = 0xFFFFFFFFu, hi = 0u;
    for (int base = t; base < total; base += 1024 * kUnroll) {   // independent loads in flight
      float v[kUnroll];
#pragma unroll
      for (int j = 0; j < kUnroll; ++j) v[j] = base + 1024 * j < total ? cs[base + 1024 * j] : cs[t];
#pragma unroll
      for (int j = 0; j < kUnroll; ++j) {
        const unsigned u = ord_key(v[j]);
        lo = min(lo, u);
        hi = max(hi, u);
      }
    }
    atomicMin(&kmin, lo);
    atomicMax(&kmax, hi);
  }
  __syncthreads();
  const unsigned k0 = kmin, span = kmax - kmin;
  const int shift = span == 0u ? 0 : max(0, 32 - __clz((int)span) - kCutBits);
  auto bin_of = [&](unsigned u) { return (int)((u - k0) >> shift); };
  for (int base = t; base < total; base += 1024 * kUnroll) {
    float v[kUnroll];
#pragma unroll
    for (int j = 0; j < kUnroll; ++j) v[j] = base + 1024 * j < total ? cs[base + 1024 * j] : 0.f;
#pragma unroll
    for (int j = 0; j < kUnroll; ++j)
      if (base + 1024 * j < total) atomicAdd(&cnt[bin_of(ord_key(v[j]))], 1);
  }
  __syncthreads();
  constexpr int PER = kCutBins / 1024;   // thread t owns bins [PER t, PER t + PER)
  int own = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) own += cnt[PER * t + j];
  tsum[t] = own;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {   // inclusive suffix scan over threads
    const int v = t + off < 1024 ? tsum[t + off] : 0;
    __syncthreads();
    tsum[t] += v;
    __syncthreads();
  }
  {
    int run = tsum[t] - own;
    for (int j = PER - 1; j >= 0; --j) {
      const int bin = PER * t + j, c = cnt[bin];
      start[bin] = run;
      if (run < k && run + c >= k) cut_bin = bin;
      run += c;
    }
  }
  __syncthreads();
  const int cb = cut_bin;
  const int n = start[cb] + cnt[cb];   // read before the scatter counts cnt down
  {
    int m = 0;
    for (int j = 0; j < PER; ++j) {
      const int bin = PER * t + j;
      if (bin >= cb) m = max(m, cnt[bin]);
    }
    atomicMax(&max_bin, m);
  }
  __syncthreads();
  if (t == 0) {
    a.counts[b] = k;
    a.n_cut[b] = n;
    a.mode[b] = max_bin > kMaxBinRank ? SEL_SORT : SEL_RANK;
  }
  if (max_bin > kMaxBinRank) return;
  unsigned long long* key = a.cut_key + o;
  int2* range = a.cut_range + o;
  for (int base = t; base < total; base += 1024 * kUnroll) {
    float v[kUnroll];
    int idx[kUnroll];
#pragma unroll
    for (int j = 0; j < kUnroll; ++j) {
      const bool on = base + 1024 * j < total;
      v[j] = on ? cs[base + 1024 * j] : 0.f;
      idx[j] = on ? ci[base + 1024 * j] : 0;
    }
#pragma unroll
    for (int j = 0; j < kUnroll; ++j) {
      const unsigned u = ord_key(v[j]);
      const int bin = bin_of(u);
      if (base + 1024 * j >= total || bin < cb) continue;
      const int s0 = start[bin], s1 = bin > 0 ? start[bin - 1] : total;   // bin's range
      const int pos = s0 + atomicSub(&cnt[bin], 1) - 1;
      key[pos] = sort_key(u, idx[j]);
      range[pos] = make_int2(s0, s1);
    }
  }
}

// Final position of each cutoff-set element: its bin's start plus the bin mates with a
// larger key.  Positions >= k are dropped (they can only come from the cutoff bin).
__global__ __launch_bounds__(256) void sel_rank_kernel(SelArgs a) {
  const int b = blockIdx.y, e = blockIdx.x * 256 + threadIdx.x;
  if (a.mode[b] != SEL_RANK || e >= a.n_cut[b]) return;
  const int64_t o = b * a.bs;
  const unsigned long long* key = a.cut_key + o;
  const unsigned long long me = key[e];
  const int2 r = a.cut_range[o + e];
  int rank = r.x;
  for (int f = r.x; f < r.y; ++f) rank += key[f] > me ? 1 : 0;
  if (rank < a.max_kp) emit(a, b, rank, me);
}

// Bitonic sort of keys[0, P) descending (P a power of two), whole workgroup.
__device__ void bitonic_desc(unsigned long long* keys, int P) {
  for (int size = 2; size <= P; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
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
}

// SEL_SORT (a tie bin larger than kMaxBinRank): exact radix select of the k-th largest key
// over the candidates, the first winners among equal keys in raster order, and a bitonic
// sort of the k winners in LDS.  One workgroup per sample.
__global__ __launch_bounds__(1024) void sel_sort_kernel(SelArgs a) {
  extern __shared__ unsigned long long keys[];   // [kMaxSortKeys]
  __shared__ int tsum[1024];
  __shared__ int hist[256];
  __shared__ unsigned prefix_s, mask_s;
  __shared__ int need_s, ngt_s, neq_s;
  const int b = blockIdx.x, t = threadIdx.x;
  if (a.mode[b] != SEL_SORT) return;
  const int total = a.total[b], k = a.max_kp;
  const int64_t o = b * a.bs;
  const float* cs = a.cand_score + o;
  const int* ci = a.cand_idx + o;
  if (t == 0) {
    prefix_s = 0u;
    mask_s = 0u;
    need_s = k;
    ngt_s = 0;
    neq_s = 0;
  }
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = t; i < 256; i += 1024) hist[i] = 0;
    __syncthreads();
    const unsigned pre = prefix_s, msk = mask_s;
    for (int i = t; i < total; i += 1024) {
      const unsigned u = ord_key(cs[i]);
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
      need_s = need;
    }
    __syncthreads();
  }
  const unsigned thr_u = prefix_s;
  int P = 1;
  while (P < k) P <<= 1;
  for (int i = t; i < P; i += 1024) keys[i] = 0ull;
  __syncthreads();
  const int n_eq = need_s, n_gt = k - n_eq;
  for (int base = 0; base < total; base += 1024) {   // equal keys: first n_eq in raster order
    const int i = base + t;
    const unsigned u = i < total ? ord_key(cs[i]) : 0u;
    const bool gt = i < total && u > thr_u, eq = i < total && u == thr_u;
    tsum[t] = eq ? 1 : 0;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const int v = t >= off ? tsum[t - off] : 0;
      __syncthreads();
      tsum[t] += v;
      __syncthreads();
    }
    const int eq_before = neq_s;
    if (gt) keys[atomicAdd(&ngt_s, 1)] = sort_key(u, ci[i]);
    if (eq) {
      const int r = eq_before + tsum[t] - 1;
      if (r < n_eq) keys[n_gt + r] = sort_key(u, ci[i]);
    }
    __syncthreads();
    if (t == 1023) neq_s = eq_before + tsum[1023];
    __syncthreads();
  }
  bitonic_desc(keys, P);
  for (int i = t; i < k; i += 1024) emit(a, b, i, keys[i]);
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
// 16 keypoints per workgroup are written through LDS as [256][k] columns.
__global__ __launch_bounds__(256) void sample_nhwc_kernel(const float* __restrict__ kpts,
                                                          const int* __restrict__ counts,
                                                          const float* __restrict__ dense,
                                                          int max_kp, int h, int w, int s,
                                                          int align_corners,
                                                          float* __restrict__ out) {
#pragma clang fp contract(off)
  constexpr int KPB = 16;   // keypoints per workgroup
  __shared__ float tile[256][KPB + 1];
  const int b = blockIdx.y, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int k0 = blockIdx.x * KPB;
  const int cnt = counts[b];
  const float* D = dense + (int64_t)b * h * w * 256;
  for (int kk = wave; kk < KPB; kk += 4) {
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
  for (int e = threadIdx.x; e < 256 * KPB; e += 256) {
    const int c = e / KPB, kk = e % KPB;
    if (k0 + kk < max_kp) O[(int64_t)c * max_kp + k0 + kk] = tile[c][kk];
  }
}

// ---- plan ----
struct DetPlan {   // NMS + selection scratch
  float *mask, *supp, *ss;        // [H][W]
  float* cand_score;
  int *cand_idx, *chunk_count, *chunk_off, *total, *mode, *n_cut;
  unsigned long long* cut_key;
  int2* cut_range;
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
  p.mode = c.take<int>(B);
  p.n_cut = c.take<int>(B);
  p.cut_key = c.take<unsigned long long>(B * hw);
  p.cut_range = c.take<int2>(B * hw);
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

template <int CIN, int KS, class TL, bool POOL, int EPI>
int conv_launch(const float* x, int B, int H, int W, const float* packed, int layer, float* y,
                hipStream_t st) {
  const SpLayer& L = kSp[layer];
  if (L.cin != CIN || L.k != KS || L.cout_pad % TL::BN != 0) {
    set_error("superpoint: layer %s does not fit its conv instantiation", kSpNames[layer]);
    return ONEPOSE_ERR_INVALID;
  }
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
  a.mtiles = ceil_div(pix, POOL ? TL::BM / 4 : TL::BM);
  a.ntiles = L.cout_pad / TL::BN;
  a.stamp = prof_stamp_slot(K_SP_CONV);
  a.y_bs = EPI == CE_SOFTMAX ? (int64_t)H * W * 64 : (int64_t)pix * L.cout;
  OP_LAUNCH(K_SP_CONV, st, (conv_kernel<CIN, KS, TL, POOL, EPI>), dim3(a.mtiles * a.ntiles, B),
            dim3(TL::NT), 0, st, a);
  return ONEPOSE_OK;
}

// The 512^2..128^2 layers on TileBig (the tile sweep of docs/EXPERIMENTS.md §3b chose it).
template <int CIN, bool POOL>
int big_conv(const float* x, int B, int H, int W, const float* packed, int layer, float* y,
             hipStream_t st) {
  return conv_launch<CIN, 3, TileBig, POOL, CE_RELU>(x, B, H, W, packed, layer, y, st);
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
  switch (nms_radius) {   // fused single pass for the radii OnePose uses; 5 launches beyond
    case 0: OP_LAUNCH(K_SP_NMS, st, nms_fused_kernel<0>, ng, dim3(256), 0, st, na); break;
    case 1: OP_LAUNCH(K_SP_NMS, st, nms_fused_kernel<1>, ng, dim3(256), 0, st, na); break;
    case 2: OP_LAUNCH(K_SP_NMS, st, nms_fused_kernel<2>, ng, dim3(256), 0, st, na); break;
    case 3: OP_LAUNCH(K_SP_NMS, st, nms_fused_kernel<3>, ng, dim3(256), 0, st, na); break;
    case 4: OP_LAUNCH(K_SP_NMS, st, nms_fused_kernel<4>, ng, dim3(256), 0, st, na); break;
    default:
      OP_LAUNCH(K_SP_NMS, st, nms_kernel<NMS_INIT>, ng, dim3(256), 0, st, na);
      for (int it = 0; it < 2; ++it) {
        OP_LAUNCH(K_SP_NMS, st, nms_kernel<NMS_SUPP>, ng, dim3(256), 0, st, na);
        OP_LAUNCH(K_SP_NMS, st, nms_kernel<NMS_GROW>, ng, dim3(256), 0, st, na);
      }
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
  sa.mode = p.mode;
  sa.n_cut = p.n_cut;
  sa.cut_key = p.cut_key;
  sa.cut_range = p.cut_range;
  sa.cand_score = p.cand_score;
  sa.cand_idx = p.cand_idx;
  sa.kpts = keypoints;
  sa.kscores = scores;
  sa.counts = counts;
  OP_LAUNCH(K_SP_SELECT, st, sel_count_kernel, dim3(sa.chunks, B), dim3(256), 0, st, sa);
  OP_LAUNCH(K_SP_SELECT, st, sel_scan_kernel, dim3(B), dim3(256), 0, st, sa);
  OP_LAUNCH(K_SP_SELECT, st, sel_scatter_kernel, dim3(sa.chunks, B), dim3(256), 0, st, sa);
  OP_LAUNCH(K_SP_SELECT, st, sel_cut_kernel, dim3(B), dim3(1024), 0, st, sa);
  if (max_kp <= kMaxSortKeypoints) {   // otherwise max_kp >= h*w: never more candidates
    // the cutoff set holds at most k - 1 + kMaxBinRank elements in SEL_RANK mode
    OP_LAUNCH(K_SP_SELECT, st, sel_rank_kernel, dim3(ceil_div(max_kp + kMaxBinRank, 256), B),
              dim3(256), 0, st, sa);
    static bool attr_set = false;
    if (!attr_set) {
      OP_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(sel_sort_kernel),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, kMaxSortKeys * 8));
      attr_set = true;
    }
    OP_LAUNCH(K_SP_SELECT, st, sel_sort_kernel, dim3(B), dim3(1024), (size_t)kMaxSortKeys * 8, st,
              sa);
  }
  OP_LAUNCH(K_SP_DESC, st, sample_nhwc_kernel, dim3(ceil_div(max_kp, 16), B), dim3(256), 0, st,
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
  OP_LAUNCH(K_SP_CONV, st, conv1a_kernel, dim3(ceil_div(h * w, 64), B), dim3(256), 0, st, image,
            (int64_t)h * w, P + layer_offset(0), P + layer_offset(0) + 64 * 9, h, w, p.f0,
            (int64_t)h * w * 64);
  if ((rc = big_conv<64, true>(p.f0, B, h, w, P, 1, p.f1, st))) return rc;
  if ((rc = big_conv<64, false>(p.f1, B, h / 2, w / 2, P, 2, p.f0, st)))
    return rc;
  if ((rc = big_conv<64, true>(p.f0, B, h / 2, w / 2, P, 3, p.f1, st)))
    return rc;
  if ((rc = big_conv<64, false>(p.f1, B, h / 4, w / 4, P, 4, p.f0, st)))
    return rc;
  if ((rc = big_conv<128, true>(p.f0, B, h / 4, w / 4, P, 5, p.f1, st)))
    return rc;
  if ((rc = conv_launch<128, 3, TileSmall, false, CE_RELU>(p.f1, B, h / 8, w / 8, P, 6, p.f0, st)))
    return rc;
  if ((rc = conv_launch<128, 3, TileSmall, false, CE_RELU>(p.f0, B, h / 8, w / 8, P, 7, p.x4, st)))
    return rc;
  // score head: convPa + ReLU, convPb -> softmax(65)[:64] -> pixel shuffle -> [H][W]
  if ((rc = conv_launch<128, 3, TileSmall, false, CE_RELU>(p.x4, B, h / 8, w / 8, P, 8, p.head,
                                                           st)))
    return rc;
  if ((rc = conv_launch<256, 1, TileHead, false, CE_SOFTMAX>(p.head, B, h / 8, w / 8, P, 9,
                                                             p.score, st)))
    return rc;
  // descriptor head: convDa + ReLU, convDb, normalise (the score head's hidden map is dead)
  if ((rc = conv_launch<128, 3, TileSmall, false, CE_RELU>(p.x4, B, h / 8, w / 8, P, 10, p.head,
                                                           st)))
    return rc;
  if ((rc = conv_launch<256, 1, TileSmall, false, CE_BIAS>(p.head, B, h / 8, w / 8, P, 11,
                                                           p.dense, st)))
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
