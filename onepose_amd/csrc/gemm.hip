// fp32 MFMA grouped token-GEMM (see gemm.h).
//
// Tile: 64 tokens x 64 outputs x 32-deep K step, 256 threads = 4 waves in a 2x2 grid, each
// wave one 32x32 accumulator of v_mfma_f32_32x32x2_f32.  Operands are staged through
// double-buffered LDS images [row][k] with a 36-float row pitch: a ds_read_b128 lane group
// (16 lanes, 16 distinct rows, same k) then covers 16 distinct 16-byte slots of the
// 64-bank row -- conflict free (9*i mod 16 is a permutation).  Each b128 read feeds four
// MFMAs: within one group of 8 k-values, lane half h carries k = 8*kk + 4*h + j into MFMA
// j, identically for A and W, so the k-sum is unchanged (a pure re-ordering of the sum).
// One barrier per K step; the next step's global loads are in flight during the MFMAs.
#include "gemm.h"

namespace onepose {

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int BM = kGemmBM, BN = kGemmBN, BK = kGemmBK;
constexpr int PITCH = BK + 4;   // 36 floats

struct Stage {
  float4 a[2];
  float4 w[2];
};

// Per-launch problem fields, selected field by field from the kernel arguments (a
// dynamically indexed kernel-argument struct would be copied to scratch).
struct Ctx {
  const float *a0, *a1, *w, *mean, *rstd;
  int lda0, lda1, ksplit, ldw, M, N, K;
};

template <int PRO>
__device__ __forceinline__ void load_stage(const Ctx& c, int m0, int n0, int k0, Stage& s) {
  const int t = threadIdx.x;
  const int kq = (t & 7) * 4;
  const bool first = k0 < c.ksplit;
  const float* A = first ? c.a0 : c.a1;
  const int lda = first ? c.lda0 : c.lda1;
  const int kk = first ? (k0 + kq) : (k0 - c.ksplit + kq);
  float4 mean, rstd;
  if (PRO == PRO_NORM_RELU) {
    mean = *reinterpret_cast<const float4*>(c.mean + k0 + kq);
    rstd = *reinterpret_cast<const float4*>(c.rstd + k0 + kq);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (t >> 3) + 32 * i;
    const int m = m0 + row;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (m < c.M) {
      v = *reinterpret_cast<const float4*>(A + (int64_t)m * lda + kk);
      if (PRO == PRO_NORM_RELU) {
        v.x = fmaxf((v.x - mean.x) * rstd.x, 0.f);
        v.y = fmaxf((v.y - mean.y) * rstd.y, 0.f);
        v.z = fmaxf((v.z - mean.z) * rstd.z, 0.f);
        v.w = fmaxf((v.w - mean.w) * rstd.w, 0.f);
      }
    }
    s.a[i] = v;
    const int o = n0 + row;
    float4 wv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (o < c.N) wv = *reinterpret_cast<const float4*>(c.w + (int64_t)o * c.ldw + k0 + kq);
    s.w[i] = wv;
  }
}

__device__ __forceinline__ void store_stage(float* lds_a, float* lds_w, const Stage& s) {
  const int t = threadIdx.x;
  const int kq = (t & 7) * 4;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (t >> 3) + 32 * i;
    *reinterpret_cast<float4*>(lds_a + row * PITCH + kq) = s.a[i];
    *reinterpret_cast<float4*>(lds_w + row * PITCH + kq) = s.w[i];
  }
}

template <int EPI, int PRO>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs args) {
  __shared__ __attribute__((aligned(16))) float lds[2 * 2 * BM * PITCH];

  int bid = blockIdx.x;
  const bool second = bid >= args.p[0].tiles;
#define F(x) (second ? args.p[1].x : args.p[0].x)
  if (second) bid -= args.p[0].tiles;
  const int mtiles = F(mtiles), ntiles = F(ntiles);
  const int per_sample = mtiles * ntiles;
  const int b = bid / per_sample;
  const int r = bid - b * per_sample;
  const int mt = r / ntiles;
  const int nt = r - mt * ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  Ctx c;
  c.a0 = F(A0) + b * F(a0_bs);
  c.a1 = F(A1) + b * F(a1_bs);
  c.w = F(W) + b * F(w_bs);
  c.mean = F(pro_mean) + b * F(pro_bs);
  c.rstd = F(pro_rstd) + b * F(pro_bs);
  c.lda0 = F(lda0);
  c.lda1 = F(lda1);
  c.ksplit = F(ksplit);
  c.ldw = F(ldw);
  c.M = F(M);
  c.N = F(N);
  c.K = F(K);

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  floatx16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;

  const int nk = c.K / BK;
  Stage st;
  load_stage<PRO>(c, m0, n0, 0, st);
  store_stage(lds, lds + BM * PITCH, st);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    float* la = lds + (kt & 1) * 2 * BM * PITCH;
    float* lw = la + BM * PITCH;
    if (kt + 1 < nk) load_stage<PRO>(c, m0, n0, (kt + 1) * BK, st);
    const float* pa = la + (wm * 32 + (lane & 31)) * PITCH + (lane >> 5) * 4;
    const float* pw = lw + (wn * 32 + (lane & 31)) * PITCH + (lane >> 5) * 4;
#pragma unroll
    for (int kk = 0; kk < BK / 8; ++kk) {
      const float4 a = *reinterpret_cast<const float4*>(pa + kk * 8);
      const float4 w = *reinterpret_cast<const float4*>(pw + kk * 8);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, w.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, w.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, w.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, w.w, acc, 0, 0, 0);
    }
    if (kt + 1 < nk) {
      float* na = lds + ((kt + 1) & 1) * 2 * BM * PITCH;
      store_stage(na, na + BM * PITCH, st);
    }
    __syncthreads();
  }

  // ---- epilogue ----
  const int col = wn * 32 + (lane & 31);
  const int gn = n0 + col;
  const int M = c.M, N = c.N;
  const bool col_ok = gn < N;
  const float* biasp = F(bias);
  float bias = 0.f;
  if (EPI != EPI_SCORE && biasp != nullptr && col_ok) bias = biasp[gn];
  float* Y = F(Y) + b * F(y_bs);
  const int ldy = F(ldy);
  const float* R = (EPI == EPI_RESID) ? F(R) + b * F(r_bs) : nullptr;
  const int ldr = F(ldr);
  const float scale = F(scale), vdiv = F(vdiv);
  const int phi_cols = F(phi_cols);
  float* tile = lds;   // [64][65] staging for the reducing epilogues
  constexpr int TP = BN + 1;

#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
    const int gm = m0 + row;
    float y;
    if (EPI == EPI_SCORE) {
      y = acc[i] / scale;
    } else {
      y = acc[i] + bias;
      if (EPI == EPI_QKV) y = (gn < phi_cols) ? (elu1(y) + 1.0f) : (y / vdiv);
    }
    if (gm < M && col_ok) {
      if (EPI == EPI_RESID) y = R[(int64_t)gm * ldr + gn] + y;
      Y[(int64_t)gm * ldy + gn] = y;
    }
    if (EPI == EPI_STATS || EPI == EPI_SCORE) tile[row * TP + col] = y;
  }

  if (EPI == EPI_STATS) {
    __syncthreads();
    const int t = threadIdx.x;
    const int rows = min(BM, M - m0);
    if (t < BN && n0 + t < N) {
      float s = 0.f;
      for (int rr = 0; rr < rows; ++rr) s += tile[rr * TP + t];
      const float mean = s / (float)rows;
      float m2 = 0.f;
      for (int rr = 0; rr < rows; ++rr) {
        const float d = tile[rr * TP + t] - mean;
        m2 += d * d;
      }
      float* st_out = F(stats) + ((int64_t)b * mtiles + mt) * 2 * N;
      st_out[n0 + t] = mean;
      st_out[N + n0 + t] = m2;
    }
  }
  if (EPI == EPI_SCORE) {
    __syncthreads();
    const int t = threadIdx.x;
    const int rows = min(BM, M - m0);
    const int cols = min(BN, N - n0);
    if (t < BM) {
      if (t < rows) {   // row partial over this tile's columns
        float mx = -INFINITY;
        for (int cc = 0; cc < cols; ++cc) mx = fmaxf(mx, tile[t * TP + cc]);
        float s = 0.f;
        for (int cc = 0; cc < cols; ++cc) s += expf(tile[t * TP + cc] - mx);
        float* o = F(rowstat) + (((int64_t)b * M + m0 + t) * ntiles + nt) * 2;
        o[0] = mx;
        o[1] = s;
      }
    } else if (t < BM + BN) {
      const int cc = t - BM;
      if (cc < cols) {   // column partial over this tile's rows
        float mx = -INFINITY;
        for (int rr = 0; rr < rows; ++rr) mx = fmaxf(mx, tile[rr * TP + cc]);
        float s = 0.f;
        for (int rr = 0; rr < rows; ++rr) s += expf(tile[rr * TP + cc] - mx);
        float* o = F(colstat) + (((int64_t)b * N + n0 + cc) * mtiles + mt) * 2;
        o[0] = mx;
        o[1] = s;
      }
    }
  }
#undef F
}

template <int EPI, int PRO>
void launch_one(GemmArgs& args, int grid, hipStream_t stream) {
  hipLaunchKernelGGL((gemm_f32_kernel<EPI, PRO>), dim3(grid), dim3(256), 0, stream, args);
}

}  // namespace

int gemm_launch(int epi, int pro, GemmArgs& args, hipStream_t stream, int kind) {
  int grid = 0;
  for (int i = 0; i < 2; ++i) {
    GemmProb& P = args.p[i];
    if (i >= args.nprob) {
      P.tiles = 0;
      continue;
    }
    OP_REQUIRE(P.K % kGemmBK == 0, "gemm: K=%d not a multiple of %d", P.K, kGemmBK);
    OP_REQUIRE(P.ksplit % kGemmBK == 0, "gemm: ksplit=%d", P.ksplit);
    OP_REQUIRE(P.lda0 % 4 == 0 && P.ldw % 4 == 0, "gemm: unaligned leading dimension");
    P.mtiles = ceil_div(P.M, kGemmBM);
    P.ntiles = ceil_div(P.N, kGemmBN);
    P.tiles = P.mtiles * P.ntiles * P.batch;
    grid += P.tiles;
  }
  if (grid == 0) return ONEPOSE_OK;
#define CASE(E, PR)                               \
  if (epi == E && pro == PR) {                    \
    prof_pre(kind, stream);                       \
    launch_one<E, PR>(args, grid, stream);        \
    prof_post(kind, stream);                      \
    OP_LAUNCHED();                                \
    return ONEPOSE_OK;                            \
  }
  CASE(EPI_BIAS, PRO_PLAIN)
  CASE(EPI_QKV, PRO_PLAIN)
  CASE(EPI_STATS, PRO_PLAIN)
  CASE(EPI_RESID, PRO_NORM_RELU)
  CASE(EPI_SCORE, PRO_PLAIN)
#undef CASE
  set_error("gemm: unsupported epilogue/prologue %d/%d", epi, pro);
  return ONEPOSE_ERR_INVALID;
}

}  // namespace onepose
